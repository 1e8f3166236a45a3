"""Golden SPARC cases (mirrors tests/golden/make_golden_sparc.py SPARC_CASES)."""
SPARC_CASES = [
    ("reg15", {'P': 15.0, 'R': 1.5, 'L': 32, 'M': 512}, {'t_max': 25}, 1.0, 5),
    ("reg13", {'P': 15.0, 'R': 1.3, 'L': 32, 'M': 512}, {'t_max': 25}, 1.0, 5),
    ("reg12m2", {'P': 15.0, 'R': 1.2, 'L': 64, 'M': 64}, {'t_max': 25, 'phi_est_method': 2}, 1.0, 3),
    ("pa", {'P': 15.0, 'R': 1.4, 'L': 64, 'M': 64, 'power_allocated': True, 'B': 4,
            'R_PA_ratio': 1.0}, {'t_max': 30}, 1.0, 3),
    ("sc", {'P': 15.0, 'R': 1.2, 'L': 32, 'M': 64, 'spatially_coupled': True, 'omega': 2,
            'Lambda': 4}, {'t_max': 40}, 1.0, 3),
    ("scpa", {'P': 15.0, 'R': 1.2, 'L': 64, 'M': 32, 'spatially_coupled': True, 'omega': 2,
              'Lambda': 4, 'power_allocated': True, 'B': 2, 'R_PA_ratio': 0.8}, {'t_max': 40},
     1.0, 2),
]


def all_seeds():
    for name, cp, dp, var, ns in SPARC_CASES:
        for si in range(ns):
            yield name, dict(cp), dict(dp), var, si


def design(g, name, si, cp, var):
    """(W, L, M, n, order0, order1) of a golden case, orders as the reference drew them."""
    import numpy as np
    from ldpc_sparc_amd import sparc
    cp = dict(cp)
    sparc.check_code_params(cp)
    tmp = cp.copy()
    tmp.update({'awgn_var': var})
    W = sparc.create_base_matrix(**tmp)
    key = f"{name}_s{si}"
    n = int(g[key + "_n"])
    L, M = cp['L'], cp['M']
    o0, o1 = g[key + "_order0"], g[key + "_order1"]
    if W.ndim == 0:
        return W, L, M, n, o0[0], o1[0]
    if W.ndim == 1:
        return W, L, M, n, o0, o1
    Lr, Lc = W.shape
    O0 = np.zeros((Lr, Lc, o0.shape[1]), np.uint32)
    O1 = np.zeros((Lr, Lc, o1.shape[1]), np.uint32)
    nz = [(r, c) for r in range(Lr) for c in range(Lc) if W[r, c] != 0]
    for t, (r, c) in enumerate(nz):
        O0[r, c] = o0[t]
        O1[r, c] = o1[t]
    return W, L, M, n, O0, O1
