"""TEST INFRASTRUCTURE ONLY -- numpy/scipy restatement of the SPARC AMP path.

Restates sparc_public/sparc.py (sub_dct :648-701, sparc_transforms :703-880,
msg_vector_mmse_estimator :402-465 with K=1, msg_vector_map_estimator
:467-512, sparc_amp :883-999) and sparc_sophie/sparc_new.py (dense Gaussian
design: sparc_amp :885-912, msg_vector_mmse_estimator :1040-1066,
msg_vector_map_estimator :1099-1116, beta_estimate_to_bp_probs :1118-1138)
with the same numpy operations and order, so that it reproduces the
reference's double-precision results (pinned against reference traces in
tests/test_oracle_pin.py).  Used by tests/ as the checker and by bench.py as
the CPU baseline ("port").  Never imported by the product.
"""
import numpy as np
from scipy.fftpack import dct, idct


def _transform_size(Mr, Mc):
    return 2 ** int(np.ceil(np.log2(max(Mr + 1, Mc + 1))))


def sub_dct_ops(Mr, Mc, order0, order1):
    """A x and A^T y of one sub-sampled DCT block (sparc.py:687-699)."""
    w = _transform_size(Mr, Mc)

    def Ax(x):
        ext = np.zeros(w)
        ext[order1] = x.reshape(Mc)
        return np.sqrt(w) * dct(ext, norm='ortho')[order0]

    def Ay(y):
        ext = np.zeros(w)
        ext[order0] = y
        return np.sqrt(w) * idct(ext, norm='ortho')[order1]
    return Ax, Ay


def dct_operators(W, L, M, n, order0, order1):
    """Ab / Az over all blocks of W (sparc.py:777-875); order arrays shaped as
    generate_ordering returns them."""
    W = np.asarray(W, dtype=float)
    if W.ndim == 0:
        ax, ay = sub_dct_ops(n, L * M, order0, order1)
        return (lambda x: np.sqrt(W / L) * ax(x)), (lambda y: np.sqrt(W / L) * ay(y))
    if W.ndim == 1:
        B = W.size
        Mc = L * M // B
        ops = [sub_dct_ops(n, Mc, order0[b], order1[b]) for b in range(B)]

        def Ab(x):
            out = np.zeros(n)
            for b in range(B):
                out += np.sqrt(W[b] / L) * ops[b][0](x[b * Mc:(b + 1) * Mc])
            return out

        def Az(y):
            out = np.zeros(B * Mc)
            for b in range(B):
                out[b * Mc:(b + 1) * Mc] += np.sqrt(W[b] / L) * ops[b][1](y)
            return out
        return Ab, Az
    Lr, Lc = W.shape
    Mc, Mr = L * M // Lc, n // Lr
    ops = {(r, c): sub_dct_ops(Mr, Mc, order0[r, c], order1[r, c])
           for r in range(Lr) for c in range(Lc) if W[r, c] != 0}

    def Ab(x):
        out = np.zeros(Lr * Mr)
        for r in range(Lr):
            for c in range(Lc):
                if W[r, c] != 0:
                    out[r * Mr:(r + 1) * Mr] += np.sqrt(W[r, c] / L) * ops[r, c][0](x[c * Mc:(c + 1) * Mc])
        return out

    def Az(y):
        out = np.zeros(Lc * Mc)
        for r in range(Lr):
            for c in range(Lc):
                if W[r, c] != 0:
                    out[c * Mc:(c + 1) * Mc] += np.sqrt(W[r, c] / L) * ops[r, c][1](y[r * Mr:(r + 1) * Mr])
        return out
    return Ab, Az


def mmse_estimator(s, tau, M):
    """Per-section softmax with the global maximum, exp in float128 (sparc.py:429-432,463)."""
    x = s.real / tau
    top = np.exp(x - x.max(), dtype=np.longdouble)
    bot = top.reshape(-1, M).sum(axis=1).repeat(M)
    return (top / bot).astype(np.float64)


def map_estimator(s, M):
    L = s.size // M
    beta = np.zeros((L, M))
    beta[np.arange(L), s.reshape(L, -1).argmax(axis=1)] = 1
    return beta.ravel()


def amp(y, W, L, M, n, awgn_var, t_max, Ab, Az, beta0, rtol=1e-6, phi_method=1, trace=None):
    """AMP loop of sparc.py:913-999.  trace(t, dict) is called after every
    iteration with the state (s, beta, z, tau, phi, psi).  Returns
    (beta_map, t_final, nmse, psi)."""
    W = np.asarray(W, dtype=float)
    beta = np.zeros(L * M)
    z = y
    atol = 2 * np.finfo(np.float64).resolution
    if W.ndim == 0:
        gamma = W
        nmse = np.ones(t_max)
    else:
        if W.ndim == 2:
            Lr = W.shape[0]
            Mr = n // Lr
        Lc = W.shape[-1]
        Mc = L * M // Lc
        gamma = np.dot(W, np.ones(Lc)) / Lc
        nmse = np.ones((t_max, Lc))
    psi = phi = None
    for t in range(t_max - 1):
        if t > 0:
            psi_prev = np.copy(psi)
            phi_prev = np.copy(phi)
            gamma = W * psi if W.ndim == 0 else np.dot(W, psi) / Lc
            b = gamma / phi_prev
            z = y - Ab(beta) + (b * z if W.ndim != 2 else b.repeat(Mr) * z)
        if phi_method == 1:
            phi = awgn_var + gamma
        else:
            phi = (np.abs(z) ** 2).mean() if W.ndim != 2 else (np.abs(z) ** 2).reshape(Lr, -1).mean(axis=1)
        if W.ndim == 0:
            tau = (L * phi / n) / W
            tau_use, phi_use = tau, phi
        elif W.ndim == 1:
            tau = (L * phi / n) / W
            tau_use, phi_use = tau.repeat(Mc), phi
        else:
            tau = (L / Mr) / np.dot(W.T, 1 / phi)
            tau_use, phi_use = tau.repeat(Mc), phi.repeat(Mr)
        s = beta + tau_use * Az(z / phi_use)
        beta = mmse_estimator(s, tau_use, M)
        if W.ndim == 0:
            psi = 1 - (np.abs(beta) ** 2).sum() / L
            nmse[t + 1] = (np.abs(beta - beta0) ** 2).sum() / L
        else:
            psi = 1 - (np.abs(beta) ** 2).reshape(Lc, -1).sum(axis=1) / (L / Lc)
            nmse[t + 1] = (np.abs(beta - beta0) ** 2).reshape(Lc, -1).sum(axis=1) / (L / Lc)
        if trace is not None:
            trace(t, {'s': s, 'beta': beta, 'z': np.array(z), 'tau': tau, 'phi': phi, 'psi': psi})
        if t > 0 and np.allclose(psi, psi_prev, rtol, atol=atol):
            nmse[t:] = nmse[t]
            break
    return map_estimator(s, M), t + 1, nmse, psi


# ---------------------------------------------------------------- dense Gaussian design (sophie)

def dense_mmse_estimator(s, tau_sqr, n, P_l, M):
    """sparc_new.py:1040-1066 (global maximum, float64)."""
    x = np.sqrt(n * P_l) * (s / tau_sqr)
    top = np.exp(x - x.max(), dtype=np.float64)
    bot = top.reshape(-1, M).sum(axis=1).repeat(M)
    return ((np.sqrt(n * P_l)) * (top / bot)).astype(np.float64)


def dense_amp(y, A, P, L, M, t_max):
    """sparc_new.py:885-912: fixed t_max iterations, empirical tau^2.  Returns (beta, s)."""
    n = len(y)
    P_l = P / L
    AT = A.T
    beta = np.zeros(L * M)
    z = y
    for t in range(t_max):
        if t > 0:
            Ab = np.dot(A, beta)
            ons = (z / tau_sqr) * (P - ((np.sum(beta ** 2)) / n))
            z = y - Ab + ons
        s = beta + np.dot(AT, z)
        tau_sqr = np.sum(z ** 2) / n
        beta = dense_mmse_estimator(s, tau_sqr, n, P_l, M)
    return beta, s


def beta_to_bit_probs(beta, L, M, sqrt_nP_l):
    """P(bit = 0) per section bit, MSB first (sparc_new.py:1118-1138), vectorised."""
    logM = int(np.log2(M))
    b = beta.reshape(L, M) / sqrt_nP_l
    j = np.arange(M)
    out = np.zeros((L, logM))
    for pos in range(logM):
        bit = logM - 1 - pos
        out[:, pos] = b[:, ((j >> bit) & 1) == 0].sum(axis=1)
    return out.reshape(L * logM)
