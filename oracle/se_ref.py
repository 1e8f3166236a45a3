"""TEST INFRASTRUCTURE ONLY -- numpy restatement of SPARC state evolution,
sparc_public/sparc_se.py: sparc_se_E :82-115 (K = 1 and 2) and the tau / psi
recursion of sparc_se :117-183.  Pinned against tests/golden/se_golden.npz
(the reference run with seeded numpy samples) in tests/test_oracle_pin.py.
Never imported by the product."""
import numpy as np

from ldpc_sparc_amd.sparc import create_base_matrix


def se_E(tau, K, u):
    """sparc_se.py:82-115 for K in (1, 2)."""
    itau = 1 / tau
    rtau = np.sqrt(itau)
    if K == 1:
        a = np.exp(itau + rtau * u[:, 0])
        c = np.exp(rtau * u[:, 1:])
    else:
        a = np.sinh(itau + rtau * u[:, 0])
        c = np.cosh(rtau * u[:, 1:])
    return (a / (a + c.sum(axis=1))).mean()


def se(awgn_var, code_params, t_max, u):
    """sparc_se.py:117-183 with the Monte-Carlo samples u supplied."""
    cp = dict(code_params)
    tmp = dict(cp, awgn_var=awgn_var)
    W = create_base_matrix(**tmp)
    P, R, M = cp['P'], cp['R'], cp['M']
    K = cp['K'] if cp.get('modulated') else 1
    if cp.get('complex'):
        R /= 2
    if W.ndim == 0:
        psi = np.ones(t_max)
    else:
        Lr, Lc = (1, W.size) if W.ndim == 1 else W.shape
        psi = np.ones((t_max, Lc))
    for t in range(t_max - 1):
        if t > 0:
            tau_prev = np.copy(tau)
        if W.ndim == 0:
            tau = (np.log(2) * R / np.log(K * M)) * (awgn_var / P + psi[t])
        else:
            phi = awgn_var + np.dot(W, psi[t]) / Lc
            tau = (np.log(2) * R * Lr / np.log(K * M)) / np.dot(W.T, 1 / phi)
        if (t > 0) and np.allclose(tau, tau_prev, rtol=1e-6, atol=0):
            psi[t:] = psi[t]
            break
        if W.ndim == 0:
            psi[t + 1] = 1 - se_E(tau, K, u)
        else:
            for c in range(Lc):
                psi[t + 1, c] = 1 - se_E(tau[c], K, u)
    return psi, tau
