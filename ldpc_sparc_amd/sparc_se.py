"""SPARC state evolution (drop-in for sparc_public/sparc_se.py).

sparc_se(awgn_var, code_params, t_max, mc_samples) keeps the reference's
arguments, code_params rewrite (check_code_params) and return value
(psi [t_max] or [t_max, Lc], final tau).  The Monte-Carlo samples are drawn
exactly as the reference draws them -- np.random.randn(mc_samples, M) from
numpy's global state -- then stay resident on the GPU, where every
expectation sparc_se_E (:82-115) of an iteration is evaluated for all column
blocks in one launch (se.hip).  Real SPARCs (K = 1, and K = 2 modulated) and
complex unmodulated ones are supported; complex PSK-modulated SPARCs (K > 2)
are outside the engine.
"""
import ctypes as ct
from copy import copy

import numpy as np

from . import _native
from .sparc import create_base_matrix, is_power_of_2


def check_code_params(code_params):
    """Validate and rewrite code_params in place (sparc_se.py:13-80): the type
    flags default to False; P, R, M are required; K for modulated, B and
    R_PA_ratio for power allocated, omega and Lambda for spatially coupled."""
    keep = {}

    def need(keys):
        missing = [k for k in keys if k not in code_params]
        if missing:
            raise Exception('Need code parameters {}.'.format(keys))
        for k in keys:
            keep[k] = copy(code_params[k])

    for flag in ('complex', 'modulated', 'power_allocated', 'spatially_coupled'):
        code_params.setdefault(flag, False)
        assert type(code_params[flag]) == bool, "'{}' must be boolean".format(flag)
        keep[flag] = code_params[flag]
    need(['P', 'R', 'M'])
    P, R, M = code_params['P'], code_params['R'], code_params['M']
    assert isinstance(P, (float, np.float64)) and P > 0
    assert isinstance(R, (float, np.float64)) and R > 0
    assert type(M) == int and M > 0 and is_power_of_2(M)
    if code_params['modulated']:
        need(['K'])
        K = code_params['K']
        assert type(K) == int and K > 1 and is_power_of_2(K)
        if not code_params['complex']:
            assert K == 2, 'Real-modulated SPARCs requires K=2'
    if code_params['power_allocated']:
        need(['B', 'R_PA_ratio'])
        assert type(code_params['B']) == int and code_params['B'] > 1
        assert isinstance(code_params['R_PA_ratio'], (float, np.float64)) and code_params['R_PA_ratio'] >= 0
    if code_params['spatially_coupled']:
        need(['omega', 'Lambda'])
        assert type(code_params['omega']) == int and code_params['omega'] > 1
        assert type(code_params['Lambda']) == int and code_params['Lambda'] >= 2 * code_params['omega'] - 1
    code_params.clear()
    code_params.update(keep)


class SeSamples:
    """Monte-Carlo samples u [mc, M] resident on the GPU."""

    def __init__(self, u):
        _native.require_gpu()
        self.u = np.ascontiguousarray(u, dtype=np.float64)
        self.h = ct.c_void_p()
        _native.check(_native.lib().sg_se_samples_create(_native.ptr(self.u), self.u.shape[0], self.u.shape[1],
                                                         ct.byref(self.h)))

    def expectation(self, taus, K):
        taus = np.ascontiguousarray(np.atleast_1d(taus), dtype=np.float64)
        E = np.empty_like(taus)
        _native.check(_native.lib().sg_se_expectation(self.h, int(K), _native.ptr(taus), taus.size, _native.ptr(E)))
        return E

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                _native.lib().sg_se_samples_destroy(h)
            except Exception:
                pass


def sparc_se_E(tau, K, u):
    """Mean over the samples of the posterior weight of the true entry
    (sparc_se.py:82-115), on the GPU; tau may be a vector."""
    if K not in (1, 2):
        raise NotImplementedError("complex PSK-modulated SPARCs (K > 2) are not part of the GPU engine")
    E = SeSamples(u).expectation(tau, K)
    return E if np.ndim(tau) else float(E[0])


def sparc_se(awgn_var, code_params, t_max, mc_samples):
    """State evolution for SPARCs (sparc_se.py:117-183).  Returns (psi, tau)."""
    check_code_params(code_params)
    tmp = code_params.copy()
    tmp.update({'awgn_var': awgn_var})
    W = create_base_matrix(**tmp)
    assert 0 <= W.ndim <= 2
    P, R, M = map(code_params.get, ['P', 'R', 'M'])
    K = code_params['K'] if code_params['modulated'] else 1
    if code_params['complex']:
        R /= 2
    if W.ndim == 0:
        psi = np.ones(t_max)
    else:
        Lr, Lc = (1, W.size) if W.ndim == 1 else W.shape
        psi = np.ones((t_max, Lc))
    if K > 2:
        raise NotImplementedError("complex PSK-modulated SPARCs (K > 2) are not part of the GPU engine")
    u = np.random.randn(mc_samples, M)  # the reference's draw from numpy's global state
    samples = SeSamples(u)
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
        psi[t + 1] = 1 - samples.expectation(tau, K) if W.ndim else 1 - samples.expectation(tau, K)[0]
    return psi, tau
