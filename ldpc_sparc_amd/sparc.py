"""Sparse regression codes (SPARCs) with a GPU AMP decoder.

Drop-in for sparc_public/sparc.py (Kuan Hsieh's SPARC library as vendored in
SophieLangdon27/LDPC_SPARC): same function names, argument meaning, dict
mutation and return values.  The AMP loop (sparc_amp, sparc.py:883-999) and
the design operators returned by sparc_transforms (sparc.py:703-880) run on
the MI355X through libldpc_sparc_amd (include/ldpc_sparc_amd.h); the code
parameter handling, bit <-> message-vector formats, base matrices and the
random orderings are host-side and follow the reference exactly.

Engine knobs (not in the reference, ignored by it): decode_params may carry
'precision' ('f64' default, the reference's arithmetic; 'f32' the throughput
path).  Complex / PSK-modulated SPARCs (sub_fft, K>1) are not part of the
GPU engine and raise NotImplementedError.
"""
import ctypes as ct
from copy import copy

import numpy as np

from . import _native

# ------------------------------------------------------------------ helpers


def is_power_of_2(x):
    return (x > 0) and ((x & (x - 1)) == 0)


def _precision(decode_params):
    p = (decode_params or {}).get('precision', 'f64')
    if p not in ('f64', 'f32'):
        raise ValueError("decode_params['precision'] must be 'f64' or 'f32'")
    return _native.SG_F64 if p == 'f64' else _native.SG_F32


# ------------------------------------------------------------------ encode / decode


def sparc_encode(code_params, awgn_var, rand_seed):
    """Bits -> message vector -> codeword x = A beta0 (sparc.py:17-53).
    Mutates code_params (check_code_params, then adds 'n' and 'R_actual')."""
    check_code_params(code_params)
    R, L, M = map(code_params.get, ['R', 'L', 'M'])
    K = code_params['K'] if code_params['modulated'] else 1
    if K != 1:
        raise NotImplementedError("modulated SPARCs are not part of the GPU engine")

    bit_len = int(round(L * np.log2(K * M)))
    bits_in = rnd_bin_arr(bit_len, rand_seed)
    beta0 = bin_arr_2_msg_vector(bits_in, M, K)

    tmp = code_params.copy()
    tmp.update({'awgn_var': awgn_var})
    W = create_base_matrix(**tmp)

    n = int(round(bit_len / R))
    if W.ndim == 2:
        Lr, _ = W.shape
        Mr = int(round(n / Lr))
        n = Mr * Lr
    R_actual = bit_len / n
    code_params.update({'n': n, 'R_actual': R_actual})

    Ab, Az = sparc_transforms(W, L, M, n, rand_seed, code_params['complex'])
    x = Ab(beta0)
    return bits_in, beta0, x, Ab, Az


def sparc_decode(y, code_params, decode_params, awgn_var, rand_seed, beta0, Ab=None, Az=None):
    """AMP decode + hard decision + bits (sparc.py:55-74)."""
    check_decode_params(decode_params)
    beta, t_final, nmse, psi = sparc_amp(y, code_params, decode_params, awgn_var, rand_seed, beta0,
                                         Ab, Az)
    expect_err = psi.mean() >= 0.001
    K = code_params['K'] if code_params['modulated'] else 1
    bits_out = msg_vector_2_bin_arr(beta, code_params['M'], K)
    return bits_out, beta, t_final, nmse, expect_err


# ------------------------------------------------------------------ parameter checks


def check_code_params(code_params):
    """Validate and rewrite code_params in place (sparc.py:77-149)."""
    out = {}

    def take(keys):
        if all(k in code_params for k in keys):
            for k in keys:
                out[k] = copy(code_params[k])
        else:
            raise Exception('Need code parameters {}.'.format(keys))

    for flag in ('complex', 'modulated', 'power_allocated', 'spatially_coupled'):
        if flag not in code_params:
            code_params[flag] = False
        else:
            assert type(code_params[flag]) == bool, "'{}' must be boolean".format(flag)
        out[flag] = copy(code_params[flag])

    take(['P', 'R', 'L', 'M'])
    P, R, L, M = map(code_params.get, ['P', 'R', 'L', 'M'])
    assert (type(P) == float or type(P) == np.float64) and P > 0
    assert (type(R) == float or type(R) == np.float64) and R > 0
    assert type(L) == int and L > 0
    assert type(M) == int and M > 0 and is_power_of_2(M)

    if code_params['modulated']:
        take(['K'])
        K = code_params['K']
        assert type(K) == int and K > 1 and is_power_of_2(K)
        if not code_params['complex']:
            assert K == 2, 'Real-modulated SPARCs requires K=2'

    if code_params['power_allocated']:
        take(['B', 'R_PA_ratio'])
        B, R_PA_ratio = map(code_params.get, ['B', 'R_PA_ratio'])
        assert type(B) == int and B > 1
        assert L % B == 0, 'B must divide L'
        assert type(R_PA_ratio) == float or type(R_PA_ratio) == np.float64
        assert R_PA_ratio >= 0

    if code_params['spatially_coupled']:
        take(['omega', 'Lambda'])
        omega, Lambda = map(code_params.get, ['omega', 'Lambda'])
        assert type(omega) == int and omega > 1
        assert type(Lambda) == int and Lambda >= (2 * omega - 1)
        assert L % Lambda == 0, 'Lambda must divide L'

    if code_params['power_allocated'] and code_params['spatially_coupled']:
        assert L % (Lambda * B) == 0, 'Lambda*B must divide L'

    code_params.clear()
    code_params.update(dict(out))


def check_decode_params(decode_params):
    """Validate decode_params and fill defaults in place (sparc.py:151-170)."""
    if 't_max' not in decode_params:
        raise Exception('Need decode parameters {}.'.format(['t_max']))
    for key, val in {'rtol': 1e-6, 'phi_est_method': 1}.items():
        if key not in decode_params:
            decode_params[key] = val
    t_max, rtol, phi_est_method = map(decode_params.get, ['t_max', 'rtol', 'phi_est_method'])
    assert type(t_max) == int and t_max > 1
    assert type(rtol) == float and 0 < rtol < 1
    assert phi_est_method == 1 or phi_est_method == 2


# ------------------------------------------------------------------ bits and message vectors


def rnd_bin_arr(k, rand_seed):
    """k random bits from RandomState(rand_seed) (sparc.py:174-180)."""
    assert type(k) == int
    return np.random.RandomState(rand_seed).randint(2, size=k, dtype='bool')


def bin_arr_2_int(bin_array):
    """MSB-first bits -> integer (sparc.py:182-189)."""
    assert bin_array.dtype == 'bool'
    k = bin_array.size
    assert 0 < k < 64
    return bin_array.dot(1 << np.arange(k)[::-1])


def int_2_bin_arr(integer, arr_length):
    """Integer -> MSB-first bits of length arr_length (sparc.py:191-197, with the
    numpy-1.26 semantics the reference pins)."""
    assert integer >= 0
    return ((int(integer) >> np.arange(arr_length)[::-1]) & 1).astype(bool)


def _bits_to_indices(bin_arr, logM):
    w = 1 << np.arange(logM)[::-1]
    return bin_arr.reshape(-1, logM).astype(np.int64) @ w


def _indices_to_bits(idx, logM):
    return ((np.asarray(idx, dtype=np.int64)[:, None] >> np.arange(logM)[::-1]) & 1).astype(bool).ravel()


def rnd_msg_vector(L, M, rand_seed, K=1):
    """Random unmodulated message vector (sparc.py:303-328, K=1)."""
    if K != 1:
        raise NotImplementedError("modulated SPARCs are not part of the GPU engine")
    rng = np.random.RandomState(rand_seed)
    assert type(M) == int and M > 0 and is_power_of_2(M)
    mv = np.zeros((L, M))
    mv[(np.arange(L), rng.randint(0, M, L))] = np.ones(L)
    return mv.ravel()


def bin_arr_2_msg_vector(bin_arr, M, K=1):
    """Bits -> one-hot message vector, log2 M MSB-first bits per section
    (sparc.py:330-364, K=1)."""
    assert type(M) == int and M > 0 and is_power_of_2(M)
    if K != 1:
        raise NotImplementedError("modulated SPARCs are not part of the GPU engine")
    logM = int(round(np.log2(M)))
    assert bin_arr.size % logM == 0
    L = bin_arr.size // logM
    mv = np.zeros(L * M)
    mv[np.arange(L) * M + _bits_to_indices(np.asarray(bin_arr, dtype=bool), logM)] = 1
    return mv


def msg_vector_2_bin_arr(msg_vector, M, K=1):
    """One-hot message vector -> bits (sparc.py:366-400, K=1)."""
    assert type(msg_vector) == np.ndarray
    assert type(M) == int and M > 0 and is_power_of_2(M)
    assert msg_vector.size % M == 0
    if K != 1:
        raise NotImplementedError("modulated SPARCs are not part of the GPU engine")
    logM = int(round(np.log2(M)))
    L = msg_vector.size // M
    rows, cols = np.nonzero(msg_vector.reshape(L, M))
    assert np.array_equal(rows, np.arange(L))
    return _indices_to_bits(cols, logM)


def msg_vector_mmse_estimator(s, tau, M, K=1):
    """Per-section softmax of s/tau (sparc.py:402-465, K=1), evaluated on the GPU
    in double precision with a per-section maximum (the reference's global
    maximum in float128 is the same function)."""
    assert type(s) == np.ndarray
    assert s.size % M == 0
    if K != 1 or np.iscomplexobj(s):
        raise NotImplementedError("modulated SPARCs are not part of the GPU engine")
    _native.require_gpu()
    x = np.ascontiguousarray(s.real / tau, dtype=np.float64)
    out = np.empty_like(x)
    _native.check(_native.lib().sg_section_softmax(_native.ptr(x), x.size // M, M, 1.0,
                                                   _native.ptr(out)))
    return out


def msg_vector_map_estimator(s, M, K=1):
    """One-hot argmax per section (sparc.py:467-512, K=1), on the GPU."""
    assert type(s) == np.ndarray
    assert s.size % M == 0
    if K != 1 or np.iscomplexobj(s):
        raise NotImplementedError("modulated SPARCs are not part of the GPU engine")
    _native.require_gpu()
    L = s.size // M
    x = np.ascontiguousarray(s.real, dtype=np.float64)
    idx = np.empty(L, dtype=np.int32)
    _native.check(_native.lib().sg_section_argmax(_native.ptr(x), L, M, _native.ptr(idx)))
    beta = np.zeros((L, M))
    beta[np.arange(L), idx] = 1
    return beta.ravel()


# ------------------------------------------------------------------ base matrices


def pa_iterative(P, sigmaSqr, B, R_PA):
    """Iterative power allocation from asymptotic SE (sparc.py:516-533)."""
    Q = np.zeros(B)
    for b in range(B):
        phi = sigmaSqr + P - Q.mean()
        p_block = 2 * np.log(2) * R_PA * phi
        p_spread = (B * P - Q.sum()) / (B - b)
        if p_block > p_spread:
            Q[b:b + 1] = p_block
        else:
            Q[b:] = p_spread
            break
    Q /= Q.mean() / P
    return Q


def sc_basic(Q, omega, Lambda):
    """(omega, Lambda) spatially coupled base matrix (sparc.py:535-568)."""
    assert type(Q) == np.ndarray
    Lr = Lambda + omega - 1
    if Q.ndim == 0:
        W = np.zeros((Lr, Lambda))
        for c in range(Lambda):
            W[c:c + omega, c] = Q * Lr / omega
    elif Q.ndim == 1:
        B = Q.size
        W = np.zeros((Lr, Lambda * B))
        for c in range(Lambda):
            for r in range(c, c + omega):
                W[r, c * B:(c + 1) * B] = Q * Lr / omega
    else:
        raise Exception('Something wrong with Q')
    assert np.isclose(W.mean(), np.mean(Q)), "Average base matrix values must equal P"
    return W


def create_base_matrix(P, power_allocated=False, spatially_coupled=False, **kwargs):
    """Base entry / vector / matrix W (sparc.py:570-589)."""
    if not power_allocated:
        Q = np.array(P)
    else:
        awgn_var, B, R, R_PA_ratio = map(kwargs.get, ['awgn_var', 'B', 'R', 'R_PA_ratio'])
        Q = pa_iterative(P, awgn_var, B, R * R_PA_ratio)
    if not spatially_coupled:
        return Q
    omega, Lambda = map(kwargs.get, ['omega', 'Lambda'])
    return sc_basic(Q, omega, Lambda)


# ------------------------------------------------------------------ design operator


def transform_size(Mr, Mc):
    """w = 2^ceil(log2(max(Mr+1, Mc+1))) (sparc.py:673,744)."""
    return 2 ** int(np.ceil(np.log2(max(Mr + 1, Mc + 1))))


def generate_ordering(W, Mr, Mc, rand_seed, csparc=False):
    """Row/column sub-sampling orders (sparc.py:735-775): one RandomState, the
    same two index arrays re-shuffled cumulatively for every block (row-major
    over the nonzero entries of W)."""
    if csparc:
        raise NotImplementedError("complex SPARCs (sub_fft) are not part of the GPU engine")
    shape = W.shape
    order0 = np.zeros(shape + (Mr,), dtype=np.uint32)
    order1 = np.zeros(shape + (Mc,), dtype=np.uint32)
    w = transform_size(Mr, Mc)
    rows = np.arange(1, w, dtype=np.uint32)
    cols = np.arange(1, w, dtype=np.uint32)
    rng = np.random.RandomState(rand_seed)
    if W.ndim == 0:
        rng.shuffle(rows)
        rng.shuffle(cols)
        return rows[:Mr], cols[:Mc]
    blocks = [(b,) for b in range(shape[0])] if W.ndim == 1 else \
        [(r, c) for r in range(shape[0]) for c in range(shape[1]) if W[r, c] != 0]
    if W.ndim > 2:
        raise Exception("Something is wrong with the ordering")
    for blk in blocks:
        rng.shuffle(rows)
        rng.shuffle(cols)
        order0[blk] = rows[:Mr]
        order1[blk] = cols[:Mc]
    return order0, order1


class DesignOperator:
    """A sub-sampled DCT design matrix A (n x LM) on the GPU.

    Holds the base matrix and orders; `Ab(x)` = A x and `Az(y)` = A^T y are the
    callables sparc_transforms returns (sparc.py:786-875).  Plans (device
    tables) are built lazily per precision and reused by the AMP decoder."""

    def __init__(self, W, L, M, n, order0, order1):
        self.W = np.array(W, dtype=np.float64)
        self.L, self.M, self.n = int(L), int(M), int(n)
        self.LM = self.L * self.M
        nd = self.W.ndim
        self.Lr = self.W.shape[0] if nd == 2 else 1
        self.Lc = self.W.shape[-1] if nd >= 1 else 1
        self.Mr = self.n // self.Lr if nd == 2 else self.n
        self.Mc = self.LM // self.Lc
        if nd == 0:
            o0, o1 = [np.asarray(order0)], [np.asarray(order1)]
        elif nd == 1:
            o0 = [order0[b] for b in range(self.Lc)]
            o1 = [order1[b] for b in range(self.Lc)]
        else:
            nz = [(r, c) for r in range(self.Lr) for c in range(self.Lc) if self.W[r, c] != 0]
            o0 = [order0[r, c] for r, c in nz]
            o1 = [order1[r, c] for r, c in nz]
        self.order0 = np.ascontiguousarray(np.stack(o0), dtype=np.uint32)
        self.order1 = np.ascontiguousarray(np.stack(o1), dtype=np.uint32)
        self.w = transform_size(self.Mr, self.Mc)
        self._plans = {}

    def plan(self, precision=_native.SG_F64):
        if precision not in self._plans:
            _native.require_gpu()
            h = ct.c_void_p()
            Wf = np.ascontiguousarray(self.W.reshape(-1), dtype=np.float64)
            _native.check(_native.lib().sg_amp_plan_create(
                self.W.ndim, _native.ptr(Wf), self.Lr, self.Lc, self.L, self.M, self.n,
                _native.ptr(self.order0), _native.ptr(self.order1), precision, ct.byref(h)))
            self._plans[precision] = h
        return self._plans[precision]

    def __del__(self):
        for h in getattr(self, "_plans", {}).values():
            try:
                _native.lib().sg_amp_plan_destroy(h)
            except Exception:
                pass

    def apply(self, x, transpose, precision=_native.SG_F64):
        x = np.ascontiguousarray(x, dtype=np.float64)
        batched = x.ndim == 2
        X = x if batched else x[None, :]
        B = X.shape[0]
        out = np.empty((B, self.LM if transpose else self.n))
        _native.check(_native.lib().sg_amp_apply(self.plan(precision), int(transpose), _native.ptr(X),
                                                 B, _native.ptr(out)))
        return out if batched else out[0]

    def Ab(self, x):
        assert np.asarray(x).shape[-1] == self.LM
        return self.apply(x, False)

    def Az(self, y):
        assert np.asarray(y).shape[-1] == self.n
        return self.apply(y, True)


def sparc_transforms(W, L, M, n, rand_seed, csparc=False):
    """Ab(x) = A x and Az(y) = A^T y for the design given by (W, seed)
    (sparc.py:703-880), evaluated on the GPU."""
    assert type(W) == np.ndarray
    assert type(L) == int and type(M) == int and type(n) == int
    assert L > 0 and M > 0 and n > 0
    if csparc:
        raise NotImplementedError("complex SPARCs (sub_fft) are not part of the GPU engine")
    if W.ndim == 0:
        Mr, Mc = n, L * M
    elif W.ndim == 1:
        assert L % W.size == 0
        Mr, Mc = n, L * M // W.size
    elif W.ndim == 2:
        Lr, Lc = W.shape
        assert L % Lc == 0
        assert n % Lr == 0
        Mr, Mc = n // Lr, L * M // Lc
    else:
        raise Exception('Something wrong with base matrix input W')
    order0, order1 = generate_ordering(W, Mr, Mc, rand_seed, csparc)
    op = DesignOperator(W, L, M, n, order0, order1)
    return op.Ab, op.Az


def operator_of(Ab, Az):
    """The DesignOperator behind Ab/Az callables from sparc_transforms, or None."""
    a, b = getattr(Ab, "__self__", None), getattr(Az, "__self__", None)
    if isinstance(a, DesignOperator) and a is b:
        return a
    return None


# ------------------------------------------------------------------ AMP


def amp_decode_batch(Y, op, awgn_var, t_max, rtol=1e-6, phi_est_method=1, true_idx=None,
                     precision=_native.SG_F64):
    """Batched AMP on the GPU for codewords sharing one design.

    Y [B, n] received words; true_idx [B, L] transmitted section indices (for
    NMSE) or None.  Returns (map_idx [B, L], t_final [B], nmse [B, t_max, Lc],
    psi [B, Lc])."""
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    if Y.ndim != 2 or Y.shape[1] != op.n:
        raise ValueError(f"received words must have shape [B, {op.n}]")
    B = Y.shape[0]
    ti = None
    if true_idx is not None:
        ti = np.ascontiguousarray(true_idx, dtype=np.int32).reshape(B, op.L)
    map_idx = np.empty((B, op.L), dtype=np.int32)
    t_final = np.empty(B, dtype=np.int32)
    nmse = np.empty((B, t_max, op.Lc))
    psi = np.empty((B, op.Lc))
    _native.check(_native.lib().sg_amp_decode(
        op.plan(precision), _native.ptr(Y), B, _native.ptr(ti), float(awgn_var), int(t_max),
        float(rtol), int(phi_est_method), _native.ptr(map_idx), _native.ptr(t_final),
        _native.ptr(nmse), _native.ptr(psi)))
    return map_idx, t_final, nmse, psi


def sparc_amp(y, code_params, decode_params, awgn_var, rand_seed, beta0, Ab=None, Az=None):
    """AMP decoder (sparc.py:883-999) on the GPU.  Returns (beta_MAP, t_final,
    nmse, psi) with the reference's shapes: nmse (t_max,) for a regular
    design, (t_max, Lc) otherwise; psi a scalar or (Lc,)."""
    P, R, L, M, n = map(code_params.get, ['P', 'R', 'L', 'M', 'n'])
    K = code_params['K'] if code_params['modulated'] else 1
    if K != 1 or code_params.get('complex', False):
        raise NotImplementedError("complex / modulated SPARCs are not part of the GPU engine")
    tmp = code_params.copy()
    tmp.update({'awgn_var': awgn_var})
    W = create_base_matrix(**tmp)
    assert 0 <= W.ndim <= 2
    t_max, rtol, phi_est_method = map(decode_params.get, ['t_max', 'rtol', 'phi_est_method'])
    assert phi_est_method == 1 or phi_est_method == 2

    if Ab is None or Az is None:
        Ab, Az = sparc_transforms(W, L, M, n, rand_seed, code_params['complex'])
    op = operator_of(Ab, Az)
    if op is None:
        raise NotImplementedError("sparc_amp runs fused on the GPU and needs the Ab/Az returned "
                                  "by ldpc_sparc_amd.sparc.sparc_transforms")
    true_idx = None
    if beta0 is not None:
        b0 = np.asarray(beta0).reshape(L, M)
        true_idx = np.argmax(b0 != 0, axis=1).astype(np.int32)[None, :]
    map_idx, t_final, nmse, psi = amp_decode_batch(np.asarray(y)[None, :], op, awgn_var, t_max,
                                                   rtol, phi_est_method, true_idx,
                                                   _precision(decode_params))
    beta = np.zeros((L, M))
    beta[np.arange(L), map_idx[0]] = 1
    if W.ndim == 0:
        return beta.ravel(), int(t_final[0]), nmse[0, :, 0].copy(), np.float64(psi[0, 0])
    return beta.ravel(), int(t_final[0]), nmse[0].copy(), psi[0].copy()


def test_bin_arr_msg_vector(k=1024 * 9, M=2 ** 9):
    """Round trip bits -> beta -> bits (sparc.py:1003-1008)."""
    seed = list(np.random.randint(2 ** 32 - 1, size=2))
    bin_array = rnd_bin_arr(k, seed)
    msg_vector = bin_arr_2_msg_vector(bin_array, M)
    assert np.array_equal(bin_array, msg_vector_2_bin_arr(msg_vector, M))
