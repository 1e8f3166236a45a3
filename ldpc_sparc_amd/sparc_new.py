"""SPARC with a dense Gaussian design, concatenated with an LDPC outer code.

Drop-in for sparc_sophie/sparc_new.py (the Sophie Langdon fork's SPARC/LDPC
library): the main encode/decode path and its helpers keep the reference's
names, arguments and return values.  AMP (sparc_amp, sparc_new.py:885-912),
the section estimators, the AMP -> BP glue (beta_estimate_to_bp_probs
:1118-1138) and BP (ldpc_bp :1162-1193) run on the MI355X through
libldpc_sparc_amd; the design matrix and the message bits are drawn on the
host with the reference's numpy generators so that results are reproducible
seed for seed (parity mode).

The AMP <-> BP integrated decoders (naively_integrated_decoder :257-282,
naively_integrated_decoder_posteriors :411-439, integrated_decoder :472-502,
integrated_decoder_posteriors :675-705) run as one batched device loop
(sg_integrated_decode); their pieces (eta :709-735, eta_posteriors :793-822,
differentiated_eta_calc(_posteriors) :824-869, update_using_bp_probs
:1030-1038, bp_output_to_beta_estimate :1260-1279) are available on their
own.  integrated_decode_batch decodes many received words sharing one design.

Not provided (the fork's diagnostic variants): *_decode_loop,
*_test*, sparc_amp_loop/_termination, no_onsager_decoder.

Engine knobs (absent from the reference): decode_params may carry
'precision' ('f64' default; 'f32' runs the products on the matrix cores).
"""
import ctypes as ct

import numpy as np

from . import _native
from .ldpc import code

# ------------------------------------------------------------------ device plans


class DenseDesign:
    """A dense design matrix A [n][L*M] resident on the GPU (one plan per precision)."""

    def __init__(self, A=None, P=None, L=None, M=None, n=None, seed=None):
        self.A = None if A is None else np.ascontiguousarray(A, dtype=np.float64)
        self.P, self.L, self.M = float(P), int(L), int(M)
        self.n = int(self.A.shape[0]) if self.A is not None else int(n)
        self.seed = seed
        if self.A is not None:
            assert self.A.shape == (self.n, self.L * self.M)
        self._plans = {}

    def plan(self, precision=_native.SG_F64):
        if precision not in self._plans:
            _native.require_gpu()
            h = ct.c_void_p()
            L = _native.lib()
            if self.A is not None:
                _native.check(L.sg_dense_plan_create(_native.ptr(self.A), self.n, self.L, self.M, self.P,
                                                     precision, ct.byref(h)))
            else:
                _native.check(L.sg_dense_plan_create_random(self.n, self.L, self.M, self.P,
                                                            int(self.seed or 0), precision, ct.byref(h)))
            self._plans[precision] = h
        return self._plans[precision]

    def release(self):
        for h in self._plans.values():
            try:
                _native.lib().sg_dense_plan_destroy(h)
            except Exception:
                pass
        self._plans = {}

    def __del__(self):
        self.release()


_design_cache = {"key": None, "design": None}


def _design_for(A, P, L, M):
    """Reuse the device copy of A when the caller passes the same matrix again."""
    key = (id(A), A.shape, float(P), int(L), int(M), A.__array_interface__['data'][0])
    if _design_cache["key"] != key:
        if _design_cache["design"] is not None:
            _design_cache["design"].release()
        _design_cache["design"] = DenseDesign(A, P, L, M)
        _design_cache["key"] = key
    return _design_cache["design"]


def _precision(decode_params):
    p = (decode_params or {}).get('precision', 'f64')
    if p not in ('f64', 'f32'):
        raise ValueError("decode_params['precision'] must be 'f64' or 'f32'")
    return _native.SG_F64 if p == 'f64' else _native.SG_F32


def dense_amp_batch(Y, design, t_max, precision=_native.SG_F64):
    """Batched AMP for codewords sharing one design: Y [B, n] -> (beta, s) [B, L*M]."""
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    if Y.ndim != 2 or Y.shape[1] != design.n:
        raise ValueError(f"received words must have shape [B, {design.n}]")
    B = Y.shape[0]
    LM = design.L * design.M
    beta = np.empty((B, LM))
    s = np.empty((B, LM))
    _native.check(_native.lib().sg_dense_amp(design.plan(precision), _native.ptr(Y), B, int(t_max),
                                             _native.ptr(beta), _native.ptr(s)))
    return beta, s


# ------------------------------------------------------------------ main encode / decode


def sparc_ldpc_encode(sparc_params, ldpc_params, lengths, ldpc_bool, rand_seed):
    """Random user bits -> (LDPC) -> SPARC codeword (sparc_new.py:15-51).
    Returns (user_bits, total_bits, beta0, x, A)."""
    P, R, L, M = sparc_params['P'], sparc_params['R'], sparc_params['L'], sparc_params['M']
    logM = int(np.log2(M))
    if ldpc_bool:
        L_unprotected, k_ldpc, mults = lengths['L_unprotected'], lengths['k_ldpc'], lengths['mults']
        unprotected_bit_len = int(L_unprotected * logM)
        user_bits_len = int(k_ldpc + unprotected_bit_len)
    else:
        user_bits_len = L * logM
    rng = np.random.default_rng(rand_seed)
    user_bits = rng.integers(0, 2, size=user_bits_len)
    if ldpc_bool:
        total_bits = encode_ldpc(user_bits, ldpc_params, mults, unprotected_bit_len)
    else:
        total_bits = user_bits.astype(bool)
    encoded_bit_len = total_bits.size
    assert encoded_bit_len == L * logM
    n = int(encoded_bit_len / R)
    P_l = P / L
    beta0 = bin_arr_2_msg_vector(total_bits, M, n, P_l)
    A = create_design_matrix(L, M, n, rand_seed)
    x = np.dot(A, beta0)
    return user_bits, total_bits, beta0, x, A


def sparc_ldpc_decode(y, sparc_params, ldpc_params, decode_params, ldpc_bool, lengths, A):
    """AMP to completion, then BP on the protected sections (sparc_new.py:53-82)."""
    P, R, L, M = sparc_params['P'], sparc_params['R'], sparc_params['L'], sparc_params['M']
    n = len(y)
    sqrt_nP_l = np.sqrt(n * (P / L))
    beta_soft_estimate, s = sparc_amp(y, sparc_params, decode_params, A)
    if ldpc_bool:
        c = code(ldpc_params["standard"], ldpc_params["rate"], ldpc_params["z"])
        L_unprotected = lengths['L_unprotected']
        unprotected_sparse_len = int(L_unprotected * M)
        protected_beta_estimate = beta_soft_estimate[unprotected_sparse_len:]
        unprotected = msg_vector_map_estimator(s, M, sqrt_nP_l)[:unprotected_sparse_len]
        unprotected_bits_out = msg_vector_2_bin_arr(unprotected, M)
        bp_probs = beta_estimate_to_bp_probs(protected_beta_estimate, L, M, sqrt_nP_l)
        _, protected_bits_out = ldpc_bp(bp_probs, c, 200, True)
        bits_out = np.concatenate((unprotected_bits_out, protected_bits_out))
    else:
        unprotected = msg_vector_map_estimator(s, M, sqrt_nP_l)
        bits_out = msg_vector_2_bin_arr(unprotected, M)
    return bits_out


def sparc_amp(y, sparc_params, decode_params, A):
    """AMP with fixed t_max iterations (sparc_new.py:885-912) on the GPU.
    Returns (beta, s)."""
    P, L, M = sparc_params['P'], sparc_params['L'], sparc_params['M']
    design = _design_for(A, P, L, M)
    beta, s = dense_amp_batch(np.asarray(y)[None, :], design, decode_params['t_max'],
                              _precision(decode_params))
    return beta[0], s[0]


def sparc_amp_single_it(sparc_params, y, A, AT, beta, z, tau_sqr):
    """One AMP iteration from a given state (sparc_new.py:975-990).  Returns
    (beta, z, tau_sqr).  Runs the same device kernels as sparc_amp."""
    P, L, M = sparc_params['P'], sparc_params['L'], sparc_params['M']
    design = _design_for(A, P, L, M)
    y = np.ascontiguousarray(y, dtype=np.float64)
    beta = np.ascontiguousarray(beta, dtype=np.float64)
    z = np.ascontiguousarray(z, dtype=np.float64)
    beta_o = np.empty_like(beta)
    z_o = np.empty_like(z)
    t2 = np.zeros(1)
    _native.check(_native.lib().sg_dense_amp_iteration(
        design.plan(_native.SG_F64), _native.ptr(y), _native.ptr(beta), _native.ptr(z), float(tau_sqr),
        _native.ptr(beta_o), _native.ptr(z_o), _native.ptr(t2)))
    return beta_o, z_o, float(t2[0])


# ------------------------------------------------------------------ estimators and glue


def msg_vector_mmse_estimator(s, tau_sqr, n, P_l, M):
    """sqrt(n P_l) softmax(sqrt(n P_l) s / tau^2) per section (sparc_new.py:1040-1066),
    softmax on the GPU (per-section maximum: same value as the global shift)."""
    x = np.sqrt(n * P_l) * (s / tau_sqr)
    if (np.any(x - x.max() >= 708)) or (np.any(x - x.max() <= -800)):
        print("Possible overflow from exponent in mmse_estimator")
    _native.require_gpu()
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    _native.check(_native.lib().sg_section_softmax(_native.ptr(x), x.size // M, M, float(np.sqrt(n * P_l)),
                                                   _native.ptr(out)))
    return out


def msg_vector_map_estimator(s, M, sqrt_nP_l):
    """sqrt(n P_l) at the argmax of each section (sparc_new.py:1099-1116), on the GPU."""
    _native.require_gpu()
    L = s.size // M
    x = np.ascontiguousarray(s, dtype=np.float64)
    idx = np.empty(L, dtype=np.int32)
    _native.check(_native.lib().sg_section_argmax(_native.ptr(x), L, M, _native.ptr(idx)))
    beta = np.zeros_like(s, dtype=float).reshape(L, -1)
    beta[np.arange(L), idx] = sqrt_nP_l
    return beta.ravel()


def _glue(beta, L, M, sqrt_nP_l, probs_only):
    _native.require_gpu()
    beta = np.ascontiguousarray(beta, dtype=np.float64)
    logM = int(np.log2(M))
    nl = beta.size // M
    out = np.empty(nl * logM)
    d_b = _native.DeviceBuffer.from_array(beta)
    d_o = _native.DeviceBuffer(out.nbytes)
    _native.check(_native.lib().sg_beta_to_llr_device(_native.SG_F64, d_b.ptr, 1, nl, M, float(sqrt_nP_l), 0, nl,
                                                      nl * logM, int(probs_only), d_o.ptr, None))
    _native.synchronize()
    return d_o.download(out)


def beta_estimate_to_bp_probs(beta, L, M, sqrt_nP_l):
    """P(bit = 0) for each MSB-first bit of each section from the AMP posterior
    (sparc_new.py:1118-1138).  L is accepted for the reference's signature; the
    section count is beta.size / M as in the reference's reshape."""
    return _glue(beta, L, M, sqrt_nP_l, True)


def S_k_mapping(M):
    """Indices whose k-th (MSB-first) bit is 0, per bit (sparc_new.py:1140-1160)."""
    logM = int(np.log2(M))
    S_k = [[] for _ in range(logM)]
    for i in range(logM):
        b = logM - 1 - i
        k = 0
        while k < M:
            for j in range(k, k + pow(2, i)):
                S_k[b].append(j)
            k = k + pow(2, i + 1)
    return S_k


def ldpc_bp(ldpc_probs, c, num_its, hard_decision_bool):
    """BP on every N-bit block of the bit probabilities (sparc_new.py:1162-1193);
    all blocks decode in one batched GPU launch (sumprod2, code.decode's default)."""
    eps = 1e-15
    ldpc_probs = np.clip(ldpc_probs, eps, 1 - eps)
    LLR = np.log(ldpc_probs) - np.log(1 - ldpc_probs)
    assert len(LLR) % c.N == 0
    blocks = LLR.reshape(-1, c.N)
    app, _ = c.decode_batch(blocks, num_its, 'sumprod2')
    if hard_decision_bool:
        hard_decision_bits = (app[:, :c.K] < 0).astype(int).ravel()
        ldpc_probs = 0
    else:
        app = app.ravel()
        ldpc_probs = (np.exp(app)) / (1 + np.exp(app))
        hard_decision_bits = 0
    return ldpc_probs, hard_decision_bits


def ldpc_bits_to_user_bits(ldpc_bits, c):
    """Systematic part of every N-bit block (sparc_new.py:1248-1258)."""
    return np.asarray(ldpc_bits).reshape(-1, c.N)[:, :c.K].ravel()


def ldpc_probs_to_user_bits(ldpc_probs, c):
    """Hard decisions on the systematic part of every block (sparc_new.py:1234-1246)."""
    return (np.asarray(ldpc_probs).reshape(-1, c.N)[:, :c.K].ravel() < 0.5).astype(int)


# ------------------------------------------------------------------ design matrix and bits


def create_design_matrix(L, M, n, rand_seed):
    """A ~ N(0, 1/n), shape (n, L*M), from default_rng(rand_seed) (sparc_new.py:1284-1294)."""
    rng = np.random.default_rng(rand_seed)
    return rng.normal(loc=0, scale=1 / np.sqrt(n), size=(n, M * L))


def bin_arr_2_msg_vector(bin_arr, M, n, P_l):
    """Bits -> message vector with value sqrt(n P_l) (sparc_new.py:1298-1317)."""
    logM = int(np.log2(M))
    bin_arr = np.asarray(bin_arr)
    assert bin_arr.size % logM == 0
    L = bin_arr.size // logM
    idx = bin_arr.reshape(L, logM).astype(np.int64) @ (1 << np.arange(logM)[::-1])
    msg_vector = np.zeros(L * M)
    msg_vector[np.arange(L) * M + idx] = np.sqrt(n * P_l)
    return msg_vector


def msg_vector_2_bin_arr(msg_vector, M):
    """Message vector -> MSB-first bits (sparc_new.py:1319-1341)."""
    assert type(msg_vector) == np.ndarray
    assert type(M) == int and M > 0
    assert msg_vector.size % M == 0
    logM = int(round(np.log2(M)))
    L = msg_vector.size // M
    idxs1, idxs2 = np.nonzero(msg_vector.reshape(L, M))
    assert np.array_equal(idxs1, np.arange(L))
    return ((idxs2[:, None] >> np.arange(logM)[::-1]) & 1).astype(bool).ravel()


def encode_ldpc(user_bits, ldpc_params, mults, unprotected_bit_len):
    """Unprotected bits followed by `mults` LDPC codewords (sparc_new.py:1343-1359)."""
    c = code(ldpc_params["standard"], ldpc_params["rate"], ldpc_params["z"])
    ldpc_bits = user_bits[unprotected_bit_len:]
    unprotected_bits = user_bits[:unprotected_bit_len].astype(bool)
    chunks = np.array_split(ldpc_bits, mults)
    enc = c.encode_batch(np.stack(chunks)) if len({len(ch) for ch in chunks}) == 1 else \
        np.stack([c.encode(ch) for ch in chunks])
    return np.concatenate((unprotected_bits, np.concatenate(list(enc)).astype(bool)))


def bin_arr_2_int(bin_array):
    """MSB-first bits -> integer (sparc_new.py:1363-1370)."""
    assert bin_array.dtype == 'bool'
    k = bin_array.size
    assert 0 < k < 64
    return bin_array.dot(1 << np.arange(k)[::-1])


def int_2_bin_arr(integer, arr_length):
    """Integer -> MSB-first bits (sparc_new.py:1372-1378), numpy-2 safe."""
    assert integer >= 0
    return ((int(integer) >> np.arange(arr_length)[::-1]) & 1).astype(bool)


def bit_err_rate(bits_in, bits_out):
    """Fraction of differing bits (sparc_new.py:1380-1388)."""
    assert len(bits_in == bits_out)
    return np.sum(bits_in != bits_out) / len(bits_in)


# ------------------------------------------------------------------ integrated AMP <-> BP decoders


def integrated_decode_batch(Y, design, c, mode, t_max, num_its=6, num_its_final=200, precision=_native.SG_F64):
    """Batched integrated decoding of received words sharing one design.
    mode: 'naive' | 'naive_posteriors' | 'integrated' | 'integrated_posteriors'.
    Returns (information bits uint8 [B, blocks*K], tau^2 [B, t_max])."""
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    if Y.ndim != 2 or Y.shape[1] != design.n:
        raise ValueError(f"received words must have shape [B, {design.n}]")
    logM = int(np.log2(design.M))
    assert (design.L * logM) % c.N == 0  # ldpc_bp (sparc_new.py:1171)
    B = Y.shape[0]
    bits = np.zeros((B, design.L * logM // c.N * c.K), dtype=np.uint8)
    tau2 = np.zeros((B, int(t_max)))
    _native.check(_native.lib().sg_integrated_decode(
        design.plan(precision), c._device_graph(), _native.INTEGRATED_MODES[mode], int(c.K), _native.ptr(Y), B,
        int(t_max), int(num_its), int(num_its_final), _native.ptr(bits), _native.ptr(tau2)))
    return bits, tau2


def _integrated(mode, y, sparc_params, ldpc_params, decode_params, A):
    P, L, M = sparc_params['P'], sparc_params['L'], sparc_params['M']
    c = code(ldpc_params["standard"], ldpc_params["rate"], ldpc_params["z"])
    design = _design_for(A, P, L, M)
    bits, _ = integrated_decode_batch(np.asarray(y)[None, :], design, c, mode, decode_params['t_max'],
                                      precision=_precision(decode_params))
    return bits[0].astype(int)


def naively_integrated_decoder(y, sparc_params, ldpc_params, decode_params, A):
    """AMP iteration, then 6 BP iterations whose output replaces beta; final
    200-iteration BP (sparc_new.py:257-282).  Returns the information bits."""
    return _integrated("naive", y, sparc_params, ldpc_params, decode_params, A)


def naively_integrated_decoder_posteriors(y, sparc_params, ldpc_params, decode_params, A):
    """As naively_integrated_decoder with beta updated by the BP posteriors
    (update_using_bp_probs) instead of replaced (sparc_new.py:411-439)."""
    return _integrated("naive_posteriors", y, sparc_params, ldpc_params, decode_params, A)


def integrated_decoder(y, sparc_params, ldpc_params, decode_params, A):
    """AMP with BP inside the denoiser and the differentiated-eta Onsager term
    (sparc_new.py:472-502)."""
    return _integrated("integrated", y, sparc_params, ldpc_params, decode_params, A)


def integrated_decoder_posteriors(y, sparc_params, ldpc_params, decode_params, A):
    """integrated_decoder with the posterior update and its derivative
    (sparc_new.py:675-705)."""
    return _integrated("integrated_posteriors", y, sparc_params, ldpc_params, decode_params, A)


def bp_output_to_beta_estimate(ldpc_probs, L, M, sqrt_nP_l):
    """Section estimate from bit probabilities: prod of p (bit 0) or 1 - p
    (bit 1) over the MSB-first bits, times sqrt(n P_l) (sparc_new.py:1260-1279)."""
    _native.require_gpu()
    p = np.ascontiguousarray(ldpc_probs, dtype=np.float64)
    logM = int(np.log2(M))
    assert p.size == L * logM
    out = np.empty(L * M)
    _native.check(_native.lib().sg_bp_output_to_beta(_native.SG_F64, _native.ptr(p), 1, int(L), int(M),
                                                     float(sqrt_nP_l), _native.ptr(out)))
    return out


def update_using_bp_probs(gamma, alpha, sqrt_nP_l, M):
    """sqrt(n P_l) (alpha gamma) normalised per section (sparc_new.py:1030-1038)."""
    _native.require_gpu()
    g = np.ascontiguousarray(gamma, dtype=np.float64)
    a = np.ascontiguousarray(alpha, dtype=np.float64)
    out = np.empty_like(a)
    _native.check(_native.lib().sg_update_using_bp_probs(_native.SG_F64, _native.ptr(g), _native.ptr(a), 1,
                                                         a.size // M, int(M), float(sqrt_nP_l), _native.ptr(out)))
    return out


def _deta(post, gamma, beta, vk, vk_0, alpha, tau_sqr, L, M, S_k, n, P_l):
    _native.require_gpu()
    if S_k is not None and [list(x) for x in S_k] != S_k_mapping(M):
        raise ValueError("S_k must be S_k_mapping(M)")
    arrs = [np.ascontiguousarray(v, dtype=np.float64) for v in (beta, alpha, vk, vk_0)]
    g = np.ascontiguousarray(gamma, dtype=np.float64) if post else None
    out = np.empty(L * M)
    t = np.array([float(tau_sqr)])
    _native.check(_native.lib().sg_differentiated_eta(
        _native.SG_F64, int(post), _native.ptr(arrs[0]), _native.ptr(g) if post else None, _native.ptr(arrs[1]),
        _native.ptr(arrs[2]), _native.ptr(arrs[3]), _native.ptr(t), 1, int(L), int(M), float(np.sqrt(n * P_l)),
        _native.ptr(out)))
    return out


def differentiated_eta_calc(beta, vk, vk_0, alpha, tau_sqr, L, M, S_k, n, P_l):
    """beta * d eta / d s of the BP-aided denoiser (sparc_new.py:824-841, sub_term
    :871-883), in closed form on the GPU."""
    return _deta(False, None, beta, vk, vk_0, alpha, tau_sqr, L, M, S_k, n, P_l)


def differentiated_eta_calc_posteriors(gamma, beta, vk, vk_0, alpha, tau_sqr, L, M, S_k, n, P_l):
    """Derivative of the posterior-updated denoiser (sparc_new.py:843-869)."""
    return _deta(True, gamma, beta, vk, vk_0, alpha, tau_sqr, L, M, S_k, n, P_l)


def eta(s, tau_sqr, n, P_l, M, L, c, num_its, num_its_final, hard_decision_bool):
    """BP-aided denoiser (sparc_new.py:709-735): returns
    (alpha, vk_0, vk, beta, hard_decision_bits)."""
    sqrt_nP_l = np.sqrt(n * P_l)
    weighted_alpha = msg_vector_mmse_estimator(s, tau_sqr, n, P_l, M)
    alpha = weighted_alpha / sqrt_nP_l
    vk_0 = beta_estimate_to_bp_probs(weighted_alpha, L, M, sqrt_nP_l)
    if hard_decision_bool:
        vk, hard_decision_bits = ldpc_bp(vk_0, c, num_its_final, True)
        beta = np.zeros(L * M)
    else:
        vk, hard_decision_bits = ldpc_bp(vk_0, c, num_its, False)
        beta = bp_output_to_beta_estimate(vk, L, M, sqrt_nP_l)
    return alpha, vk_0, vk, beta, hard_decision_bits


def eta_posteriors(s, tau_sqr, n, P_l, M, L, c, num_its, num_its_final, hard_decision_bool):
    """Posterior-updating denoiser (sparc_new.py:793-822): returns
    (alpha, vk_0, vk, beta, gamma, hard_decision_bits)."""
    sqrt_nP_l = np.sqrt(n * P_l)
    weighted_alpha = msg_vector_mmse_estimator(s, tau_sqr, n, P_l, M)
    alpha = weighted_alpha / sqrt_nP_l
    vk_0 = beta_estimate_to_bp_probs(weighted_alpha, L, M, sqrt_nP_l)
    if hard_decision_bool:
        vk, hard_decision_bits = ldpc_bp(vk_0, c, num_its_final, True)
        beta = np.zeros(L * M)
        gamma = np.zeros(L * M)
    else:
        vk, hard_decision_bits = ldpc_bp(vk_0, c, num_its, False)
        gamma = bp_output_to_beta_estimate(vk, L, M, sqrt_nP_l) / sqrt_nP_l
        beta = update_using_bp_probs(gamma, alpha, sqrt_nP_l, M)
    return alpha, vk_0, vk, beta, gamma, hard_decision_bits
