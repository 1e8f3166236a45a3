"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the AMP <-> BP integrated
decoders of sparc_sophie/sparc_new.py.

Follows, function by function:
  * bp_output_to_beta_estimate  sparc_new.py:1260-1279 (same product order)
  * update_using_bp_probs       sparc_new.py:1030-1038
  * differentiated_eta_calc     sparc_new.py:824-841 with sub_term :871-883,
    and differentiated_eta_calc_posteriors :843-869, in closed form: for
    q in S_k (the indices whose MSB-first bit k is 0) sub_term sums
    alpha_q c (delta_qi - alpha_i), i.e. c alpha_i ([i in S_k] - A_lk) with
    A_lk = sum_{q in S_k} alpha_lq and c = sqrt(n P_l) / tau^2;
  * ldpc_bp                     sparc_new.py:1162-1193 (sumprod2 through the
    C restatement oracle/bp_oracle.c)
  * naively_integrated_decoder  :257-282, naively_integrated_decoder_posteriors
    :411-439, integrated_decoder :472-502, integrated_decoder_posteriors
    :675-705, with eta :709-735 and eta_posteriors :793-822.

Pinned against tests/golden/integrated_golden.npz (made by running the
reference, tests/golden/make_golden_integrated.py) in tests/test_oracle_pin.py.
Used only by tests/ as the checker.  Never imported by the product.
"""
import numpy as np

from . import bp as bp_oracle
from .sparc_ref import beta_to_bit_probs, dense_mmse_estimator

MODES = ("naive", "naivepost", "integ", "integpost")


def _bits_msb(M):
    logM = int(np.log2(M))
    j = np.arange(M)
    return np.stack([(j >> (logM - 1 - k)) & 1 for k in range(logM)], axis=1)  # [M][logM]


def bp_output_to_beta(probs, L, M, sqrt_nP_l):
    """sparc_new.py:1260-1279: prod_j (p_j if bit j of i is 0 else 1 - p_j), MSB first, times sqrt(n P_l)."""
    logM = int(np.log2(M))
    p = probs.reshape(L, logM)
    bits = _bits_msb(M)
    amp = np.ones((L, M))
    for j in range(logM):  # the reference's left-to-right product
        amp = amp * np.where(bits[None, :, j] == 0, p[:, j:j + 1], 1 - p[:, j:j + 1])
    return amp.reshape(L * M) * sqrt_nP_l


def update_using_bp_probs(gamma, alpha, sqrt_nP_l, M):
    """sparc_new.py:1030-1038."""
    top = alpha * gamma
    bot = top.reshape(-1, M).sum(axis=1).repeat(M)
    return sqrt_nP_l * (top / bot)


def _main_term(vk, vk_0, alpha, tau_sqr, L, M, n, P_l):
    logM = int(np.log2(M))
    a = alpha.reshape(L, M)
    bits = _bits_msb(M)
    c = np.sqrt(n * P_l) / tau_sqr
    A = np.stack([a[:, bits[:, k] == 0].sum(axis=1) for k in range(logM)], axis=1)  # [L][logM]
    v = np.clip(vk_0.reshape(L, logM), 1e-10, 1 - 1e-10)
    w = 1 / (v * (1 - v))
    vks = vk.reshape(L, logM)
    mt = np.zeros((L, M))
    for k in range(logM):
        zero = bits[None, :, k] == 0
        sub = w[:, k:k + 1] * (c * a * (zero.astype(float) - A[:, k:k + 1]))
        mt = mt + np.where(zero, (1 - vks[:, k:k + 1]) * sub, -vks[:, k:k + 1] * sub)
    return mt.reshape(L * M)


def differentiated_eta(beta, vk, vk_0, alpha, tau_sqr, L, M, n, P_l):
    """sparc_new.py:824-841."""
    return beta * _main_term(vk, vk_0, alpha, tau_sqr, L, M, n, P_l)


def differentiated_eta_posteriors(gamma, beta, vk, vk_0, alpha, tau_sqr, L, M, n, P_l):
    """sparc_new.py:843-869."""
    snp = np.sqrt(n * P_l)
    mt = _main_term(vk, vk_0, alpha, tau_sqr, L, M, n, P_l)
    alpha_dash = alpha * (snp / tau_sqr) * (1 - alpha)
    gamma_dash = gamma * mt
    top = alpha * gamma
    bot = top.reshape(-1, M).sum(axis=1).repeat(M)
    top_dash = (alpha_dash * gamma) + (alpha * gamma_dash)
    bot_dash = top_dash.reshape(-1, M).sum(axis=1).repeat(M)
    return (snp * ((top_dash * bot) - (top * bot_dash))) / (bot ** 2)


def ldpc_bp(probs, graph, N, K, num_its, hard):
    """sparc_new.py:1162-1193 with sumprod2: returns P(bit=0) (soft) or the
    information bits app[:K] < 0 of every block (hard)."""
    p = np.clip(probs, 1e-15, 1 - 1e-15)
    llr = (np.log(p) - np.log(1 - p)).reshape(-1, N)
    app, _ = bp_oracle.decode_batch("sumprod2", llr, *graph, max_it=num_its)
    if hard:
        return (app[:, :K] < 0).astype(np.uint8).ravel()
    app = app.ravel()
    return np.exp(app) / (1 + np.exp(app))


def decode(mode, y, A, P, L, M, graph, N, K, t_max, num_its=6, num_its_final=200):
    """The four integrated decoders (MODES) on one codeword; returns
    (information bits, [tau^2 per iteration])."""
    n = len(y)
    P_l = P / L
    snp = np.sqrt(n * P_l)
    AT = A.T
    taus = []
    if mode in ("naive", "naivepost"):  # :257-282 / :411-439
        beta = np.zeros(L * M)
        z = 0
        tau_sqr = 1
        for i in range(t_max):
            Ab = np.dot(A, beta)  # sparc_amp_single_it :975-990
            ons = (z / tau_sqr) * (P - ((np.sum(beta ** 2)) / n))
            z = y - Ab + ons
            s = beta + np.dot(AT, z)
            tau_sqr = np.sum(z ** 2) / n
            beta = dense_mmse_estimator(s, tau_sqr, n, P_l, M)
            taus.append(tau_sqr)
            probs = beta_to_bit_probs(beta, L, M, snp)
            if i != t_max - 1:
                probs = ldpc_bp(probs, graph, N, K, num_its, False)
                old = bp_output_to_beta(probs, L, M, snp)
                if mode == "naive":
                    beta = old
                else:
                    beta = update_using_bp_probs(old / snp, beta / snp, snp, M)
            else:
                return ldpc_bp(probs, graph, N, K, num_its_final, True), taus
    beta = np.zeros(L * M)  # :472-502 / :675-705
    z = 0
    deta_sum = 0.0
    for t in range(t_max):
        if t != 0:
            if mode == "integ":
                deta_sum = np.sum(differentiated_eta(beta, vk, vk_0, alpha, tau_sqr, L, M, n, P_l))
            else:
                deta_sum = np.sum(differentiated_eta_posteriors(gamma, beta, vk, vk_0, alpha, tau_sqr, L, M, n, P_l))
        if mode == "integ":
            z = y - (np.dot(A, beta)) + (z / n) * deta_sum
        else:
            z = y - (np.dot(A, beta)) + z * (deta_sum / n)
        s = np.dot(AT, z) + beta
        tau_sqr = np.sum(z ** 2) / n
        taus.append(tau_sqr)
        weighted_alpha = dense_mmse_estimator(s, tau_sqr, n, P_l, M)  # eta :709-735
        alpha = weighted_alpha / snp
        vk_0 = beta_to_bit_probs(weighted_alpha, L, M, snp)
        if t == t_max - 1:
            return ldpc_bp(vk_0, graph, N, K, num_its_final, True), taus
        vk = ldpc_bp(vk_0, graph, N, K, num_its, False)
        if mode == "integ":
            beta = bp_output_to_beta(vk, L, M, snp)
        else:  # eta_posteriors :793-822
            gamma = bp_output_to_beta(vk, L, M, snp) / snp
            beta = update_using_bp_probs(gamma, alpha, snp, M)
