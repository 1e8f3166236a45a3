"""SPARC fixtures from the reference (sparc_public and sparc_sophie), written to
tests/golden/sparc_golden.npz and tests/golden/sophie_golden.npz.

Build-container only (imports /root/reference via ref_harness).  The hooks
wrap reference functions to record what the reference computed:
  * sparc.sub_dct       -> the row/column orders of every design block;
  * sparc.msg_vector_mmse_estimator -> per-iteration (s, tau) of the AMP loop.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402

SPARC_CASES = [
    # name, code_params, decode_params, awgn_var, seeds, traced seed index
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
TRACE_ITERS = (0, 1, 2, 4)


def make_sparc():
    ldpc, sparc, sparc_sim, _, _, _ = ref_harness.import_reference()
    out = {}
    orig_sub_dct = sparc.sub_dct
    orig_mmse = sparc.msg_vector_mmse_estimator
    for name, cp0, dp0, awgn_var, nseeds in SPARC_CASES:
        for si in range(nseeds):
            seed = [7 * si + 1, 1000 + si]
            cp, dp = dict(cp0), dict(dp0)
            orders = []

            def sub_dct_hook(m, n, seed=0, order0=None, order1=None):
                orders.append((np.array(order0, dtype=np.uint32), np.array(order1, dtype=np.uint32)))
                return orig_sub_dct(m, n, seed, order0, order1)
            trace = []

            def mmse_hook(s, tau, M, K=1):
                trace.append((np.array(s), np.array(tau, dtype=float)))
                return orig_mmse(s, tau, M, K)
            sparc.sub_dct = sub_dct_hook
            sparc.msg_vector_mmse_estimator = mmse_hook
            try:
                bits_i, beta0, x, Ab, Az = sparc.sparc_encode(cp, awgn_var, seed)
                y = sparc_sim.awgn_channel(x, awgn_var, seed)
                bits_o, beta, T, nmse, expect = sparc.sparc_decode(y, cp, dp, awgn_var, seed, beta0, Ab, Az)
            finally:
                sparc.sub_dct = orig_sub_dct
                sparc.msg_vector_mmse_estimator = orig_mmse
            L, M = cp['L'], cp['M']
            key = f"{name}_s{si}"
            out[key + "_seed"] = np.array(seed)
            out[key + "_n"] = np.array(cp['n'])
            out[key + "_R_actual"] = np.array(cp['R_actual'])
            out[key + "_bits"] = bits_i
            out[key + "_y"] = y
            out[key + "_x"] = x
            out[key + "_order0"] = np.stack([o[0] for o in orders])
            out[key + "_order1"] = np.stack([o[1] for o in orders])
            out[key + "_map"] = np.argmax(beta.reshape(L, M), axis=1).astype(np.int32)
            out[key + "_t_final"] = np.array(T)
            out[key + "_nmse"] = np.array(nmse)
            out[key + "_expect"] = np.array(bool(expect))
            out[key + "_bits_out"] = bits_o
            out[key + "_tau"] = np.array([np.asarray(tr[1]).reshape(-1)[::M][:64] for tr in trace]
                                         if np.ndim(trace[0][1]) else [tr[1] for tr in trace])
            if si == 0:
                for it in TRACE_ITERS:
                    if it < len(trace):
                        out[key + f"_s_it{it}"] = trace[it][0].astype(np.float64)
            res = sparc_sim.sparc_sim(dict(cp0), dict(dp0), awgn_var, seed)
            out[key + "_sim_ber"] = np.array(res['ber'])
            out[key + "_sim_ser"] = np.array(res['ser'])
            out[key + "_sim_t"] = np.array(res['t_final'])
            out[key + "_sim_detect"] = np.array(res['detect'])
            out[key + "_sim_nsec"] = np.array(res['num_of_sec_errs'])
            out[key + "_sim_locs"] = np.array(res['loc_of_sec_errs'])
            print(key, "n", cp['n'], "T", T, "ber", res['ber'], "blocks", len(orders))
    # bit/message-vector round trip (sparc.py:1003-1008) on fixed seeds
    for k, M in ((9216, 512), (96, 4)):
        bits = sparc.rnd_bin_arr(k, [11, 22])
        mv = sparc.bin_arr_2_msg_vector(bits, M)
        out[f"rt_{k}_{M}_bits"] = bits
        out[f"rt_{k}_{M}_idx"] = np.flatnonzero(mv).astype(np.int64)
    # base matrices
    out["pa_16"] = sparc.pa_iterative(15.0, 1.0, 16, 1.4)
    out["sc_6_32"] = sparc.sc_basic(np.array(15.0), 6, 32)
    out["scpa_2_4_q"] = sparc.sc_basic(sparc.pa_iterative(15.0, 1.0, 2, 0.96), 2, 4)
    np.savez_compressed(os.path.join(HERE, "sparc_golden.npz"), **out)
    print("wrote sparc_golden.npz", sum(v.nbytes for v in out.values()) / 1e6, "MB raw")


def make_sophie():
    ldpc, sparc, sparc_sim, sparc_new, sim_new, param_calc = ref_harness.import_reference()
    out = {}
    # dense Gaussian AMP (sparc_new.py:885-912), uncoded, small
    for si, (L, M, R) in enumerate(((16, 64, 1.0), (32, 16, 0.8))):
        sp = {'P': 15.0, 'R': R, 'L': L, 'M': M}
        seed = [3 + si, 44]
        ub, tb, beta0, x, A = sparc_new.sparc_ldpc_encode(sp, None, None, False, seed)
        y = sim_new.awgn_channel(x, 1.0, seed)
        beta, s = sparc_new.sparc_amp(y, sp, {'t_max': 25}, A)
        bits_o = sparc_new.sparc_ldpc_decode(y, sp, None, {'t_max': 25}, False, None, A)
        key = f"dense{si}"
        out[key + "_seed"] = np.array(seed)
        out[key + "_user_bits"] = ub
        out[key + "_y"] = y
        out[key + "_beta"] = beta
        out[key + "_s"] = s
        out[key + "_bits_out"] = bits_o
        print(key, "n", len(y), "ber", sparc_new.bit_err_rate(ub, bits_o))
    # AMP -> BP glue (sparc_new.py:1118-1193) with the reference c_ldpc.c sumprod2
    rng = np.random.default_rng(5)
    c = ldpc.code('802.11n', '1/2', 27)
    L, M = 72, 512  # 72*9 = 648 = N
    logit = rng.standard_normal((L, M)) * 3
    true = rng.integers(0, M, L)
    logit[np.arange(L), true] += 6
    p = np.exp(logit - logit.max(axis=1, keepdims=True))
    beta = (p / p.sum(axis=1, keepdims=True)).ravel() * 2.5
    probs = sparc_new.beta_estimate_to_bp_probs(beta, L, M, 2.5)
    _, hard = sparc_new.ldpc_bp(probs, c, 200, True)
    soft, _ = sparc_new.ldpc_bp(probs, c, 6, False)
    out["glue_beta"] = beta
    out["glue_probs"] = probs
    out["glue_hard_bits"] = hard
    out["glue_soft_probs"] = soft
    # concatenated SPARC + LDPC end to end (sparc_sim_new.py:12-23), small fully protected case
    ovr, Ls, Lsl, lengths = param_calc.param_calc(1, 6, '802.11n', '1/2', 1 / 2, 27, 1.0)
    sp_ldpc = {'P': 15.0, 'R': 1.0, 'L': Lsl, 'M': 64}
    lp = {'standard': '802.11n', 'rate': '1/2', 'z': 27, 'int_rate': 0.5, 'mults': 1}
    for si, var in enumerate((1.2, 2.0)):
        seed = [91 + si, 7]
        bi, bo, ber = sim_new.sparc_ldpc_sim(sp_ldpc, lp, lengths, True, {'t_max': 25}, var, seed)
        out[f"cat{si}_seed"] = np.array(seed)
        out[f"cat{si}_var"] = np.array(var)
        out[f"cat{si}_bits_in"] = bi
        out[f"cat{si}_bits_out"] = bo
        out[f"cat{si}_ber"] = np.array(ber)
        print("cat", si, "L", Lsl, "ber", ber)
    out["cat_lengths"] = np.array([lengths['k_ldpc'], lengths['mults'], lengths['L_unprotected']])
    out["cat_L"] = np.array(Lsl)
    # semi-protected parameter arithmetic (param_calc.py:31-58)
    r = param_calc.param_calc_semi_protected(1.5, 4, 0.8, 512, '802.11n', '1/2', 1 / 2, 81)
    out["semi_params"] = np.array([r[0], r[1], r[2], r[3]['k_ldpc'], r[3]['mults'],
                                   r[3]['L_unprotected'], r[4]], dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "sophie_golden.npz"), **out)
    print("wrote sophie_golden.npz", sum(v.nbytes for v in out.values()) / 1e6, "MB raw")


if __name__ == "__main__":
    make_sparc()
    make_sophie()
