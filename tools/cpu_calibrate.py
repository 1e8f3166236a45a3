"""Calibrate the CPU baselines against the reference itself (build container only).

bench.py's cpu_baseline legs time the CPU restatements in oracle/ ("port"), not
the reference, because the reference does not exist on the GPU box.  This
script times both on the SAME host, single-threaded, on the same inputs, and
writes the restatement-to-reference speed ratio that bench.py quotes in every
cpu_baseline note (profiles/r05_cpu_calibration.json):

  * AMP (C2 family): the reference's own sparc_public/sparc.py sparc_decode
    (sparc.py:55-74 -> sparc_amp :883-999, float128 softmax; imported through
    tests/golden/ref_harness.py with its numpy-2 shims) against
    oracle/sparc_ref.amp on the same received words y and the same design
    orders (captured from the reference's sub_dct, sparc.py:648), L=1024,
    M=512, P=15, sigma^2=1, t_max=25, at R=1.5 (n=6144) and R=1.3 (n=7089);
    the decisions and t_final of both are compared.
  * BP (C3 code, 802.11n r1/2 z=81, Eb/N0 2 dB, 50 iterations, the channel
    LLRs of bench.py bp_setup): the reference's c_ldpc.c compiled from its
    source (oracle/_ref/libc_ldpc_ref.so) against oracle/bp_oracle.c, one
    codeword per ctypes call as the reference's ldpc.code.decode makes it
    (ldpc.py:463-490): sumprod2 (c_ldpc.c:234-292) both sides, and min-sum
    (c_ldpc.c:339-381) with the reference's loop-index defect both sides
    (or_minsum_refbug) plus the corrected min-sum the bench times.  Results are
    compared (bit-identical / same iteration counts expected).

Run: OMP_NUM_THREADS=1 python tools/cpu_calibrate.py [--amp-codewords 4] [--bp-codewords 512]
"""
import argparse
import json
import os
import platform
import sys
import time

for _v in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS", "NUMEXPR_NUM_THREADS"):
    os.environ[_v] = "1"

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

import ref_harness  # noqa: E402
from oracle import bp as obp, sparc_ref  # noqa: E402


def cpu_name():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def amp_case(R, ncw, t_max=25):
    _, sparc, sparc_sim, _, _, _ = ref_harness.import_reference()
    L, M, P, awgn_var = 1024, 512, 15.0, 1.0
    orig_sub_dct = sparc.sub_dct
    t_ref = t_port = 0.0
    it_ref = it_port = 0
    same_map = same_tf = 0
    rows = []
    for k in range(ncw):
        seed = [11 + k, 2025]
        cp, dp = {'P': P, 'R': R, 'L': L, 'M': M}, {'t_max': t_max}
        orders = []

        def hook(m, n, seed=0, order0=None, order1=None):
            orders.append((np.array(order0), np.array(order1)))
            return orig_sub_dct(m, n, seed, order0, order1)
        sparc.sub_dct = hook
        try:
            bits_i, beta0, x, Ab, Az = sparc.sparc_encode(cp, awgn_var, seed)
        finally:
            sparc.sub_dct = orig_sub_dct
        y = sparc_sim.awgn_channel(x, awgn_var, seed)
        n = cp['n']
        # the reference's decode (what sparc_sim.py:179-204 times per codeword)
        t0 = time.perf_counter()
        bits_o, beta, T, nmse, _ = sparc.sparc_decode(y, cp, dp, awgn_var, seed, beta0, Ab, Az)
        t1 = time.perf_counter()
        o0, o1 = orders[0]
        pAb, pAz = sparc_ref.dct_operators(np.array(P), L, M, n, o0, o1)
        t2 = time.perf_counter()
        bm, tf, _, _ = sparc_ref.amp(y, np.array(P), L, M, n, awgn_var, t_max, pAb, pAz, beta0)
        t3 = time.perf_counter()
        rmap = np.argmax(np.asarray(beta).reshape(L, M), 1)
        pmap = np.argmax(bm.reshape(L, M), 1)
        same_map += int(np.array_equal(rmap, pmap))
        same_tf += int(int(T) == int(tf))
        t_ref += t1 - t0
        t_port += t3 - t2
        it_ref += int(T)
        it_port += int(tf)
        rows.append({"seed": seed, "t_final_ref": int(T), "t_final_port": int(tf), "ref_s": round(t1 - t0, 3),
                     "port_s": round(t3 - t2, 3), "same_decisions": bool(np.array_equal(rmap, pmap))})
        print(f"  AMP R={R} codeword {k}: reference {t1 - t0:.2f} s ({T} it), restatement {t3 - t2:.2f} s ({tf} it), "
              f"same decisions {np.array_equal(rmap, pmap)}", flush=True)
    return {"workload": f"L={L}, M={M}, n={n}, R={R}, P={P}, sigma^2={awgn_var}, t_max={t_max}, {ncw} codewords",
            "reference": "sparc_public/sparc.py sparc_decode (imported, numpy-2 shims of tests/golden/ref_harness.py)",
            "port": "oracle/sparc_ref.amp (+ MAP) on the reference's y and design orders",
            "reference_codewords_per_s": ncw / t_ref, "port_codewords_per_s": ncw / t_port,
            "reference_s_per_iteration": t_ref / it_ref, "port_s_per_iteration": t_port / it_port,
            "port_over_reference_speed": (ncw / t_port) / (ncw / t_ref),
            "port_over_reference_speed_per_iteration": (t_ref / it_ref) / (t_port / it_port),
            "identical_decisions": same_map, "identical_t_final": same_tf, "codewords": ncw, "per_codeword": rows}


def bp_case(ncw, ebn0=2.0, max_it=50, reps=3):
    from ldpc_sparc_amd.ldpc import code
    c = code("802.11n", "1/2", 81)
    rng = np.random.default_rng(2000)  # bench.py bp_setup, rank 0
    X = c.encode_batch(rng.integers(0, 2, (ncw, c.K)))
    R = c.K / c.N
    s2 = 1 / (2 * R * 10 ** (ebn0 / 10))
    ch = 2 * ((1 - 2 * X) + np.sqrt(s2) * rng.standard_normal(X.shape)) / s2
    v, cd, il = c.vdeg, c.cdeg, c.intrlv
    out = {"workload": f"802.11n r1/2 z=81 (n={c.N}), Eb/N0 {ebn0} dB, {max_it} iterations, {ncw} codewords "
                       f"(bench.py bp_setup's LLRs), one codeword per ctypes call, best of {reps} passes"}

    def run(kind, use_ref):
        best = None
        for _ in range(reps):
            apps, its = [], []
            t0 = time.perf_counter()
            for b in range(ncw):
                a, i = obp.decode(kind, ch[b], v, cd, il, max_it, 0.7, use_ref=use_ref)
                apps.append(a)
                its.append(i)
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        return np.array(apps), np.array(its), best

    for label, pk, rk in (("sumprod2", "sumprod2", "sumprod2"), ("minsum_shipped", "minsum_refbug", "minsum_refbug")):
        pa, pi, pt = run(pk, False)
        ra, ri, rt = run(rk, True)
        out[label] = {"reference_codewords_per_s": ncw / rt, "port_codewords_per_s": ncw / pt,
                      "port_over_reference_speed": rt / pt, "codeword_iterations": int(ri.sum()),
                      "identical_iteration_counts": float((pi == ri).mean()),
                      "app_bit_identical": bool(np.array_equal(pa.view(np.uint64), ra.view(np.uint64)))}
        print(f"  BP {label}: reference {ncw / rt:.0f} cw/s, restatement {ncw / pt:.0f} cw/s, "
              f"ratio {rt / pt:.3f}, identical app {out[label]['app_bit_identical']}", flush=True)
    ma, mi, mt = run("minsum", False)
    ra, ri, rt = run("minsum_refbug", True)
    out["minsum_corrected"] = {"port_codewords_per_s": ncw / mt, "reference_shipped_minsum_codewords_per_s": ncw / rt,
                               "port_over_reference_speed": rt / mt,
                               "codeword_iterations_port": int(mi.sum()), "codeword_iterations_reference": int(ri.sum()),
                               "port_over_reference_speed_per_iteration": (rt / ri.sum()) / (mt / mi.sum()),
                               "note": "the bench times the corrected min-sum (c_ldpc.c:364 loop index fixed); the "
                                       "reference ships the defective loop, so the work per codeword differs: "
                                       "compare per iteration"}
    print(f"  BP minsum corrected: {ncw / mt:.0f} cw/s vs the reference's shipped min-sum {ncw / rt:.0f} cw/s "
          f"(per iteration ratio {out['minsum_corrected']['port_over_reference_speed_per_iteration']:.3f})", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--amp-codewords", type=int, default=4)
    ap.add_argument("--bp-codewords", type=int, default=512)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r05_cpu_calibration.json"))
    a = ap.parse_args()
    res = {"what": "restatement (oracle/, what bench.py's cpu_baseline times) against the reference itself, "
                   "same host, one thread each, same inputs (tools/cpu_calibrate.py)",
           "host": cpu_name(), "threads": 1}
    res["bp"] = bp_case(a.bp_codewords)
    res["amp_r15"] = amp_case(1.5, a.amp_codewords)
    res["amp_r13"] = amp_case(1.3, a.amp_codewords)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({"amp_r15": res["amp_r15"]["port_over_reference_speed"],
                      "amp_r13": res["amp_r13"]["port_over_reference_speed"],
                      "bp_sumprod2": res["bp"]["sumprod2"]["port_over_reference_speed"],
                      "bp_minsum_shipped": res["bp"]["minsum_shipped"]["port_over_reference_speed"],
                      "bp_minsum_corrected_per_iteration":
                          res["bp"]["minsum_corrected"]["port_over_reference_speed_per_iteration"]}))


if __name__ == "__main__":
    main()
