"""C2 divergence trace.

Decodes the bench's C2 batch (bench.amp_setup: Philox seed 1, rank 0, R=1.5
or --rate) with the shipped f32 engine, then re-decodes it with t_max = T for
T = 2 .. t_max to record psi after every iteration (the decode is
deterministic, so the state after iteration T-2 of a run with t_max = T is
the state of the full run).  The CPU restatement (oracle/sparc_ref.amp,
float128 softmax: sparc.py:883-999) decodes the same received words with a
trace of psi.  For every codeword whose t_final differs by more than 2, and for
a few that agree, it writes the two psi trajectories, the relative change
|psi_t - psi_(t-1)| / psi_(t-1) that the stop rule compares with rtol
(sparc.py:984-986), and the f64 GPU engine's t_final of the same codeword.

Output: one JSON document (stdout or --out).  Test infrastructure: the oracle
is imported only as the checker.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rate", type=float, default=1.5)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--t-max", type=int, default=25)
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import bench
    from ldpc_sparc_amd import _native, sparc
    from oracle import cpu_pool, sparc_ref

    _native.require_gpu()
    args = argparse.Namespace(batch=256, rate=a.rate, precision="f32", seed=a.seed, t_max=a.t_max)
    st = bench.amp_setup(args, 0)
    L, M, n, B = st["L"], st["M"], st["n"], st["B"]
    lib = _native.lib()
    Y = st["d_y"].download(np.zeros((B, n), np.float32)).astype(np.float64)
    true = st["d_true"].download(np.zeros((B, L), np.int32))

    d_psi = _native.DeviceBuffer(B * 8)

    def gpu_decode(tm):
        lib_ok = lib.sg_amp_decode_device(st["plan"], st["d_y"].ptr, B, st["d_true"].ptr, 1.0, tm, 1e-6, 1,
                                          st["d_map"].ptr, st["d_tf"].ptr, None, d_psi.ptr, None)
        _native.check(lib_ok)
        _native.device_synchronize()
        return (st["d_map"].download(np.zeros((B, L), np.int32)), st["d_tf"].download(np.zeros(B, np.int32)),
                d_psi.download(np.zeros(B, np.float64)))

    gmap, gtf, _ = gpu_decode(a.t_max)
    psi_gpu = np.full((B, a.t_max), np.nan)
    for tm in range(2, a.t_max + 1):
        _, tf_t, ps = gpu_decode(tm)
        # after a run with t_max = tm, psi is the value after iteration min(t_final, tm - 1)
        psi_gpu[:, tm - 1] = ps
    res, el = cpu_pool.amp_decode(cpu_pool.host_cores(a.procs), st["W"], L, M, n, st["o0"], st["o1"], Y, true,
                                  a.t_max)
    ctf = np.array([res[b][1] for b in range(B)])
    cmap = np.stack([res[b][0] for b in range(B)])
    diff = np.abs(ctf - gtf)
    out = {"rate": a.rate, "n": n, "B": B, "t_max": a.t_max, "cpu_seconds": el,
           "t_final_hist_diff": {str(k): int(v) for k, v in zip(*np.unique(ctf - gtf, return_counts=True))},
           "identical_section_decisions": float((cmap == gmap).mean()),
           "identical_codeword_decisions": float((cmap == gmap).all(1).mean()),
           "cpu_fer": float((cmap != true).any(1).mean()), "gpu_fer": float((gmap != true).any(1).mean()),
           "cpu_ser": float((cmap != true).mean()), "gpu_ser": float((gmap != true).mean()),
           "codewords": []}
    outl = [int(b) for b in np.nonzero(diff > 2)[0]]
    agree = [int(b) for b in np.nonzero(diff == 0)[0][:2]]
    Ab, Az = sparc_ref.dct_operators(st["W"], L, M, n, st["o0"], st["o1"])
    op64 = sparc.DesignOperator(st["W"], L, M, n, st["o0"], st["o1"])
    for b in outl + agree:
        tr = []
        beta0 = np.zeros(L * M)
        beta0[np.arange(L) * M + true[b]] = 1.0
        sparc_ref.amp(Y[b], st["W"], L, M, n, 1.0, a.t_max, Ab, Az, beta0,
                      trace=lambda t, d: tr.append(float(d["psi"])))
        pc = np.array(tr)
        pg = psi_gpu[b, 1:1 + len(pc)]
        m64, t64, _, _ = sparc.amp_decode_batch(Y[b:b + 1], op64, 1.0, a.t_max, true_idx=true[b:b + 1],
                                                precision=_native.SG_F64)
        rel = lambda p: [None] + [float(abs(p[i] - p[i - 1]) / abs(p[i - 1])) for i in range(1, len(p))]
        out["codewords"].append({
            "b": b, "outlier": b in outl, "gpu_t_final": int(gtf[b]), "cpu_t_final": int(ctf[b]),
            "gpu_f64_t_final": int(t64[0]), "gpu_f64_same_decisions_as_cpu": bool(np.array_equal(m64[0], cmap[b])),
            "decoded_cpu": bool(np.array_equal(cmap[b], true[b])), "decoded_gpu": bool(np.array_equal(gmap[b], true[b])),
            "same_sections": float((cmap[b] == gmap[b]).mean()),
            "psi_cpu": pc.tolist(), "psi_gpu_f32": [float(x) for x in pg],
            "psi_rel_diff": [float(abs(x - y) / abs(y)) for x, y in zip(pg, pc)],
            "dpsi_rel_cpu": rel(pc), "dpsi_rel_gpu": rel(pg)})
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(s)


if __name__ == "__main__":
    main()
