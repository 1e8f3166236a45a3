"""Benchmark of the AMP/BP decoding engine on MI355X.

Headline (BASELINE.json metric, configs[1] = SURVEY.md 8(d) C2): batched SPARC
AMP decoding, L=1024, M=512, regular design with the sub-sampled DCT operator
(w = 2^20), R=1.5 (n=6144), P=15, sigma^2=1, t_max=25, 256 codewords per GPU
per step.  One step = one AMP decode (reference sparc.py:883-999) of the
batch, MAP decision and device-side error counting, plus -- with more than one
GPU -- the RCCL all-reduce of the error counters.  Inputs are synthetic
(random messages encoded with the same design, AWGN) and resident in HBM
before the timed region.

Secondary (C3): batched min-sum BP on 802.11n r1/2 z=81 (n=1944), 50
iterations, 4096 codewords, reported in the "bp" object.  C4 (spatially
coupled, block engine) in the "sc" object, C5 (concatenated SPARC+LDPC) in
"concat".

Roofline: the AMP kernels of one iteration against HBM with SURVEY.md 8(d)'s
algorithmic bytes per codeword-iteration 4*(2LM+4n); the BP kernel with
4*(4*Nmsg+N) bytes per codeword-iteration.  Kernel durations come from HIP
events recorded on the library stream around every launch in the timed region.

CPU baseline: the CPU restatement in oracle/ (test infrastructure; here only as
the timed baseline) on one host core, on a bounded sample (rank 0, N=1 only).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: launched by torch.distributed.run, one process per GPU).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from ldpc_sparc_amd import _native, sparc  # noqa: E402
from ldpc_sparc_amd.ldpc import code  # noqa: E402

METRIC = "codewords/sec (AMP+BP) at L=1024 M=512 / n=1944; BER match vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
VALU_PEAK_TFS = 157.3  # MI355X f32 vector peak (packed FMA), MI355X_MICROARCH.md
AMP_PHASES = ("ab_passA", "ab_passB", "az_passA", "az_passB", "eta", "control", "amp_iter")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rate", type=float, default=1.5)
    ap.add_argument("--t-max", type=int, default=25)
    ap.add_argument("--bp-batch", type=int, default=4096)
    ap.add_argument("--bp-ebn0", type=float, default=2.0)
    ap.add_argument("--bp-steps", type=int, default=10)
    ap.add_argument("--no-bp", action="store_true")
    ap.add_argument("--no-concat", action="store_true")
    ap.add_argument("--no-sc", action="store_true")
    ap.add_argument("--no-r13", action="store_true", help="skip the decodable-rate (R=1.3) C2 companion line")
    ap.add_argument("--sc-batch", type=int, default=256)
    ap.add_argument("--sc-steps", type=int, default=2)
    ap.add_argument("--concat-batch", type=int, default=256)
    ap.add_argument("--concat-steps", type=int, default=2)
    ap.add_argument("--concat-ebn0", type=float, default=4.0)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="approximate CPU-baseline sample length (0 disables)")
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    ap.add_argument("--seed", type=int, default=1, help="Philox key of the synthetic inputs (stream = rank)")
    return ap.parse_args()


class Dist:
    """torch.distributed (gloo, CPU only) for rendezvous, barriers and the
    RCCL unique id; all GPU work goes through libldpc_sparc_amd."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo prints its peer-connection notice on stdout: keep stdout for
            # the one JSON line (the notice goes to stderr)
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, x):
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def bcast_bytes(self, b):
        if self.world == 1:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


class HostCounterComm:
    """Counter all-reduce through gloo on the host: only for rehearsals in which
    several ranks share one GPU (RCCL needs one GPU per rank)."""

    def __init__(self, d):
        self.d = d

    def allreduce_sum_i64(self, dbuf, count):
        import torch
        v = dbuf.download(np.zeros(count, np.int64))
        t = torch.from_numpy(v)
        self.d.dist.all_reduce(t)
        dbuf.upload(t.numpy())

    def destroy(self):
        pass


def pmc_traffic(section, field):
    """HBM bytes per unit from the committed PMC passes of tools/pmc_bench.sh
    (profiles/r01_pmc_traffic_bench.json), or None."""
    path = os.path.join(REPO, "profiles", "r01_pmc_traffic_bench.json")
    try:
        with open(path) as f:
            return json.load(f)[section][field]
    except (OSError, KeyError, ValueError):
        return None


# ------------------------------------------------------------------ AMP (C2)

def amp_setup(args, rank, rate=None):
    L, M = 1024, 512
    logM = 9
    n = int(round(L * logM / (rate or args.rate)))
    W = np.array(15.0)
    prec = _native.SG_F32 if args.precision == "f32" else _native.SG_F64
    o0, o1 = sparc.generate_ordering(W, n, L * M, 0)  # one design shared by every rank
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    plan = op.plan(prec)
    B = args.batch
    # throughput-mode input: Philox bits keyed by the rank
    # -> section indices -> x = A beta0 (sparc.py:51) -> AWGN, all on the GPU
    lib = _native.lib()
    es = 4 if prec == _native.SG_F32 else 8
    d_bits = _native.DeviceBuffer(B * L * logM)
    d_true = _native.DeviceBuffer(B * L * 4)
    d_x = _native.DeviceBuffer(B * n * es)
    d_y = _native.DeviceBuffer(B * n * es)
    _native.check(lib.sg_rng_bits_device(args.seed, rank, B, L * logM, d_bits.ptr, None))
    _native.check(lib.sg_bits_to_sections_device(d_bits.ptr, B, L, logM, d_true.ptr, None))
    _native.check(lib.sg_amp_encode_device(plan, d_true.ptr, B, d_x.ptr, None))
    _native.check(lib.sg_awgn_device(prec, args.seed, rank, d_x.ptr, B, n, 1.0, d_y.ptr, None))
    _native.synchronize()
    del d_bits, d_x
    st = dict(L=L, M=M, logM=logM, n=n, B=B, op=op, plan=plan, prec=prec, d_y=d_y, d_true=d_true,
              d_map=_native.DeviceBuffer(B * L * 4), d_tf=_native.DeviceBuffer(B * 4),
              d_cnt=_native.DeviceBuffer(4 * 8), W=W, o0=o0, o1=o1)
    return st


def amp_step(st, args, comm):
    lib = _native.lib()
    _native.check(lib.sg_memset(st["d_cnt"].ptr, 0, 32, None))
    _native.check(lib.sg_amp_decode_device(st["plan"], st["d_y"].ptr, st["B"], st["d_true"].ptr, 1.0,
                                           args.t_max, 1e-6, 1, st["d_map"].ptr, st["d_tf"].ptr,
                                           None, None, None))
    _native.check(lib.sg_amp_count_errors_device(st["d_map"].ptr, st["d_true"].ptr, st["d_tf"].ptr,
                                                 st["B"], st["L"], st["logM"], st["d_cnt"].ptr, None))
    if comm is not None:
        comm.allreduce_sum_i64(st["d_cnt"], 4)


def amp_decodable(args, d, comm, cpu_seconds):
    """SURVEY.md 8(d) C2 companion: the same engine at R=1.3 (n=7089), where AMP
    decodes in 14-18 iterations, so the BER comparison with the CPU
    restatement is made on codewords that mostly decode."""
    rate = 1.3
    st = amp_setup(args, d.rank, rate)
    a = argparse.Namespace(**{**vars(args), "rate": rate})
    amp_step(st, a, comm)
    _native.device_synchronize()
    d.barrier()
    t0 = time.perf_counter()
    steps = max(1, args.steps // 2)
    for _ in range(steps):
        amp_step(st, a, comm)
    _native.device_synchronize()
    el = d.max(time.perf_counter() - t0)
    cnt = st["d_cnt"].download(np.zeros(4, np.int64))
    tf = st["d_tf"].download(np.zeros(st["B"], np.int32))
    out = {"workload": f"C2 at R={rate}: L=1024, M=512, n={st['n']}, same design family, t_max={args.t_max}",
           "value": d.world * st["B"] * steps / el, "unit": "codewords/s", "batch_per_gpu": st["B"],
           "avg_iterations": float(tf.mean()), "section_errors": int(cnt[0]), "bit_errors": int(cnt[1]),
           "codeword_errors": int(cnt[2]),
           "ber": float(cnt[1]) / (d.world * st["B"] * st["L"] * st["logM"])}
    if cpu_seconds > 0:
        out["cpu_baseline"] = amp_cpu_baseline(st, a, cpu_seconds)
    return out


def amp_cpu_baseline(st, args, seconds):
    """oracle/sparc_ref.py (scipy DCT operators, float128 softmax as the
    reference) on one core, on as many codewords of the same batch as fit."""
    from oracle import sparc_ref
    L, M, n = st["L"], st["M"], st["n"]
    Ab, Az = sparc_ref.dct_operators(st["W"], L, M, n, st["o0"], st["o1"])
    # the same received words and message indices the GPU decodes
    dt = np.float32 if st["prec"] == _native.SG_F32 else np.float64
    Y = st["d_y"].download(np.zeros((st["B"], n), dt)).astype(np.float64)
    true = st["d_true"].download(np.zeros((st["B"], L), np.int32))
    gmap = st["d_map"].download(np.zeros((st["B"], L), np.int32))  # the GPU's decisions, same codewords
    t0 = time.perf_counter()
    done = iters = 0
    cbits = gbits = csec = gsec = same = 0
    while True:
        b = done
        beta0 = np.zeros(L * M)
        beta0[np.arange(L) * M + true[b]] = 1.0
        bh, tf, _, _ = sparc_ref.amp(Y[b], st["W"], L, M, n, 1.0, args.t_max, Ab, Az, beta0)
        cidx = np.argmax(bh.reshape(L, M), 1)
        cbits += int(sum(bin(int(v)).count("1") for v in (cidx ^ true[b])))
        gbits += int(sum(bin(int(v)).count("1") for v in (gmap[b] ^ true[b])))
        csec += int((cidx != true[b]).sum())
        gsec += int((gmap[b] != true[b]).sum())
        same += int((cidx == gmap[b]).sum())
        done += 1
        iters += tf
        el = time.perf_counter() - t0
        if el >= seconds or done >= st["B"]:
            break
    nb = done * L * st["logM"]
    return {"value": done / el, "unit": "codewords/s", "cores": 1, "kind": "port",
            "sample": f"{done} C2 codewords (R={args.rate}, t_max={args.t_max}, {iters} AMP "
                      f"iterations, {el:.1f} s) decoded by oracle/sparc_ref.py (numpy/scipy "
                      f"fftpack DCT, float128 softmax) on 1 host core",
            "ber_match": {"codewords": done, "cpu_ber": cbits / nb, "gpu_ber": gbits / nb,
                          "cpu_ser": csec / (done * L), "gpu_ser": gsec / (done * L),
                          "identical_section_decisions": same / (done * L),
                          "note": "the GPU's decisions for the same received words (f32 engine vs the f64/"
                                  "float128 CPU restatement)"}}


# ------------------------------------------------------------------ BP (C3)

def bp_setup(args, rank):
    c = code("802.11n", "1/2", 81)
    B = args.bp_batch
    rng = np.random.default_rng(2000 + rank)
    X = c.encode_batch(rng.integers(0, 2, (B, c.K)))
    R = c.K / c.N
    s2 = 1 / (2 * R * 10 ** (args.bp_ebn0 / 10))
    ch = 2 * ((1 - 2 * X) + np.sqrt(s2) * rng.standard_normal(X.shape)) / s2
    g = c._device_graph()
    return dict(c=c, B=B, g=g, ch=ch, X=X,
                d_ch=_native.DeviceBuffer.from_array(ch.astype(np.float32)),
                d_app=_native.DeviceBuffer(B * c.N * 4), d_it=_native.DeviceBuffer(B * 4),
                d_x=_native.DeviceBuffer.from_array(X.astype(np.uint8)),
                d_cnt=_native.DeviceBuffer(32))


def bp_step(st):
    lib = _native.lib()
    c = st["c"]
    _native.check(lib.sg_memset(st["d_cnt"].ptr, 0, 32, None))
    _native.check(lib.sg_ldpc_decode_device(st["g"], _native.SG_MINSUM, _native.SG_F32, st["d_ch"].ptr,
                                            st["B"], 50, 0.7, st["d_app"].ptr, st["d_it"].ptr, None))
    _native.check(lib.sg_ldpc_count_errors_device(st["g"], _native.SG_F32, st["d_app"].ptr, st["d_x"].ptr,
                                                  st["d_it"].ptr, st["B"], c.K, st["d_cnt"].ptr, None))


def bp_cpu_baseline(st, seconds):
    """oracle/bp_oracle.c min-sum (reference c_ldpc.c with the loop index
    corrected) on one host core."""
    from oracle import bp
    c = st["c"]
    gapp = st["d_app"].download(np.zeros((st["B"], c.N), np.float32))  # the GPU's output, same codewords
    t0 = time.perf_counter()
    done = 0
    cerr = gerr = cfe = gfe = same = 0
    while True:
        chunk = st["ch"][done:done + 64]
        app, _ = bp.decode_batch("minsum", chunk, c.vdeg, c.cdeg, c.intrlv, 50, 0.7)
        x = st["X"][done:done + len(chunk)]
        ch_, gh = (app < 0).astype(np.int64), (gapp[done:done + len(chunk)] < 0).astype(np.int64)
        cerr += int((ch_[:, :c.K] != x[:, :c.K]).sum())
        gerr += int((gh[:, :c.K] != x[:, :c.K]).sum())
        cfe += int((ch_[:, :c.K] != x[:, :c.K]).any(1).sum())
        gfe += int((gh[:, :c.K] != x[:, :c.K]).any(1).sum())
        same += int((ch_ == gh).all(1).sum())
        done += len(chunk)
        el = time.perf_counter() - t0
        if el >= seconds or done >= st["B"]:
            break
    return {"value": done / el, "unit": "codewords/s", "cores": 1, "kind": "port",
            "sample": f"{done} C3 codewords (802.11n r1/2 z=81, min-sum, 50 it, Eb/N0 "
                      f"{st.get('ebn0')} dB) by oracle/bp_oracle.c on 1 host core",
            "ber_match": {"codewords": done, "cpu_ber": cerr / (done * c.K), "gpu_ber": gerr / (done * c.K),
                          "cpu_fer": cfe / done, "gpu_fer": gfe / done,
                          "identical_codeword_decisions": same / done,
                          "note": "information-bit errors of the GPU (f32) and the CPU restatement (f64) on the same "
                                  "channel LLRs"}}


# ------------------------------------------------------------------ spatially coupled (C4)

def sc_bench(args, d, comm, cpu_seconds):
    """C4 (BASELINE.json configs[3], sparc_demo_sc_decode_wave): spatially
    coupled SPARC, omega=6, Lambda=32 (W 37x32, 192 transforms of w=2^15),
    L=1024, M=512, R=1.5 (n=6142), P=15, sigma^2=1, t_max=40; block engine
    (amp_block.hip).  Synthetic inputs generated on the GPU as for C2."""
    L, M, P, omega, Lam, logM = 1024, 512, 15.0, 6, 32, 9
    W = sparc.sc_basic(np.array(P), omega, Lam)
    Lr, Lc = W.shape
    n = int(round(L * logM / args.rate))
    Mr = int(round(n / Lr))
    n = Mr * Lr
    o0, o1 = sparc.generate_ordering(W, Mr, L * M // Lc, 0)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    plan = op.plan(_native.SG_F32)
    lib = _native.lib()
    B, t_max = args.sc_batch, 40
    d_bits = _native.DeviceBuffer(B * L * logM)
    d_true = _native.DeviceBuffer(B * L * 4)
    d_x = _native.DeviceBuffer(B * n * 4)
    d_y = _native.DeviceBuffer(B * n * 4)
    _native.check(lib.sg_rng_bits_device(args.seed + 7, d.rank, B, L * logM, d_bits.ptr, None))
    _native.check(lib.sg_bits_to_sections_device(d_bits.ptr, B, L, logM, d_true.ptr, None))
    _native.check(lib.sg_amp_encode_device(plan, d_true.ptr, B, d_x.ptr, None))
    _native.check(lib.sg_awgn_device(_native.SG_F32, args.seed + 7, d.rank, d_x.ptr, B, n, 1.0, d_y.ptr, None))
    d_map, d_tf, d_cnt = _native.DeviceBuffer(B * L * 4), _native.DeviceBuffer(B * 4), _native.DeviceBuffer(32)

    def step():
        _native.check(lib.sg_memset(d_cnt.ptr, 0, 32, None))
        _native.check(lib.sg_amp_decode_device(plan, d_y.ptr, B, d_true.ptr, 1.0, t_max, 1e-6, 1, d_map.ptr,
                                               d_tf.ptr, None, None, None))
        _native.check(lib.sg_amp_count_errors_device(d_map.ptr, d_true.ptr, d_tf.ptr, B, L, logM, d_cnt.ptr,
                                                     None))
        if comm is not None:
            comm.allreduce_sum_i64(d_cnt, 4)

    step()
    _native.device_synchronize()
    prof = _native.Profiler()
    d.barrier()
    _native.device_synchronize()
    t0 = time.perf_counter()
    for _ in range(args.sc_steps):
        step()
    _native.device_synchronize()
    el = d.max(time.perf_counter() - t0)
    ph = prof.stop()
    tf = d_tf.download(np.zeros(B, np.int32))
    cnt = d_cnt.download(np.zeros(4, np.int64))
    cw_it = int(tf.sum()) * args.sc_steps
    kms = sum(ph.get(k, (0.0, 0))[0] for k in AMP_PHASES)
    w = int(op.w)
    flops = 2 * int(np.count_nonzero(W)) * 2.5 * w * np.log2(w) + 20 * L * M  # per codeword-iteration
    ach = flops * cw_it / (kms * 1e-3) / 1e12 if kms else None
    out = {"workload": "C4: spatially coupled SPARC (omega=6, Lambda=32, W 37x32, 192 transforms of w=2^15), "
                       f"L=1024, M=512, R={args.rate} (n={n}), P=15, sigma^2=1, t_max=40",
           "value": d.world * B * args.sc_steps / el, "unit": "codewords/s", "batch_per_gpu": B,
           "avg_iterations": float(tf.mean()), "section_errors": int(cnt[0]), "codeword_errors": int(cnt[2]),
           "ser": float(cnt[0]) / (d.world * B * L),
           "roofline": {"bound": "valu-f32", "achieved": ach, "peak": VALU_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": ach / VALU_PEAK_TFS if ach else None,
                        "traffic": pmc_traffic("sc", "hbm_bytes_per_codeword_iteration_approx"),
                        "traffic_unit": "HBM bytes per codeword-iteration, block-engine kernels (PMC, "
                                        "profiles/r01_pmc_traffic_bench.json)",
                        "kernel": "blk_ab + blk_g + blk_az + control (amp_block.hip)",
                        "algorithmic_flops_per_codeword_iteration": flops,
                        "note": "2 nT transforms x 2.5 w log2 w + 20 L M per codeword-iteration; each transform "
                                "runs in one workgroup's LDS, so HBM sees only beta, z and the tables",
                        "kernel_ms": {k: round(v[0], 3) for k, v in ph.items()},
                        "launches": {k: v[1] for k, v in ph.items()}}}
    if d.rank == 0 and d.world == 1 and cpu_seconds > 0:
        from oracle import sparc_ref
        Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
        Y = d_y.download(np.zeros((B, n), np.float32)).astype(np.float64)
        true = d_true.download(np.zeros((B, L), np.int32))
        t0 = time.perf_counter()
        done = iters = 0
        while True:
            beta0 = np.zeros(L * M)
            beta0[np.arange(L) * M + true[done]] = 1.0
            _, t_f, _, _ = sparc_ref.amp(Y[done], W, L, M, n, 1.0, t_max, Ab, Az, beta0)
            done += 1
            iters += t_f
            cel = time.perf_counter() - t0
            if cel >= cpu_seconds or done >= B:
                break
        out["cpu_baseline"] = {"value": done / cel, "unit": "codewords/s", "cores": 1, "kind": "port",
                               "sample": f"{done} C4 codewords ({iters} AMP iterations, {cel:.1f} s) decoded by "
                                         "oracle/sparc_ref.py (scipy fftpack DCT per block, float128 softmax) "
                                         "on 1 host core"}
    return out


# ------------------------------------------------------------------ concatenated (C5)

MFMA_F32_PEAK_TFS = 157.3  # MI355X f32 MFMA dense peak (MI355X_MICROARCH.md)


def concat_bench(args, d):
    """C5: SPARC(L=1024, M=512, n=6144, dense Gaussian design shared by the
    batch) + 4 x LDPC 802.11n r1/2 z=81, semi-protected (160 uncoded sections),
    AMP 25 it -> glue -> sumprod2 BP 200 it, all on the device."""
    from ldpc_sparc_amd.pipeline import ConcatPipeline
    L, M, n, P, Lu, mults = 1024, 512, 6144, 15.0, 160, 4
    pipe = ConcatPipeline(L, M, n, P, Lu, mults, design_seed=1234 + d.rank, precision="f32", t_max=25)
    R_overall = (Lu * 9 + mults * pipe.c.K) / n
    var = P / (2 * R_overall * 10 ** (args.concat_ebn0 / 10))
    B = args.concat_batch
    pipe.make_batch(B, var, np.random.default_rng(5000 + d.rank))
    pipe.reset_counts()
    pipe.decode()  # warmup
    _native.device_synchronize()
    pipe.reset_counts()
    prof = _native.Profiler()
    d.barrier()
    _native.device_synchronize()
    t0 = time.perf_counter()
    for _ in range(args.concat_steps):
        pipe.decode()
    _native.device_synchronize()
    el = d.max(time.perf_counter() - t0)
    ph = prof.stop()
    cnt = pipe.counts()
    gemm_ms = ph.get("dense_gemm", (0.0, 0))[0]
    flops = 4.0 * n * L * M * B * (2 * 25 - 1) / 2 * args.concat_steps  # 2 n LM B per product, 49 products
    ach = flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms else None
    user_bits = Lu * 9 + mults * pipe.c.K
    return {"workload": "C5: SPARC(L=1024, M=512, n=6144, dense Gaussian design shared by the batch) + "
                        "4 x LDPC 802.11n r1/2 z=81 semi-protected (160 uncoded sections); AMP 25 it, "
                        "glue, sumprod2 BP 200 it",
            "value": d.world * B * args.concat_steps / el, "unit": "codewords/s", "batch_per_gpu": B,
            "ebn0_db": args.concat_ebn0, "awgn_var": var, "R_overall": R_overall,
            "ber": float(cnt[1]) / (cnt[0] * user_bits) if cnt[0] else None,
            "codeword_errors": int(cnt[2]), "codewords": int(cnt[0]),
            "roofline": {"bound": "mfma", "achieved": ach, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": ach / MFMA_F32_PEAK_TFS if ach else None, "traffic": None,
                         "kernel": "gemm_f32_mfma (A beta split-K NT + A^T z NN, v_mfma_f32_32x32x2_f32)",
                         "algorithmic_flops_per_batch_iteration": 4.0 * n * L * M * B,
                         "kernel_ms": {k: round(v[0], 3) for k, v in ph.items()},
                         "launches": {k: v[1] for k, v in ph.items()}}}


def main():
    args = parse()
    d = Dist()
    _native.require_gpu()
    ndev = _native.device_count()
    _native.check(_native.lib().sg_set_device(d.local % max(ndev, 1)))
    comm = None
    counter_path = "none"
    if d.world > 1:
        if d.world > ndev and os.environ.get("BENCH_FORCE_RCCL") != "1":
            comm, counter_path = HostCounterComm(d), "gloo (ranks share a GPU: rehearsal only)"
        else:
            uid = d.bcast_bytes(_native.Comm.unique_id() if d.rank == 0 else None)
            comm, counter_path = _native.Comm(d.world, d.rank, uid), "rccl"

    st = amp_setup(args, d.rank)
    for _ in range(args.warmup):
        amp_step(st, args, comm)
    _native.device_synchronize()
    prof = _native.Profiler()
    d.barrier()
    _native.device_synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        amp_step(st, args, comm)
    _native.device_synchronize()
    el = time.perf_counter() - t0
    phases = prof.stop()
    el_max = d.max(el)
    cnt = st["d_cnt"].download(np.zeros(4, np.int64))  # last step, summed over ranks
    tf = st["d_tf"].download(np.zeros(st["B"], np.int32))
    cw_it = int(tf.sum()) * args.steps  # executed codeword-iterations on this rank
    amp_ms = sum(phases.get(p, (0.0, 0))[0] for p in AMP_PHASES)
    bytes_per_cwit = 4 * (2 * st["L"] * st["M"] + 4 * st["n"])
    w = int(st["op"].w)  # transform length (2^20 at C2)
    flops_per_cwit = 2 * 2.5 * w * np.log2(w) + 20 * st["L"] * st["M"]
    achieved = bytes_per_cwit * cw_it / (amp_ms * 1e-3) / 1e9 if amp_ms > 0 else None
    total_cw = d.world * st["B"] * args.steps
    # the engine this batch ran on (2: per-codeword amp_cw.hip, 1: staged amp_fused.hip)
    engine = _native.lib().sg_amp_plan_engine(st["plan"], st["B"])
    engine_name = {1: "staged (amp_fused.hip)", 2: "per-codeword (amp_cw.hip)"}.get(engine, str(engine))
    traffic = None
    tfile = "r01_pmc_traffic_amp_c2_cw.json" if engine == 2 else "r01_pmc_traffic_amp_c2.json"
    tpath = os.path.join(REPO, "profiles", tfile)
    if os.path.exists(tpath):  # rocprofv3 --pmc passes of tools/pmc_traffic.py (same engine, B=256)
        with open(tpath) as f:
            traffic = json.load(f)["hbm_bytes_per_codeword_iteration"]
    out = {
        "metric": METRIC,
        "value": total_cw / el_max,
        "unit": "codewords/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * el_max / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if st["prec"] == _native.SG_F32 else "f64",
        "data": "synthetic: Philox random messages (stream = rank), encoded x = A beta0 with the benchmark "
                "design and AWGN sigma^2=1 on the GPU (throughput mode), resident in HBM before timing",
        "config": {"workload": "C2: SPARC AMP, regular design, sub-sampled DCT operator w=2^20",
                   "L": st["L"], "M": st["M"], "n": st["n"], "R": args.rate, "P": 15.0,
                   "awgn_var": 1.0, "t_max": args.t_max, "batch_per_gpu": st["B"],
                   "parallelism": f"mc-shard x{d.world} (independent codewords per GPU, "
                                  "RCCL all-reduce of error counters)",
                   "counter_allreduce": counter_path},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                     "traffic_unit": "HBM bytes per codeword-iteration (PMC FETCH_SIZE*2 + WRITE_SIZE, "
                                     f"profiles/{tfile})",
                     "engine": engine_name,
                     "kernel": ("cw_iter (one launch per AMP iteration)" if engine == 2 else
                                "one AMP iteration = " + "+".join(AMP_PHASES[:6])),
                     "algorithmic_bytes_per_codeword_iteration": bytes_per_cwit,
                     "codeword_iterations": cw_it,
                     "kernel_ms": {k: round(v[0], 3) for k, v in phases.items()},
                     "launches": {k: v[1] for k, v in phases.items()}},
        "roofline_flops": {"bound": "valu-f32", "achieved": flops_per_cwit * cw_it / (amp_ms * 1e-3) / 1e12
                           if amp_ms > 0 else None, "peak": VALU_PEAK_TFS, "unit": "TFLOP/s",
                           "frac": flops_per_cwit * cw_it / (amp_ms * 1e-3) / 1e12 / VALU_PEAK_TFS
                           if amp_ms > 0 else None,
                           "algorithmic_flops_per_codeword_iteration": flops_per_cwit,
                           "note": "SURVEY.md 8(d): 2 transforms x 2.5 w log2 w + 20 L M; the FFTs run on the "
                                   "vector ALUs (packed f32), so the f32 vector peak applies"},
        "amp": {"avg_iterations": float(tf.mean()), "section_errors": int(cnt[0]),
                "bit_errors": int(cnt[1]), "codeword_errors": int(cnt[2]),
                "ber": float(cnt[1]) / (d.world * st["B"] * st["L"] * st["logM"])},
    }

    if not args.no_r13:
        out["amp_r13"] = amp_decodable(args, d, comm, args.cpu_seconds / 2 if d.world == 1 and d.rank == 0 else 0)

    if not args.no_bp:
        bst = bp_setup(args, d.rank)
        bst["ebn0"] = args.bp_ebn0
        for _ in range(2):
            bp_step(bst)
        _native.device_synchronize()
        prof = _native.Profiler()
        d.barrier()
        _native.device_synchronize()
        t0 = time.perf_counter()
        for _ in range(args.bp_steps):
            bp_step(bst)
        _native.device_synchronize()
        bel = d.max(time.perf_counter() - t0)
        ph = prof.stop()
        its = bst["d_it"].download(np.zeros(bst["B"], np.int32))
        bcnt = bst["d_cnt"].download(np.zeros(4, np.int64))
        c = bst["c"]
        exec_it = np.where(its < 50, its + 1, 50)  # executed iterations per codeword
        bp_ms = ph.get("bp_flood", (0.0, 0))[0]
        bbytes = 4 * (4 * c.Nmsg + c.N)
        bach = bbytes * exec_it.sum() * args.bp_steps / (bp_ms * 1e-3) / 1e9 if bp_ms else None
        out["bp"] = {"workload": "C3: 802.11n r1/2 z=81 (n=1944), min-sum (corr 0.7), max 50 it, "
                                 f"Eb/N0 {args.bp_ebn0} dB, random codewords",
                     "value": d.world * bst["B"] * args.bp_steps / bel, "unit": "codewords/s",
                     "batch_per_gpu": bst["B"], "avg_executed_iterations": float(exec_it.mean()),
                     "frame_errors": int(bcnt[1]), "bit_errors": int(bcnt[0]),
                     "roofline": {"bound": "hbm", "achieved": bach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": bach / HBM_PEAK_GBS if bach else None,
                                  "traffic": pmc_traffic("bp", "hbm_bytes_per_codeword_iteration"),
                                  "traffic_unit": "HBM bytes per codeword-iteration (PMC, messages stay in LDS; "
                                                  "profiles/r01_pmc_traffic_bench.json)",
                                  "kernel": "bp_flood_kernel<float, minsum>",
                                  "algorithmic_bytes_per_codeword_iteration": bbytes,
                                  "kernel_ms": bp_ms, "launches": ph.get("bp_flood", (0, 0))[1]}}

    if not args.no_sc:
        out["sc"] = sc_bench(args, d, comm, args.cpu_seconds / 2 if d.world == 1 else 0)

    if not args.no_concat:
        out["concat"] = concat_bench(args, d)

    if d.rank == 0 and d.world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = amp_cpu_baseline(st, args, args.cpu_seconds)
        if not args.no_bp:
            out["bp"]["cpu_baseline"] = bp_cpu_baseline(bst, args.cpu_seconds / 3)
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.destroy()
    d.close()


if __name__ == "__main__":
    main()
