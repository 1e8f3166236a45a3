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
events recorded on the library stream in the timed region: around every AMP
iteration of the C2 line (its four kernels; an event between two kernels holds
the second back, so the per-kernel split is taken from the last warmup step),
around every launch elsewhere.

Roofline: the C2 headline leads with the binding bound, the f32 vector ALUs
(SURVEY.md 8(d) flops per codeword-iteration; the FFTs run on the VALU), with
the HBM bound beside it; BP leads with the LDS bound (its messages never leave
LDS), HBM beside it.

CPU baseline: the CPU restatements in oracle/ (test infrastructure; here only
as the timed baseline) on one single-threaded process per host core
(oracle/cpu_pool.py, OMP_NUM_THREADS=1, core count stated), over the same
received words the GPU decoded, bounded in time (rank 0, N=1 only).  The
decisions of both are compared over the whole sample.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       N>1 without a launcher's environment: bench.py starts its N ranks
       itself (ldpc_sparc_amd.launch, one process per GPU, no PyTorch) before
       touching the GPU, and exits non-zero when fewer than N GPUs are
       visible; under torch.distributed.run the ranks meet the same way
       (ldpc_sparc_amd.rendezvous).
"""
import argparse
import json
import os
import socket
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
# FP64 vector peak: MI355X_MICROARCH.md has no FP64 row.  v_fma_f64 issues at half the f32 packed-FMA
# rate on CDNA3/CDNA4 (MI300X: 81.7 vs 163.4 TF), i.e. 157.3 / 2 = 78.6 TF, AMD's MI355X figure; the
# dependent-FMA microbenchmark tools/fp64peak.hip measures it on the box (profiles/r04_fp64peak.txt).
VALU_F64_PEAK_TFS = 78.65
VALU_F64_PEAK_SOURCE = ("157.3 TF f32 vector peak (MI355X_MICROARCH.md) / 2: v_fma_f64 at half the packed-f32 "
                        "FMA rate (AMD MI355X spec 78.6 TF FP64 vector); measured: profiles/r04_fp64peak.txt")
AMP_PHASES = ("ab_passA", "ab_passB", "az_passA", "az_passB", "eta", "control", "amp_iter")


# Restatement-to-reference speed on one host (tools/cpu_calibrate.py, run in the
# build container where the reference exists: the imported sparc_public/sparc.py
# and oracle/_ref's compile of c_ldpc.c against oracle/ on the same inputs, one
# thread each).  Quoted in every cpu_baseline so the "port" figure can be read
# as the reference's speed.
CALIB_FILE = os.path.join(REPO, "profiles", "r05_cpu_calibration.json")


def calib(key):
    try:
        with open(CALIB_FILE) as f:
            c = json.load(f)
    except (OSError, ValueError):
        return {"port_over_reference_speed": None, "source": f"{os.path.relpath(CALIB_FILE, REPO)} missing"}
    src = {"amp_r15": ("amp_r15", "port_over_reference_speed", "C2 at R=1.5"),
           "amp_r13": ("amp_r13", "port_over_reference_speed", "C2 at R=1.3"),
           "bp_minsum": ("bp", "minsum_corrected", "C3 min-sum, per iteration (the reference ships the c_ldpc.c:364 "
                                                   "defect, which never stops early)"),
           "bp_sumprod2": ("bp", "sumprod2", "C3 code, sumprod2")}[key]
    if src[0] == "bp":
        e = c["bp"][src[1]]
        r = e.get("port_over_reference_speed_per_iteration", e.get("port_over_reference_speed"))
    else:
        e = c[src[0]]
        r = e[src[1]]
    return {"port_over_reference_speed": r, "measured_on": src[2], "host": c.get("host"), "threads": 1,
            "source": os.path.relpath(CALIB_FILE, REPO) + " (tools/cpu_calibrate.py, build container: the reference "
                      "itself against the restatement on the same inputs)",
            "note": "reference speed on that host = port speed / this ratio"}


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
    ap.add_argument("--no-f64", action="store_true", help="skip the double-precision C2 companion line")
    ap.add_argument("--bp-ebn0-extra", type=float, nargs="*", default=[1.0, 1.5],
                    help="further C3 operating points (SURVEY.md 8(d): Eb/N0 1.0, 1.5, 2.0 dB)")
    ap.add_argument("--sc-batch", type=int, default=256)
    ap.add_argument("--sc-steps", type=int, default=2)
    ap.add_argument("--no-sc-notebook", action="store_true",
                    help="skip the notebook geometry (L=2048, w=2^16) spatially coupled line")
    ap.add_argument("--sc-notebook-batch", type=int, default=256)
    ap.add_argument("--concat-batch", type=int, default=256)
    ap.add_argument("--concat-steps", type=int, default=2)
    ap.add_argument("--concat-ebn0", type=float, default=5.5)
    ap.add_argument("--concat-n", type=int, default=9216,
                    help="C5 codeword length (9216: R_overall 0.58, decodable above ~5 dB Eb/N0)")
    ap.add_argument("--timed-prof-level", type=int, default=2, choices=(0, 2),
                    help="HIP-event scopes during the timed C2 steps: 2 (default) around every AMP iteration, "
                         "0 none (A/B of the events' own cost; no roofline)")
    ap.add_argument("--cpu-seconds", type=float, default=60.0,
                    help="wall-time cap of the C2 CPU-baseline sample (the other legs scale from it; 0 disables)")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="CPU-baseline processes (default: the host cores available, at most 16)")
    ap.add_argument("--rendezvous-check", action="store_true",
                    help="launch/rendezvous only (no GPU): rank 0 prints the ranks that joined")
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    ap.add_argument("--seed", type=int, default=1, help="Philox key of the synthetic inputs (stream = rank)")
    ap.add_argument("--detail-dir", default="profiles",
                    help="directory of bench_detail_<libsha>.json, the full per-configuration record")
    return ap.parse_args()


# Library knobs that change what the timed region runs (engine forcing, tuning,
# diagnostics).  A benchmark runs the shipped defaults only.
ENGINE_ENV_PREFIX = "SG_AMP_"


def guard_env():
    bad = sorted(k for k in os.environ if k.startswith(ENGINE_ENV_PREFIX))
    if bad:
        sys.stderr.write("bench.py: refusing to run with engine knobs set (%s): the benchmark measures the shipped "
                         "defaults; unset them\n" % ", ".join(bad))
        sys.exit(3)


def _visible_list(var):
    v = os.environ.get(var)
    if v is None:
        return None
    return [x for x in v.split(",") if x.strip() != ""]


def visible_gpus():
    """GPUs this process could use, counted through amdsmi (the kernel
    driver's view) without any HIP call, so the launcher parent never
    initialises the GPU: torch.cuda.device_count() goes through amdsmi too on
    this image but falls back to hipGetDeviceCount when amdsmi fails, which
    would initialise HIP here.  The *_VISIBLE_DEVICES masks narrow the count.
    If amdsmi cannot count, the launcher refuses (exit 2) rather than guess."""
    try:
        import amdsmi
        amdsmi.amdsmi_init(amdsmi.AmdSmiInitFlags.INIT_AMD_GPUS)
        try:
            n = len(amdsmi.amdsmi_get_processor_handles())
        finally:
            amdsmi.amdsmi_shut_down()
    except Exception as e:  # no driver, no library: refuse, never fall back to a HIP call
        sys.stderr.write(f"bench.py: cannot count GPUs through amdsmi ({type(e).__name__}: "
                         f"{str(e).strip().splitlines()[-1] if str(e).strip() else ''}); refusing to launch\n")
        sys.exit(2)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        lst = _visible_list(var)
        if lst is not None:
            n = min(n, len(lst))
    return n


def maybe_spawn(args):
    """--gpus N > 1 outside a launcher's environment: start N ranks of this
    script (ldpc_sparc_amd.launch, one process per GPU, no PyTorch) as child
    processes and exit with the job's code.  Nothing here touches the GPU, so
    the parent never holds GPU state while the ranks run."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != args.gpus:
            sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}\n")
            sys.exit(2)
        return
    if args.gpus <= 1:
        return
    if not args.rendezvous_check and os.environ.get("BENCH_REHEARSAL") != "1":
        ng = visible_gpus()
        if ng < args.gpus:
            sys.stderr.write(f"bench.py: --gpus {args.gpus} but only {ng} GPU(s) visible; refusing to run "
                             f"fewer ranks\n")
            sys.exit(2)
    from ldpc_sparc_amd import launch
    sys.exit(launch.spawn(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))


def rendezvous_check(d):
    """--rendezvous-check: every rank joins, barriers, and reports its rank;
    rank 0 prints the ranks that joined (CPU only, no GPU call)."""
    ranks = d.group.allgather_obj(d.rank) if d.world > 1 else [d.rank]
    d.barrier()
    if d.rank == 0:
        print(json.dumps({"rendezvous": "ok", "n_ranks": len(ranks), "ranks": sorted(ranks),
                          "world_size": d.world, "torch_loaded": "torch" in sys.modules}), flush=True)
    d.close()


class Dist:
    """The ranks of this job (ldpc_sparc_amd.rendezvous: standard-library TCP on
    the node) for rendezvous, barriers and the RCCL unique id; all GPU work,
    the counter all-reduce included, goes through libldpc_sparc_amd."""

    def __init__(self):
        from ldpc_sparc_amd.rendezvous import HostGroup
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.group = HostGroup(self.rank, self.world) if self.world > 1 else None

    def barrier(self):
        if self.group is not None:
            self.group.barrier()

    def max(self, x):
        return x if self.group is None else self.group.max(x)

    def bcast_bytes(self, b):
        return b if self.group is None else self.group.bcast_bytes(b if self.rank == 0 else b"")

    def close(self):
        if self.group is not None:
            self.group.barrier()
            self.group.close()


class HostCounterComm:
    """Counter all-reduce through the host rendezvous group: only for
    rehearsals in which several ranks share one GPU (RCCL needs one GPU per rank)."""

    def __init__(self, d):
        self.d = d

    def allreduce_sum_i64(self, dbuf, count):
        v = dbuf.download(np.zeros(count, np.int64))
        dbuf.upload(self.d.group.allreduce_sum_i64(v))

    def destroy(self):
        pass


def lib_digest():
    """sha256 prefix of the library this process runs: PMC summaries carry the
    digest of the build they were measured on (tools/pmc_bench.py,
    tools/pmc_sq_bench.py), and the bench reports their bytes and instruction
    counts only for that same build -- a kernel change that keeps its name can
    never borrow an older build's counters."""
    import hashlib
    with open(_native.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def _pmc_file(kind):
    """The newest profiles/*_pmc_{kind}_bench*.json measured on this build, or
    (None, None)."""
    import glob
    dig = lib_digest()
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_{kind}_bench*.json")),
                       key=os.path.getmtime, reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("lib_sha256") == dig:
            return d, os.path.basename(path)
    return None, None


def pmc_traffic(section, field, kernel_prefix=None):
    """HBM bytes per unit from the PMC passes of tools/pmc_bench.sh over this
    bench on this library build (FETCH_SIZE x2 + WRITE_SIZE): (value, file),
    or (None, None) when no pass of this build is committed."""
    d, name = _pmc_file("traffic")
    try:
        sec = d[section]
        if kernel_prefix and not str(sec.get("kernel", "")).startswith(kernel_prefix):
            return None, None
        return sec[field], name
    except (TypeError, KeyError):
        return None, None


def pmc_sq(section):
    """SQ counter summary (tools/pmc_sq_bench.sh) of this build: (dict, file) or (None, None)."""
    d, name = _pmc_file("sq")
    if d is None or section not in d:
        return None, None
    return d[section], name


# ------------------------------------------------------------------ AMP (C2)

def amp_setup(args, rank, rate=None):
    L, M = 1024, 512
    logM = 9
    n = int(round(L * logM / (rate or args.rate)))
    W = np.array(15.0)
    prec = _native.SG_F32 if args.precision == "f32" else _native.SG_F64
    o0, o1 = sparc.generate_ordering(W, n, L * M, 0)  # one design shared by every rank
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    tp = time.perf_counter()
    plan = op.plan(prec)  # host tables of every engine for this design (one-time, outside the timed region)
    plan_s = time.perf_counter() - tp
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
              d_cnt=_native.DeviceBuffer(4 * 8), W=W, o0=o0, o1=o1, plan_s=plan_s)
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


def amp_decodable(args, d, comm, cpu_seconds, procs):
    """SURVEY.md 8(d) C2 companion: the same engine at R=1.3 (n=7089), where AMP
    decodes in 14-18 iterations, so the BER comparison with the CPU
    restatement is made on codewords that mostly decode."""
    rate = 1.3
    st = amp_setup(args, d.rank, rate)
    a = argparse.Namespace(**{**vars(args), "rate": rate})
    amp_step(st, a, comm)
    _native.device_synchronize()
    prof = _native.Profiler(level=2)  # events around every AMP iteration, as the headline
    d.barrier()
    t0 = time.perf_counter()
    steps = max(1, args.steps // 2)
    for _ in range(steps):
        amp_step(st, a, comm)
    _native.device_synchronize()
    el = d.max(time.perf_counter() - t0)
    phases = prof.stop()
    cnt = st["d_cnt"].download(np.zeros(4, np.int64))
    tf = st["d_tf"].download(np.zeros(st["B"], np.int32))
    amp_ms = sum(phases.get(p, (0.0, 0))[0] for p in AMP_PHASES)
    w = int(st["op"].w)
    flops_per_cwit = 2 * 2.5 * w * np.log2(w) + 20 * st["L"] * st["M"]
    tfl = flops_per_cwit * int(tf.sum()) * steps / (amp_ms * 1e-3) / 1e12 if amp_ms > 0 else None
    out = {"workload": f"C2 at R={rate}: L=1024, M=512, n={st['n']}, same design family, t_max={args.t_max}",
           "value": d.world * st["B"] * steps / el, "unit": "codewords/s", "batch_per_gpu": st["B"],
           "avg_iterations": float(tf.mean()), "section_errors": int(cnt[0]), "bit_errors": int(cnt[1]),
           "codeword_errors": int(cnt[2]),
           "ber": float(cnt[1]) / (d.world * st["B"] * st["L"] * st["logM"]),
           "roofline": {"bound": "valu-f32", "achieved": tfl, "peak": VALU_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": tfl / VALU_PEAK_TFS if tfl else None,
                        "algorithmic_flops_per_codeword_iteration": flops_per_cwit,
                        "kernel_ms": {k: round(v[0], 3) for k, v in phases.items()},
                        "launches": {k: v[1] for k, v in phases.items()}}}
    if cpu_seconds > 0:
        out["cpu_baseline"] = amp_cpu_baseline(st, a, cpu_seconds, procs)
    return out


def amp_f64(args, d, comm, cpu_seconds, procs, steps=2):
    """C2 at the reference's precision: the same design and Philox batch in
    double precision (the f64 engines: the split per-codeword engine,
    amp_cw2d.hip, handing over to the staged regular engine, amp_fused.hip,
    once half the batch has stopped; the reference computes in float64 with a float128 softmax, sparc.py:429-432,
    463), with its decisions compared codeword by codeword with the CPU
    restatement on a bounded sample."""
    a = argparse.Namespace(**{**vars(args), "precision": "f64"})
    st = amp_setup(a, d.rank)
    amp_step(st, a, comm)
    _native.device_synchronize()
    prof = _native.Profiler()  # HIP events on the library stream around every kernel phase
    d.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        amp_step(st, a, comm)
    _native.device_synchronize()
    el = d.max(time.perf_counter() - t0)
    phases = prof.stop()
    cnt = st["d_cnt"].download(np.zeros(4, np.int64))
    tf = st["d_tf"].download(np.zeros(st["B"], np.int32))
    amp_ms = sum(phases.get(p, (0.0, 0))[0] for p in AMP_PHASES)
    cw_it = int(tf.sum()) * steps
    w = int(st["op"].w)
    flops_per_cwit = 2 * 2.5 * w * np.log2(w) + 20 * st["L"] * st["M"]
    tfl = flops_per_cwit * cw_it / (amp_ms * 1e-3) / 1e12 if amp_ms > 0 else None
    out = {"workload": f"C2 in double precision: L=1024, M=512, n={st['n']}, R={args.rate}, t_max={args.t_max}, "
                       "same design and batch as the f32 line",
           "value": d.world * st["B"] * steps / el, "unit": "codewords/s", "dtype": "f64",
           "batch_per_gpu": st["B"], "steps": steps, "avg_iterations": float(tf.mean()),
           "engine": {2: "split per-codeword (amp_cw2d.hip), staged after the hand-over",
                      1: "staged (amp_fused.hip)", 0: "general (amp_dct.hip)"}.get(
               _native.lib().sg_amp_plan_engine(st["plan"], st["B"]), "?"),
           "section_errors": int(cnt[0]), "bit_errors": int(cnt[1]), "codeword_errors": int(cnt[2]),
           "roofline": {"bound": "valu-f64", "achieved": tfl, "peak": VALU_F64_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": tfl / VALU_F64_PEAK_TFS if tfl else None,
                        "peak_source": VALU_F64_PEAK_SOURCE,
                        "algorithmic_flops_per_codeword_iteration": flops_per_cwit, "codeword_iterations": cw_it,
                        "kernel_ms": {k: round(v[0], 3) for k, v in phases.items()},
                        "launches": {k: v[1] for k, v in phases.items()},
                        "note": "same flop figure as the f32 line (SURVEY.md 8(d)) over the summed kernel time of "
                                "the timed steps (HIP events around every kernel phase on the library stream)"}}
    if cpu_seconds > 0:
        out["cpu_baseline"] = amp_cpu_baseline(st, a, cpu_seconds, procs)
    return out


def popcount32(a):
    a = np.asarray(a, np.uint32)
    return int(np.unpackbits(a.view(np.uint8)).sum())


def amp_cpu_baseline(st, args, seconds, procs):
    """oracle/sparc_ref.py (scipy fftpack DCT operators, float128 softmax, as
    sparc.py:883-999) on `procs` single-threaded processes over the same
    received words the GPU decoded (the whole batch unless the wall-time cap
    cuts it), with the GPU's decisions compared codeword by codeword."""
    from oracle import cpu_pool
    L, M, n, B = st["L"], st["M"], st["n"], st["B"]
    dt = np.float32 if st["prec"] == _native.SG_F32 else np.float64
    Y = st["d_y"].download(np.zeros((B, n), dt)).astype(np.float64)
    true = st["d_true"].download(np.zeros((B, L), np.int32))
    gmap = st["d_map"].download(np.zeros((B, L), np.int32))  # the GPU's decisions, same codewords
    gtf = st["d_tf"].download(np.zeros(B, np.int32))
    res, el = cpu_pool.amp_decode(procs, st["W"], L, M, n, st["o0"], st["o1"], Y, true, args.t_max, seconds)
    done = sorted(res)
    nd = len(done)
    cmap = np.stack([res[b][0] for b in done])
    ctf = np.array([res[b][1] for b in done])
    g, t = gmap[done], true[done]
    csec, gsec = (cmap != t), (g != t)
    nb = nd * L * st["logM"]
    iters = int(ctf.sum())
    # codewords outside t_final +-2 that the GPU stopped where the reference's
    # own relative psi change was within 10 % of rtol (a threshold stop)
    dtf = gtf[done] - ctf
    thr = 0
    for k, b in enumerate(done):
        if dtf[k] < -2:
            ps = res[b][3]
            tg = int(gtf[b])
            thr += int(abs(ps[tg - 1] - ps[tg - 2]) / abs(ps[tg - 2]) <= 1.1e-6)
    return {"value": nd / el, "unit": "codewords/s", "cores": procs, "kind": "port",
            "vs_reference": calib("amp_r13" if abs(args.rate - 1.3) < 1e-9 else "amp_r15"),
            "sample": f"{nd} of the {B} C2 codewords the GPU decoded (R={args.rate}, t_max={args.t_max}, {iters} AMP "
                      f"iterations, {el:.1f} s wall) by oracle/sparc_ref.py (numpy/scipy fftpack DCT, float128 "
                      f"softmax), one single-threaded process per core on {procs} host cores",
            "ber_match": {"codewords": nd,
                          "cpu_ber": popcount32(cmap ^ t) / nb, "gpu_ber": popcount32(g ^ t) / nb,
                          "cpu_ser": float(csec.mean()), "gpu_ser": float(gsec.mean()),
                          "cpu_fer": float(csec.any(1).mean()), "gpu_fer": float(gsec.any(1).mean()),
                          "identical_section_decisions": float((cmap == g).mean()),
                          "identical_codeword_decisions": float((cmap == g).all(1).mean()),
                          "t_final_equal": float((ctf == gtf[done]).mean()),
                          "t_final_max_abs_diff": int(np.abs(ctf - gtf[done]).max()),
                          "t_final_within_2": float((np.abs(dtf) <= 2).mean()),
                          "outside_2_at_reference_threshold": thr,
                          "outside_2_unexplained": int((np.abs(dtf) > 2).sum()) - thr,
                          "note": "the GPU's decisions for the same received words (f32 engine vs the f64/"
                                  "float128 CPU restatement), over every codeword of the CPU sample"}}


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


def bp_cpu_baseline(st, seconds, procs):
    """oracle/bp_oracle.c min-sum (reference c_ldpc.c:339-381 with the loop
    index corrected) on `procs` single-threaded processes, over every codeword
    the GPU decoded unless the wall-time cap cuts the sample."""
    from oracle import cpu_pool
    c = st["c"]
    gapp = st["d_app"].download(np.zeros((st["B"], c.N), np.float32))  # the GPU's output, same codewords
    git = st["d_it"].download(np.zeros(st["B"], np.int32))
    app, it, done, el = cpu_pool.bp_decode(procs, "minsum", st["ch"], c.vdeg, c.cdeg, c.intrlv, 50, 0.7,
                                           deadline_s=seconds)
    nd = int(done.sum())
    x = st["X"][done][:, :c.K]
    ch_, gh = (app[done] < 0).astype(np.int64), (gapp[done] < 0).astype(np.int64)
    ce, ge = (ch_[:, :c.K] != x), (gh[:, :c.K] != x)
    return {"value": nd / el, "unit": "codewords/s", "cores": procs, "kind": "port",
            "vs_reference": calib("bp_minsum"),
            "sample": f"{nd} of the {st['B']} C3 codewords the GPU decoded (802.11n r1/2 z=81, min-sum, 50 it, "
                      f"Eb/N0 {st.get('ebn0')} dB, {el:.1f} s wall) by oracle/bp_oracle.c, one single-threaded "
                      f"process per core on {procs} host cores",
            "ber_match": {"codewords": nd, "cpu_ber": float(ce.sum()) / (nd * c.K), "gpu_ber": float(ge.sum()) / (nd * c.K),
                          "cpu_fer": float(ce.any(1).mean()), "gpu_fer": float(ge.any(1).mean()),
                          "identical_codeword_decisions": float((ch_ == gh).all(1).mean()),
                          "identical_iteration_counts": float((it[done] == git[done]).mean()),
                          "note": "information-bit errors of the GPU (f32) and the CPU restatement (f64) on the same "
                                  "channel LLRs, over every codeword of the CPU sample"}}


def bp_variant(args, d, std, rate, z, dectype, prec, ebn0, B, steps, max_it=50, cpu_seconds=0.0, procs=1):
    """A BP line beside C3: another decoder / precision / code through the same
    batched engine, with the GPU's decisions compared to the CPU restatement
    (oracle/bp_oracle.c) on the same LLRs when cpu_seconds > 0."""
    c = code(std, rate, z)
    rng = np.random.default_rng(3000 + d.rank)
    X = c.encode_batch(rng.integers(0, 2, (B, c.K)))
    R = c.K / c.N
    s2 = 1 / (2 * R * 10 ** (ebn0 / 10))
    ch = 2 * ((1 - 2 * X) + np.sqrt(s2) * rng.standard_normal(X.shape)) / s2
    g = c._device_graph()
    dt = np.float32 if prec == _native.SG_F32 else np.float64
    d_ch = _native.DeviceBuffer.from_array(ch.astype(dt))
    d_app = _native.DeviceBuffer(B * c.N * np.dtype(dt).itemsize)
    d_it = _native.DeviceBuffer(B * 4)
    kind = _native.DECTYPES[dectype]
    lib = _native.lib()

    def step():
        _native.check(lib.sg_ldpc_decode_device(g, kind, prec, d_ch.ptr, B, max_it, 0.7, d_app.ptr, d_it.ptr, None))

    step()
    _native.device_synchronize()
    prof = _native.Profiler()
    d.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    _native.device_synchronize()
    el = d.max(time.perf_counter() - t0)
    ph = prof.stop()
    its = d_it.download(np.zeros(B, np.int32))
    app = d_app.download(np.zeros((B, c.N), dt))
    hard = (app < 0).astype(np.int64)
    fe = int((hard[:, :c.K] != X[:, :c.K]).any(1).sum())
    out = {"workload": f"{std} r{rate} z={z} (n={c.N}, max check degree {int(c.cdeg.max())}), {dectype}, "
                       f"{'f32' if prec == _native.SG_F32 else 'f64'}, max {max_it} it, Eb/N0 {ebn0} dB, random codewords",
           "value": d.world * B * steps / el, "unit": "codewords/s", "batch_per_gpu": B, "ebn0": ebn0,
           "avg_executed_iterations": float(np.where(its < max_it, its + 1, max_it).mean()),
           "frame_errors": fe, "kernel_ms_per_launch": ph.get("bp_flood", (0.0, 1))[0] / max(ph.get("bp_flood", (0, 1))[1], 1)}
    kname = c.decode_kernel(dectype, prec)
    if kname.startswith("bp_grouped") and out["kernel_ms_per_launch"] > 0:  # messages in LDS: the C3 bound
        cwit = float(np.where(its < max_it, its + 1, max_it).sum())
        lach = 16 * c.Nmsg * cwit / (out["kernel_ms_per_launch"] * 1e-3) / 1e9
        lpk = bp_lds_peak_gbs(_native.cu_count())
        out["roofline"] = {"bound": "lds", "achieved": lach, "peak": lpk, "unit": "GB/s", "frac": lach / lpk,
                           "kernel": kname}
    if cpu_seconds > 0:
        from oracle import cpu_pool
        capp, cit, done, cel = cpu_pool.bp_decode(procs, dectype, ch, c.vdeg, c.cdeg, c.intrlv, max_it, 0.7,
                                                  deadline_s=cpu_seconds)
        ch_ = (capp[done] < 0).astype(np.int64)
        out["cpu_baseline"] = {"value": int(done.sum()) / cel, "unit": "codewords/s", "cores": procs, "kind": "port",
                               "vs_reference": calib("bp_sumprod2" if dectype == "sumprod2" else "bp_minsum"),
                               "sample": f"{int(done.sum())} of the {B} codewords, oracle/bp_oracle.c on {procs} cores",
                               "identical_codeword_decisions": float((ch_ == hard[done]).all(1).mean()),
                               "identical_iteration_counts": float((cit[done] == its[done]).mean()),
                               "cpu_fer": float((ch_[:, :c.K] != X[done][:, :c.K]).any(1).mean()),
                               "gpu_fer": float((hard[done][:, :c.K] != X[done][:, :c.K]).any(1).mean())}
        cok = (ch_[:, :c.K] == X[done][:, :c.K]).all(1)  # codewords the CPU restatement decodes
        nb = int(done.sum()) * c.K
        out["cpu_baseline"].update({
            "identical_decisions_where_cpu_decodes": float((ch_[cok] == hard[done][cok]).all(1).mean())
            if cok.any() else None,
            "cpu_ber": float((ch_[:, :c.K] != X[done][:, :c.K]).sum()) / nb,
            "gpu_ber": float((hard[done][:, :c.K] != X[done][:, :c.K]).sum()) / nb,
            "note": ("the CPU restatement runs in float64; the f32 engine's hard decisions of codewords that do "
                     "not converge within max_it can differ in single bits, so 'identical_codeword_decisions' "
                     "falls below 1 at low Eb/N0 while FER and the decoded codewords agree; f32 min-sum is "
                     "bit-exact against a float32 restatement in tests/test_bp_f32_exact_gpu.py"
                     if prec == _native.SG_F32 else "f64 on both sides")})
    return out


# ------------------------------------------------------------------ spatially coupled (C4)

def sc_bench(args, d, comm, cpu_seconds, procs, L=1024, B=None, steps=None, seed_off=7):
    """C4 (BASELINE.json configs[3], sparc_demo_sc_decode_wave): spatially
    coupled SPARC, omega=6, Lambda=32 (W 37x32, 192 transforms of w=2^15),
    L=1024, M=512, R=1.5 (n=6142), P=15, sigma^2=1, t_max=40; block engine
    (amp_block.hip).  Synthetic inputs generated on the GPU as for C2."""
    M, P, omega, Lam, logM = 512, 15.0, 6, 32, 9
    W = sparc.sc_basic(np.array(P), omega, Lam)
    Lr, Lc = W.shape
    n = int(round(L * logM / args.rate))
    Mr = int(round(n / Lr))
    n = Mr * Lr
    o0, o1 = sparc.generate_ordering(W, Mr, L * M // Lc, 0)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    plan = op.plan(_native.SG_F32)
    lib = _native.lib()
    B, t_max = (B or args.sc_batch), 40
    steps = steps or args.sc_steps
    engine = {0: "general four-step (amp_dct.hip)",
              3: "block (amp_block.hip)" if int(op.w) <= 2 ** 15 else "two-class block (amp_block2.hip)"}.get(
        lib.sg_amp_plan_engine(plan, B), "?")
    d_bits = _native.DeviceBuffer(B * L * logM)
    d_true = _native.DeviceBuffer(B * L * 4)
    d_x = _native.DeviceBuffer(B * n * 4)
    d_y = _native.DeviceBuffer(B * n * 4)
    _native.check(lib.sg_rng_bits_device(args.seed + seed_off, d.rank, B, L * logM, d_bits.ptr, None))
    _native.check(lib.sg_bits_to_sections_device(d_bits.ptr, B, L, logM, d_true.ptr, None))
    _native.check(lib.sg_amp_encode_device(plan, d_true.ptr, B, d_x.ptr, None))
    _native.check(lib.sg_awgn_device(_native.SG_F32, args.seed + seed_off, d.rank, d_x.ptr, B, n, 1.0, d_y.ptr, None))
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
    for _ in range(steps):
        step()
    _native.device_synchronize()
    el = d.max(time.perf_counter() - t0)
    ph = prof.stop()
    tf = d_tf.download(np.zeros(B, np.int32))
    cnt = d_cnt.download(np.zeros(4, np.int64))
    cw_it = int(tf.sum()) * steps
    kms = sum(ph.get(k, (0.0, 0))[0] for k in AMP_PHASES)
    w = int(op.w)
    sc_traffic, sc_tfile = pmc_traffic("sc" if L == 1024 else "sc_notebook", "hbm_bytes_per_codeword_iteration")
    flops = 2 * int(np.count_nonzero(W)) * 2.5 * w * np.log2(w) + 20 * L * M  # per codeword-iteration
    ach = flops * cw_it / (kms * 1e-3) / 1e12 if kms else None
    out = {"workload": f"spatially coupled SPARC (omega=6, Lambda=32, W 37x32, 192 transforms of w=2^{int(np.log2(w))}), "
                       f"L={L}, M=512, R={args.rate} (n={n}), P=15, sigma^2=1, t_max=40",
           "engine": engine,
           "value": d.world * B * steps / el, "unit": "codewords/s", "batch_per_gpu": B,
           "avg_iterations": float(tf.mean()), "section_errors": int(cnt[0]), "codeword_errors": int(cnt[2]),
           "ser": float(cnt[0]) / (d.world * B * L),
           "roofline": {"bound": "valu-f32", "achieved": ach, "peak": VALU_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": ach / VALU_PEAK_TFS if ach else None,
                        "traffic": sc_traffic,
                        "traffic_unit": "HBM bytes per executed codeword-iteration: every dispatch of the "
                                        f"engine's decodes (PMC, profiles/{sc_tfile})",
                        "kernel": ("blk2_ab + blk_g + blk2_az + control (amp_block2.hip)" if "two-class" in engine else
                                   "blk_az (G slots inline, the next iteration's Ab fused) + control (amp_block.hip)") if "block" in engine else
                                  "general four-step kernels (amp_dct.hip)",
                        "algorithmic_flops_per_codeword_iteration": flops,
                        "algorithmic_bytes_per_codeword_iteration": 4 * (2 * L * M + 4 * n),
                        "note": "2 nT transforms x 2.5 w log2 w + 20 L M per codeword-iteration; each transform "
                                "runs in one workgroup's LDS, so HBM sees only beta, z and the tables",
                        "kernel_ms": {k: round(v[0], 3) for k, v in ph.items()},
                        "launches": {k: v[1] for k, v in ph.items()}}}
    if d.rank == 0 and d.world == 1 and cpu_seconds > 0:
        from oracle import cpu_pool
        Y = d_y.download(np.zeros((B, n), np.float32)).astype(np.float64)
        true = d_true.download(np.zeros((B, L), np.int32))
        gmap = d_map.download(np.zeros((B, L), np.int32))
        res, cel = cpu_pool.amp_decode(procs, W, L, M, n, o0, o1, Y, true, t_max, cpu_seconds)
        done = sorted(res)
        cmap = np.stack([res[b][0] for b in done])
        ctf = np.array([res[b][1] for b in done])
        out["cpu_baseline"] = {"value": len(done) / cel, "unit": "codewords/s", "cores": procs, "kind": "port",
                               "vs_reference": {**calib("amp_r15"), "measured_on": "C2 at R=1.5 (same restatement "
                                                "operators and float128 softmax; not timed on this geometry)"},
                               "sample": f"{len(done)} codewords of this geometry ({int(ctf.sum())} AMP iterations, {cel:.1f} s "
                                         "wall) decoded by oracle/sparc_ref.py (scipy fftpack DCT per block, float128 "
                                         f"softmax), one single-threaded process per core on {procs} host cores",
                               "ber_match": {"codewords": len(done),
                                             "cpu_ser": float((cmap != true[done]).mean()),
                                             "gpu_ser": float((gmap[done] != true[done]).mean()),
                                             "identical_section_decisions": float((cmap == gmap[done]).mean()),
                                             "t_final_equal": float((ctf == tf[done]).mean()),
                                             "t_final_max_abs_diff": int(np.abs(ctf - tf[done]).max())}}
    return out


# ------------------------------------------------------------------ concatenated (C5)

MFMA_F32_PEAK_TFS = 157.3  # MI355X f32 MFMA dense peak (MI355X_MICROARCH.md)


def concat_bench(args, d):
    """C5: SPARC(L=1024, M=512, dense Gaussian design shared by the batch) +
    4 x LDPC 802.11n r1/2 z=81, semi-protected (160 uncoded sections), AMP 25
    it -> glue -> sumprod2 BP 200 it, all on the device, including the batch:
    Philox user bits, the LDPC encoder and AWGN on the GPU.  n=9216 (R_overall
    0.58) decodes above ~5 dB Eb/N0, so the BER beside the throughput is a
    decoding result; the survey's n=6144 runs SPARC above capacity at every
    Eb/N0 up to 6 dB."""
    from ldpc_sparc_amd.pipeline import ConcatPipeline
    L, M, n, P, Lu, mults = 1024, 512, args.concat_n, 15.0, 160, 4
    pipe = ConcatPipeline(L, M, n, P, Lu, mults, design_seed=1234 + d.rank, precision="f32", t_max=25)
    R_overall = (Lu * 9 + mults * pipe.c.K) / n
    var = P / (2 * R_overall * 10 ** (args.concat_ebn0 / 10))
    B = args.concat_batch
    pipe.make_batch_device(B, var, 5000, d.rank)
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
    match = concat_decision_check(pipe, B, min(B, 16)) if args.cpu_seconds > 0 and d.rank == 0 else None
    gemm_ms = ph.get("dense_gemm", (0.0, 0))[0]
    concat_traffic, concat_tfile = pmc_traffic("concat", "hbm_bytes_per_gemm_launch")
    concat_mfma, _ = pmc_traffic("concat", "mfma_busy_frac")
    flops = 4.0 * n * L * M * B * (2 * 25 - 1) / 2 * args.concat_steps  # 2 n LM B per product, 49 products
    ach = flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms else None
    user_bits = Lu * 9 + mults * pipe.c.K
    return {"workload": f"C5: SPARC(L=1024, M=512, n={n}, dense Gaussian design shared by the batch) + "
                        "4 x LDPC 802.11n r1/2 z=81 semi-protected (160 uncoded sections); AMP 25 it, "
                        "glue, sumprod2 BP 200 it; batch generated on the GPU (Philox, device LDPC encoder)",
            "value": d.world * B * args.concat_steps / el, "unit": "codewords/s", "batch_per_gpu": B, "n": n,
            "ebn0_db": args.concat_ebn0, "awgn_var": var, "R_overall": R_overall,
            "ber": float(cnt[1]) / (cnt[0] * user_bits) if cnt[0] else None,
            "codeword_errors": int(cnt[2]), "codewords": int(cnt[0]),
            "decision_match": match,
            "cpu_baseline": {"value": None, "unit": "codewords/s", "cores": 0, "kind": "port",
                             "sample": "none: infeasible on the host at this size -- the reference's dense "
                                       "path (sparc_new.py:885-912, 1284-1294) holds A as a float64 "
                                       f"{n} x {L * M} matrix ({8.0 * n * L * M / 1e9:.1f} GB) and runs two "
                                       f"{2.0 * n * L * M / 1e9:.1f}-GFLOP matrix-vector products per AMP "
                                       "iteration per codeword; the pipeline's pieces are parity-tested against "
                                       "the CPU restatement at small L (tests/test_dense_gpu.py, "
                                       "tests/test_pipeline_gpu.py)"},
            "roofline": {"bound": "mfma", "achieved": ach, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": ach / MFMA_F32_PEAK_TFS if ach else None,
                         "traffic": concat_traffic,
                         "traffic_unit": "HBM bytes per GEMM launch (PMC FETCH_SIZE x2 + WRITE_SIZE, "
                                         f"profiles/{concat_tfile})" if concat_traffic else None,
                         "mfma_busy": concat_mfma,
                         "kernel": "gemm_f32_glds (A beta split-K NT + A^T z NN, v_mfma_f32_32x32x2_f32, LDS-DMA staging)",
                         "algorithmic_flops_per_batch_iteration": 4.0 * n * L * M * B,
                         "kernel_ms": {k: round(v[0], 3) for k, v in ph.items()},
                         "launches": {k: v[1] for k, v in ph.items()}}}


def concat_decision_check(pipe, B, k):
    """C5 glue + BP of the last timed decode against the CPU restatement on the
    first k codewords: bit LLRs of the protected sections recomputed in float64
    from the GPU's soft estimate (oracle/sparc_ref.beta_to_bit_probs and ldpc_bp's
    clip/log, sparc_new.py:1118-1138,1167-1169), and oracle/bp_oracle.c sumprod2
    (200 it) on the GPU's LLRs; the shipped f32 BP must take the oracle's
    decisions on every block the oracle decodes (tests/test_c5_full_gpu.py makes
    the same comparison at two Eb/N0)."""
    import ctypes as ct
    from oracle import bp as obp, sparc_ref
    c, L, M = pipe.c, pipe.L, pipe.M
    d_beta = ct.c_void_p()
    _native.check(_native.lib().sg_dense_state_device(pipe.plan, ct.byref(d_beta), None))
    _native.device_synchronize()
    beta = np.empty((k, L * M), np.float32)
    _native.check(_native.lib().sg_memcpy_d2h(_native.ptr(beta), d_beta, beta.nbytes, None))
    nb = k * pipe.mults
    llr = pipe.d_llr.download(np.empty((B * pipe.mults, c.N), np.float32))[:nb].astype(np.float64)
    app = pipe.d_app.download(np.empty((B * pipe.mults, c.N), np.float32))[:nb]
    err = 0.0
    for b in range(k):
        p = sparc_ref.beta_to_bit_probs(beta[b, pipe.L_unp * M:].astype(np.float64), L - pipe.L_unp, M, pipe.snp)
        pc = np.clip(p, 1e-15, 1 - 1e-15)
        ref = np.log(pc) - np.log(1 - pc)
        bar = 1e-5 * np.maximum(1.0, np.abs(ref)) + 4e-16 / np.minimum(pc, 1 - pc)
        err = max(err, float(np.max(np.abs(llr[b * pipe.mults:(b + 1) * pipe.mults].ravel() - ref) / bar)))
    oapp, oit = obp.decode_batch("sumprod2", llr, c.vdeg, c.cdeg, c.intrlv, pipe.bp_its)
    conv = oit < pipe.bp_its
    same = ((app < 0) == (oapp < 0)).all(axis=1)
    return {"codewords": k, "ldpc_blocks": nb, "llr_max_err_over_bar": err,
            "blocks_oracle_decodes": int(conv.sum()),
            "identical_block_decisions_where_oracle_decodes": float(same[conv].mean()) if conv.any() else None,
            "identical_block_decisions": float(same.mean()),
            "note": "LLR bar: 1e-5 x max(1, |LLR|) + the float64 conditioning of log(1 - p); oracle: "
                    "oracle/bp_oracle.c sumprod2 in float64 on the GPU's f32 LLRs"}


LDS_READ_B32 = 128   # B/clk/CU, ds_read_b32 (MI355X_MICROARCH.md LDS table)
LDS_WRITE_B32 = 64   # B/clk/CU, ds_write_b32
CLOCK_GHZ = 2.4      # max shader clock, MI355X_MICROARCH.md chip table


def bp_lds_peak_gbs(ncu):
    """LDS peak for BP's access mix: equal read and write bytes of f32 messages
    (ds_read_b32 at 128 B/clk/CU, ds_write_b32 at 64), i.e. the harmonic mean
    85.3 B/clk/CU over every CU at the maximum clock."""
    per_cu = 2.0 / (1.0 / LDS_READ_B32 + 1.0 / LDS_WRITE_B32)
    return per_cu * ncu * CLOCK_GHZ


def summary(out):
    """Compact per-configuration figures (value, unit, roofline fraction and its bound, decision match with the
    CPU restatement where the run made one), repeated at the end of the line."""
    def r(x, n=4):
        return None if x is None else float(f"{x:.{n}g}")

    def one(o, match=None):
        if not isinstance(o, dict):
            return None
        rf = o.get("roofline") or {}
        e = {"value": r(o.get("value"), 6), "frac": r(rf.get("frac")), "bound": rf.get("bound")}
        if match is not None:
            e["cpu_match"] = match
        return e

    def amp_match(o):
        bm = ((o or {}).get("cpu_baseline") or {}).get("ber_match") or {}
        return bm.get("identical_section_decisions")

    s = {"C2": one(out, amp_match(out)), "C2_R1.3": one(out.get("amp_r13"), amp_match(out.get("amp_r13"))),
         "C2_f64": one(out.get("amp_f64"), amp_match(out.get("amp_f64")))}
    bp = out.get("bp")
    if bp:
        s["C3"] = one(bp, (((bp.get("cpu_baseline") or {}).get("ber_match") or {}).get("identical_codeword_decisions")))
    for k, name in (("sc", "C4"), ("sc_notebook", "C4_notebook")):
        if out.get(k):
            s[name] = one(out[k], amp_match(out[k]))
    if out.get("concat"):
        s["C5"] = one(out["concat"], (out["concat"].get("decision_match") or {}).get(
            "identical_block_decisions_where_oracle_decodes"))
    rf = out.get("roofline") or {}
    s["C2_factors"] = {"valu_issue": r(rf.get("valu_issue_frac")), "flops_per_lane": r(rf.get("flops_per_lane_instr"))}
    return {k: v for k, v in s.items() if v is not None}


LINE_MAX_BYTES = 8192  # the driver ingests one stdout line; round 5's 23 KB line did not parse


def _r(x, n=4):
    return None if x is None else float(f"{x:.{n}g}")


def _companion(o, frac=None, traffic_ratio=None, cpu_match=None):
    """<= 150 B: value, roofline fraction, measured/algorithmic traffic, CPU decision match."""
    if not isinstance(o, dict):
        return None
    rf = o.get("roofline") or {}
    e = {"value": _r(o.get("value"), 5), "frac": _r(frac if frac is not None else rf.get("frac"), 3)}
    if traffic_ratio is not None:
        e["traffic_ratio"] = _r(traffic_ratio, 3)
    if cpu_match is not None:
        e["cpu_match"] = _r(cpu_match, 6)
    return e


def _bm(o, key):
    cb = (o or {}).get("cpu_baseline") or {}
    return (cb.get("ber_match") or cb).get(key)


def compact_line(out, detail_rel):
    """The one JSON line rank 0 prints (< LINE_MAX_BYTES): the contract keys, the
    C2 roofline and cpu_baseline, and one short entry per companion
    configuration; everything else goes to the detail file named in the line."""
    keys = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype")
    line = {k: out.get(k) for k in keys}
    cfg = out.get("config") or {}
    line["data"] = "synthetic: Philox messages, x = A beta0, AWGN sigma^2=1, generated on the GPU, resident in HBM"
    line["config"] = {k: cfg.get(k) for k in ("workload", "L", "M", "n", "R", "t_max", "batch_per_gpu",
                                               "parallelism", "counter_allreduce", "engine")}
    rf = out.get("roofline") or {}
    hb = out.get("roofline_hbm") or {}
    tr = rf.get("traffic_per_codeword_iteration")
    line["roofline"] = {
        "bound": rf.get("bound"), "achieved": _r(rf.get("achieved"), 5), "peak": rf.get("peak"),
        "unit": rf.get("unit"), "frac": _r(rf.get("frac"), 4), "traffic": _r(rf.get("traffic"), 5),
        "traffic_unit": "HBM bytes per launch (PMC of this build; 1 launch = 1 AMP iteration of the batch)",
        "traffic_over_algorithmic": _r(tr / hb["algorithmic_bytes_per_codeword_iteration"], 3)
        if (tr and hb.get("algorithmic_bytes_per_codeword_iteration")) else None,
        "valu_issue_frac": _r(rf.get("valu_issue_frac"), 3),
        "flops_per_lane_instr": _r(rf.get("flops_per_lane_instr"), 3),
        "lds_bank_conflict_frac": _r(rf.get("lds_bank_conflict_frac"), 3),
        "kernel": "cw2_ab+cw2_ctrl+cw2_az+cw2_merge (amp_cw2.hip)" if "split" in str(rf.get("engine")) else
        rf.get("kernel"),
        "algorithmic_flops_per_codeword_iteration": rf.get("algorithmic_flops_per_codeword_iteration"),
        "codeword_iterations_per_launch": _r(rf.get("codeword_iterations_per_launch"), 4),
        "hbm_frac": _r(hb.get("frac"), 3), "lib_sha256": rf.get("lib_sha256")}
    cb = out.get("cpu_baseline")
    if cb:
        bm = cb.get("ber_match") or {}
        line["cpu_baseline"] = {
            "value": _r(cb.get("value"), 4), "unit": cb.get("unit"), "cores": cb.get("cores"),
            "kind": cb.get("kind"),
            "sample": "%s of the %s C2 codewords the GPU decoded, oracle/sparc_ref.py (float128 softmax), "
                      "1 thread per core" % (bm.get("codewords"), cfg.get("batch_per_gpu")),
            "port_over_reference_speed": _r((cb.get("vs_reference") or {}).get("port_over_reference_speed"), 3),
            "ber_match": {k: _r(bm.get(k), 7) if isinstance(bm.get(k), float) else bm.get(k)
                          for k in ("codewords", "cpu_ber", "gpu_ber", "cpu_fer", "gpu_fer",
                                    "identical_section_decisions", "t_final_equal",
                                    "outside_2_at_reference_threshold", "outside_2_unexplained")}}
    else:
        line["cpu_baseline"] = None
    comp = {}

    def tratio(o):
        rr = (o or {}).get("roofline") or {}
        t, a = rr.get("traffic"), rr.get("algorithmic_bytes_per_codeword_iteration")
        return t / a if (t and a) else None

    comp["C2_R1.3"] = _companion(out.get("amp_r13"), cpu_match=_bm(out.get("amp_r13"), "identical_section_decisions"))
    comp["C2_f64"] = _companion(out.get("amp_f64"), cpu_match=_bm(out.get("amp_f64"), "identical_section_decisions"))
    bp = out.get("bp")
    if bp:
        bh = bp.get("roofline_hbm") or {}
        comp["C3"] = _companion(bp, traffic_ratio=(bh["traffic"] / bh["algorithmic_bytes_per_codeword_iteration"])
                                if bh.get("traffic") else None,
                                cpu_match=_bm(bp, "identical_codeword_decisions"))
    for i, o in enumerate(out.get("bp_ebn0") or []):
        comp["C3_%sdB" % o.get("ebn0", i)] = _companion(o, cpu_match=_bm(o, "identical_decisions_where_cpu_decodes"))
    for o, name in zip(out.get("bp_variants") or [], ("C3_sumprod2_f64", "C3_r56")):
        comp[name] = _companion(o, cpu_match=_bm(o, "identical_decisions_where_cpu_decodes"))
    for k, name in (("sc", "C4"), ("sc_notebook", "C4_notebook")):
        if out.get(k):
            comp[name] = _companion(out[k], traffic_ratio=tratio(out[k]),
                                    cpu_match=_bm(out[k], "identical_section_decisions"))
    cc = out.get("concat")
    if cc:
        cr = cc.get("roofline") or {}
        a_bytes = 4.0 * (cc.get("n") or 0) * 1024 * 512  # one pass over the f32 design matrix
        comp["C5"] = _companion(cc, traffic_ratio=cr["traffic"] / a_bytes if (cr.get("traffic") and a_bytes) else None,
                                cpu_match=(cc.get("decision_match") or {}).get(
                                    "identical_block_decisions_where_oracle_decodes"))
    line["companions"] = {k: v for k, v in comp.items() if v is not None}
    line["detail"] = detail_rel
    return line


def write_detail(out, detail_dir):
    """Full per-configuration detail (kernel times, CPU samples, notes) as
    <detail_dir>/bench_detail_<libsha>.json; returns the repo-relative path."""
    d = detail_dir if os.path.isabs(detail_dir) else os.path.join(REPO, detail_dir)
    path = os.path.join(d, f"bench_detail_{lib_digest()}.json")
    try:
        os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
    except OSError as e:
        sys.stderr.write(f"bench.py: could not write {path}: {e}\n")
    return os.path.relpath(path, REPO)


def main():
    args = parse()
    guard_env()
    maybe_spawn(args)  # --gpus N > 1 outside a launcher: re-launched as N ranks, exits
    d = Dist()
    if args.rendezvous_check:
        return rendezvous_check(d)
    _native.require_gpu()
    ndev = _native.device_count()
    if d.world > 1 and d.world > ndev and os.environ.get("BENCH_REHEARSAL") != "1":
        sys.stderr.write(f"bench.py: {d.world} ranks but {ndev} GPU(s) visible (BENCH_REHEARSAL=1 shares one GPU "
                         "with host-side counters, for rehearsals only)\n")
        sys.exit(2)
    _native.check(_native.lib().sg_set_device(d.local % max(ndev, 1)))
    comm = None
    counter_path = "none"
    rccl_ranks = 1
    if d.world > 1:
        if d.world > ndev:
            comm, counter_path = HostCounterComm(d), "host (BENCH_REHEARSAL: ranks share a GPU)"
        else:
            uid = d.bcast_bytes(_native.Comm.unique_id() if d.rank == 0 else None)
            comm, counter_path = _native.Comm(d.world, d.rank, uid), "rccl"
            rccl_ranks, dev = comm.info()
            # every rank on its own GPU: count the distinct (host, device) pairs
            obj = [tuple(x) for x in d.group.allgather_obj([socket.gethostname(), dev])]
            if len(set(obj)) != d.world or rccl_ranks != d.world:
                sys.stderr.write(f"bench.py: RCCL sees {rccl_ranks} ranks on {len(set(obj))} distinct GPUs, "
                                 f"expected {d.world}\n")
                sys.exit(2)
    procs = args.cpu_procs or 0
    if d.rank == 0 and d.world == 1 and args.cpu_seconds > 0 and not procs:
        from oracle import cpu_pool
        procs = cpu_pool.host_cores()

    st = amp_setup(args, d.rank)
    # per-kernel breakdown from the last warmup step; the timed steps bracket each AMP iteration only
    # (level 2: an event record between two kernels holds the second back by several microseconds)
    fine = {}
    for i in range(args.warmup):
        pf = _native.Profiler() if i == args.warmup - 1 else None
        amp_step(st, args, comm)
        if pf is not None:
            fine = pf.stop()
    _native.device_synchronize()
    prof = _native.Profiler(level=2 if args.warmup > 0 else 1) if args.timed_prof_level else None
    d.barrier()
    _native.device_synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        amp_step(st, args, comm)
    _native.device_synchronize()
    el = time.perf_counter() - t0
    phases = prof.stop() if prof is not None else {}
    el_max = d.max(el)
    cnt = st["d_cnt"].download(np.zeros(4, np.int64))  # last step, summed over ranks
    tf = st["d_tf"].download(np.zeros(st["B"], np.int32))
    cw_it = int(tf.sum()) * args.steps  # executed codeword-iterations on this rank
    amp_ms = sum(phases.get(p, (0.0, 0))[0] for p in AMP_PHASES)
    launches = sum(phases.get(p, (0.0, 0))[1] for p in AMP_PHASES)
    bytes_per_cwit = 4 * (2 * st["L"] * st["M"] + 4 * st["n"])
    w = int(st["op"].w)  # transform length (2^20 at C2)
    flops_per_cwit = 2 * 2.5 * w * np.log2(w) + 20 * st["L"] * st["M"]
    total_cw = d.world * st["B"] * args.steps
    # the engine this batch ran on (2: per-codeword amp_cw.hip, 1: staged amp_fused.hip)
    engine = _native.lib().sg_amp_plan_engine(st["plan"], st["B"])
    last = _native.amp_last_decode(st["plan"])
    split = max(phases.get("cw2_az", (0.0, 0))[1], fine.get("cw2_az", (0.0, 0))[1]) > 0
    engine_name = {1: "staged (amp_fused.hip)",
                   2: ("split per-codeword (amp_cw2.hip)" if split else "per-codeword (amp_cw.hip)")}.get(
        engine, str(engine))
    # rocprofv3 --pmc passes of tools/pmc_bench.sh over this bench command
    traffic, tfile = (pmc_traffic("amp", "hbm_bytes_per_codeword_iteration", "cw2_" if split else "cw_iter")
                      if engine == 2 else (None, None))
    cw_it_per_launch = cw_it / launches if launches else None
    tflops = flops_per_cwit * cw_it / (amp_ms * 1e-3) / 1e12 if amp_ms > 0 else None
    # the two factors of the f32-peak fraction from the SQ passes over this build (tools/pmc_sq_bench.sh):
    # VALU issue = wave64 VALU instructions x 4 cycles / (SIMDs x 2.4 GHz x kernel time), and algorithmic
    # flops per VALU lane-instruction (4 at most: v_pk_fma_f32); frac = issue x flops-per-lane / 4
    sq, sqfile = pmc_sq("amp") if (engine == 2 and split) else (None, None)
    vpc = sq["valu_wave_insts_per_codeword_iteration"] if sq else None
    ncu = _native.cu_count()
    valu_issue = (vpc * cw_it * 4.0 / (4 * ncu * 2.4e9 * amp_ms * 1e-3)) if (vpc and amp_ms > 0) else None
    flops_lane = flops_per_cwit / (64.0 * vpc) if vpc else None
    gbs = bytes_per_cwit * cw_it / (amp_ms * 1e-3) / 1e9 if amp_ms > 0 else None
    kernel = (("one AMP iteration of the batch = cw2_ab + cw2_ctrl + cw2_az + cw2_merge (four launches, "
               "amp_cw2.hip; 'launch' below = one iteration)") if (engine == 2 and split) else
              "cw_iter (one launch per AMP iteration of the batch)" if engine == 2 else
              "one AMP iteration = " + "+".join(AMP_PHASES[:6]))
    out = {
        "metric": METRIC,
        "value": total_cw / el_max,
        "unit": "codewords/s",
        "n_gpus": rccl_ranks if counter_path == "rccl" else d.world,
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
                   "counter_allreduce": counter_path, "rccl_ranks": rccl_ranks,
                   "engine_env": {}, "engine": engine_name,
                   "handover_iter": last["handover_iter"],
                   "plan_build_s": round(st["plan_s"], 3)},
        "roofline": {"bound": "valu-f32", "achieved": tflops, "peak": VALU_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": tflops / VALU_PEAK_TFS if tflops else None,
                     "traffic": traffic * cw_it_per_launch if (traffic and cw_it_per_launch) else None,
                     "traffic_unit": ("HBM bytes per launch (PMC FETCH_SIZE + WRITE_SIZE per codeword-iteration, "
                                      f"profiles/{tfile}, x codeword-iterations per launch)") if tfile else
                                     "no PMC pass of this library build committed (traffic null)",
                     "traffic_per_codeword_iteration": traffic,
                     "valu_issue_frac": valu_issue, "flops_per_lane_instr": flops_lane,
                     "valu_wave_insts_per_codeword_iteration": vpc,
                     "lds_bank_conflict_frac": sq.get("lds_bank_conflict_frac") if sq else None,
                     "sq_file": sqfile, "lib_sha256": lib_digest(),
                     "factor_note": "frac = valu_issue_frac x flops_per_lane_instr / 4 (SQ_INSTS_VALU of this "
                                    "build's SQ passes; issue at the nominal 2.4 GHz); null when no SQ pass of "
                                    "this build is committed",
                     "engine": engine_name, "kernel": kernel,
                     "algorithmic_flops_per_codeword_iteration": flops_per_cwit,
                     "codeword_iterations": cw_it, "codeword_iterations_per_launch": cw_it_per_launch,
                     "kernel_ms": {k: round(v[0], 3) for k, v in phases.items()},
                     "launches": {k: v[1] for k, v in phases.items()},
                     "kernel_ms_last_warmup_step": {k: round(v[0], 3) for k, v in fine.items()},
                     "launches_last_warmup_step": {k: v[1] for k, v in fine.items()},
                     "note": "binding bound: SURVEY.md 8(d) flops (2 transforms x 2.5 w log2 w + 20 L M) at the "
                             "f32 vector peak (the FFTs run on the VALU); achieved = flops x executed codeword-"
                             "iterations / summed kernel time (HIP events on the library stream around every AMP "
                             "iteration of the timed steps; the per-kernel split is from the last warmup step, "
                             "whose events also sit between the kernels)"},
        "roofline_hbm": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS if gbs else None,
                         "algorithmic_bytes_per_codeword_iteration": bytes_per_cwit,
                         "note": "SURVEY.md 8(d) 4(2LM + 4n) bytes per codeword-iteration over the same kernel time"},
        "amp": {"avg_iterations": float(tf.mean()), "section_errors": int(cnt[0]),
                "bit_errors": int(cnt[1]), "codeword_errors": int(cnt[2]),
                "ber": float(cnt[1]) / (d.world * st["B"] * st["L"] * st["logM"])},
    }

    cpu_on = d.rank == 0 and d.world == 1 and args.cpu_seconds > 0
    if not args.no_r13:
        out["amp_r13"] = amp_decodable(args, d, comm, 0.75 * args.cpu_seconds if cpu_on else 0, procs)
    if not args.no_f64 and args.precision == "f32":
        out["amp_f64"] = amp_f64(args, d, comm, 0.25 * args.cpu_seconds if cpu_on else 0, procs)

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
        cwit = exec_it.sum() * args.bp_steps
        lds_bytes = 16 * c.Nmsg  # var pass reads + writes, check pass reads + writes every f32 message
        lds_peak = bp_lds_peak_gbs(_native.cu_count())
        lach = lds_bytes * cwit / (bp_ms * 1e-3) / 1e9 if bp_ms else None
        bbytes = 4 * (4 * c.Nmsg + c.N)
        bach = bbytes * cwit / (bp_ms * 1e-3) / 1e9 if bp_ms else None
        bp_kernel = c.decode_kernel("minsum", _native.SG_F32)
        hbm_meas, bp_tfile = pmc_traffic("bp", "hbm_bytes_per_codeword_iteration", bp_kernel.split("<")[0])
        out["bp"] = {"workload": "C3: 802.11n r1/2 z=81 (n=1944), min-sum (corr 0.7), max 50 it, "
                                 f"Eb/N0 {args.bp_ebn0} dB, random codewords",
                     "value": d.world * bst["B"] * args.bp_steps / bel, "unit": "codewords/s",
                     "batch_per_gpu": bst["B"], "avg_executed_iterations": float(exec_it.mean()),
                     "frame_errors": int(bcnt[1]), "bit_errors": int(bcnt[0]),
                     "roofline": {"bound": "lds", "achieved": lach, "peak": lds_peak, "unit": "GB/s",
                                  "frac": lach / lds_peak if lach else None,
                                  "traffic": None,
                                  "kernel": bp_kernel,
                                  "algorithmic_lds_bytes_per_codeword_iteration": lds_bytes,
                                  "kernel_ms": bp_ms, "launches": ph.get("bp_flood", (0, 0))[1],
                                  "note": "the messages never leave LDS: 16 Nmsg bytes of f32 message reads and "
                                          "writes per codeword-iteration against the LDS peak for that mix "
                                          "(ds_read_b32 128 B/clk/CU, ds_write_b32 64 B/clk/CU, harmonic mean, "
                                          "2.4 GHz); SQ counters of this build: tools/pmc_sq_bench.sh"},
                     "roofline_hbm": {"bound": "hbm", "achieved_if_streamed": bach, "peak": HBM_PEAK_GBS,
                                      "unit": "GB/s", "algorithmic_bytes_per_codeword_iteration": bbytes,
                                      "traffic": hbm_meas,
                                      "traffic_unit": "measured HBM bytes per codeword-iteration (PMC, "
                                                      f"profiles/{bp_tfile})",
                                      "note": "SURVEY.md 8(d)'s figure assumes the messages stream through HBM; "
                                              "here they stay in LDS, so this bound does not bind (no frac)"}}

    if not args.no_bp and args.bp_ebn0_extra:
        # C3 at the survey's other operating points (1.0, 1.5, 2.0 dB), decisions vs the CPU
        cs = 0.1 * args.cpu_seconds if cpu_on else 0.0
        out["bp_ebn0"] = [bp_variant(args, d, "802.11n", "1/2", 81, "minsum", _native.SG_F32, e, args.bp_batch,
                                     args.bp_steps, 50, cs, procs) for e in args.bp_ebn0_extra]

    if not args.no_bp:
        cs = 0.1 * args.cpu_seconds if cpu_on else 0.0
        out["bp_variants"] = [
            bp_variant(args, d, "802.11n", "1/2", 81, "sumprod2", _native.SG_F64, 2.0, 1024, 3, 50, cs, procs),
            bp_variant(args, d, "802.11n", "5/6", 81, "minsum", _native.SG_F32, 3.5, 4096, 5, 50, cs, procs)]

    if not args.no_sc:
        out["sc"] = sc_bench(args, d, comm, 0.4 * args.cpu_seconds if cpu_on else 0, procs)
    if not args.no_sc_notebook:  # sparc_demo_sc_decode_wave.ipynb cell 1: the reference's published M=512 setup
        out["sc_notebook"] = sc_bench(args, d, comm, 0.2 * args.cpu_seconds if cpu_on else 0, procs, L=2048,
                                      B=args.sc_notebook_batch, steps=1, seed_off=9)

    if not args.no_concat:
        out["concat"] = concat_bench(args, d)

    if cpu_on:
        out["cpu_baseline"] = amp_cpu_baseline(st, args, args.cpu_seconds, procs)
        if not args.no_bp:
            out["bp"]["cpu_baseline"] = bp_cpu_baseline(bst, 0.4 * args.cpu_seconds, procs)
    out["summary"] = summary(out)
    if d.rank == 0:
        line = compact_line(out, write_detail(out, args.detail_dir))
        s = json.dumps(line, separators=(",", ":"))
        if len(s) >= LINE_MAX_BYTES:  # never print a line the driver cannot ingest
            sys.stderr.write(f"bench.py: line of {len(s)} B; dropping companions\n")
            line["companions"] = {k: {"value": v["value"]} for k, v in line["companions"].items()}
            s = json.dumps(line, separators=(",", ":"))
        print(s, flush=True)
    if comm is not None:
        comm.destroy()
    d.close()


if __name__ == "__main__":
    main()
