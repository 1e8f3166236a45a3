"""Monte-Carlo error-rate campaigns sharded over GPUs.

The reference parallelises only by launching independent processes with a
`sim_id` (ldpc_jossy/py/ldpc_awgn.py:125-131, ldpc_jossy/README.md:144-148).
Here one process per GPU runs a campaign together: every SNR point is split
into fixed blocks of codewords, block b being seeded by (seed, point, b) so
that the result does not depend on how many GPUs took part; each round the
blocks are dealt to ranks by contiguous ranges, and ONE all-reduce of an int64
counter vector (RCCL over xGMI between GPUs, or the host rendezvous group of
rendezvous.py for CPU tests) gives every
rank the global counts that drive the stopping rule.

Counters per point: [units, bit_errors, frame_errors, aux0, aux1] where aux
is decoder-specific (BP: executed iterations; AMP: section errors, AMP
iterations; concatenated: unprotected / protected bit errors).

Checkpoint/resume: with `checkpoint_dir`, the global counters
and next block of every point are written after each round; a restarted
campaign continues from there.
"""
import json
import os

import numpy as np

from . import _native

NC = 5


def shard_range(total, rank, world):
    """[start, end) of rank's share of `total` items (contiguous, balanced)."""
    return total * rank // world, total * (rank + 1) // world


class Aggregator:
    """Sum of int64 counter vectors over the ranks of a campaign: RCCL between
    GPUs (`comm`, a `_native.Comm`), or the host rendezvous group for CPU
    rehearsals (`group`, a `rendezvous.HostGroup`)."""

    def __init__(self, backend="none", comm=None, group=None):
        if backend not in ("none", "host", "rccl"):
            raise ValueError(f"Aggregator backend {backend!r}: one of none, host, rccl")
        if backend == "host" and group is None:
            raise ValueError("the host backend needs a rendezvous group")
        if backend == "rccl" and comm is None:
            raise ValueError("the rccl backend needs a communicator (_native.Comm)")
        self.backend = backend
        self.comm = comm
        self.group = group
        self._dbuf = None

    def allreduce(self, counts):
        counts = np.ascontiguousarray(counts, dtype=np.int64)
        if self.backend == "none":
            return counts.copy()
        if self.backend == "host":
            return self.group.allreduce_sum_i64(counts)
        if self._dbuf is None or self._dbuf.nbytes < counts.nbytes:
            self._dbuf = _native.DeviceBuffer(counts.nbytes)
        self._dbuf.upload(counts)
        self.comm.allreduce_sum_i64(self._dbuf, counts.size)
        _native.synchronize()
        return self._dbuf.download(np.empty_like(counts))


def _ckpt_path(checkpoint_dir, tag, point):
    return os.path.join(checkpoint_dir, f"{tag}_pt{point}.json")


def _first_reaching(cum, need):
    """Index of the first entry of the running count `cum` that reaches
    `need`, or None."""
    hit = np.nonzero(cum >= need)[0]
    return int(hit[0]) if hit.size else None


# Campaign parameters added to the checkpoints after round 3, with the value
# an older checkpoint implies: such a checkpoint still resumes when the new
# run uses that value (concat_ber_sweep's min_errors None).
_LEGACY_PARAM_DEFAULTS = {"min_errors": None}


def run_point(trial, point, *, block, blocks_per_round, rank, world, agg, min_errors=None, max_units=None,
              checkpoint_dir=None, tag="campaign", params=None, max_rounds=None):
    """Run one point until `min_errors` frame errors or `max_units` units
    (globally).  trial(point, first_block, n_blocks, block) -> int64[NC]
    counters of the blocks [first_block, first_block + n_blocks).

    A trial with `per_unit = True` returns int64[n_blocks * block, NC] (one
    row per codeword, in block order) instead; the round's rows of every rank
    are then combined by the same single all-reduce (each rank fills its own
    rows of a zero matrix), and the point stops exactly at the codeword where
    the frame-error count reaches `min_errors` or the unit count reaches
    `max_units`, in block order -- the stopping rule of ldpc_awgn.sim
    (ldpc_awgn.py:86-105), whatever the number of ranks.

    `params` (campaign parameters) is stored in the checkpoint; resuming with
    different parameters raises ValueError instead of adding up counts of
    different experiments.  `max_rounds` ends this call after that many rounds
    without marking the point done (an interrupted run; the checkpoint lets a
    later call continue it)."""
    total = np.zeros(NC, dtype=np.int64)
    next_block = 0
    done = False
    params = dict(params or {}, block=int(block))
    if checkpoint_dir:
        path = _ckpt_path(checkpoint_dir, tag, point)
        if os.path.exists(path):
            with open(path) as f:
                st = json.load(f)
            want = json.loads(json.dumps(params))
            for k, v in _LEGACY_PARAM_DEFAULTS.items():  # checkpoints written before the key existed
                if k not in st.get("params", {}) and want.get(k, v) == v:
                    want.pop(k, None)
            if st.get("params") != want:
                raise ValueError(f"checkpoint {path} was written with parameters {st.get('params')}, "
                                 f"not {params}: use another checkpoint_dir or tag")
            total = np.array(st["counts"], dtype=np.int64)
            next_block = int(st["next_block"])
            done = bool(st.get("done", False))
    per_unit = getattr(trial, "per_unit", False)
    rounds = 0
    while not done:
        if max_rounds is not None and rounds >= max_rounds:
            break
        rounds += 1
        if min_errors is not None and total[2] >= min_errors:
            break
        if max_units is not None and total[0] >= max_units:
            break
        nb = blocks_per_round
        if max_units is not None:
            nb = min(nb, -(-(max_units - int(total[0])) // block))
        a, b = shard_range(nb, rank, world)
        if per_unit:
            rows = np.zeros((nb * block, NC), dtype=np.int64)
            if b > a:
                rows[a * block:b * block] = trial(point, next_block + a, b - a, block)
            rows = agg.allreduce(rows.ravel()).reshape(nb * block, NC)  # the one collective per round
            cut = len(rows)
            if min_errors is not None:
                k = _first_reaching(total[2] + np.cumsum(rows[:, 2]), min_errors)
                if k is not None:
                    cut, done = min(cut, k + 1), True
            if max_units is not None and total[0] + cut >= max_units:
                cut, done = max_units - int(total[0]), True
            total = total + rows[:cut].sum(axis=0)
        else:
            local = trial(point, next_block + a, b - a, block) if b > a else np.zeros(NC, dtype=np.int64)
            total = total + agg.allreduce(local)  # the campaign's one collective per round
        next_block += nb
        if checkpoint_dir and rank == 0:
            os.makedirs(checkpoint_dir, exist_ok=True)
            tmp = _ckpt_path(checkpoint_dir, tag, point) + ".tmp"
            with open(tmp, "w") as f:
                json.dump({"counts": total.tolist(), "next_block": next_block, "done": done,
                           "params": params}, f)
            os.replace(tmp, _ckpt_path(checkpoint_dir, tag, point))
        if min_errors is None and max_units is None:
            break
    return total


# ------------------------------------------------------------------ LDPC over BPSK/AWGN


class LdpcTrial:
    """Random codewords over BPSK/AWGN at Es/N0 = snr dB (ldpc_awgn.py:39-56),
    decoded in batches on the GPU; counts over all N bits as the reference
    does (ldpc_awgn.py:97-104).  aux0 = sum of decode iteration counts."""

    def __init__(self, c, snrs, dectype="sumprod2", max_it=200, corr=0.7, precision="f32", seed=0, rng="host",
                 per_unit=False):
        self.c, self.snrs, self.dectype = c, list(snrs), dectype
        self.per_unit = bool(per_unit)  # per-codeword counter rows (exact stopping rule, run_point)
        self.max_it, self.corr, self.seed = int(max_it), float(corr), int(seed)
        self.prec = {"f64": _native.SG_F64, "f32": _native.SG_F32}[precision]
        if rng not in ("host", "device"):
            raise ValueError("rng must be 'host' (numpy, reproducible against the reference's generators) "
                             "or 'device' (Philox on the GPU, throughput mode)")
        self.rng = rng

    def _device_batch(self, point, first_block, n_blocks, block, sigma2):
        """Information bits, encoding, BPSK and noise on the GPU; Philox stream
        (point, block) so the draw does not depend on the rank or the batching."""
        c, lib, off = self.c, _native.lib(), _native.offset
        B = n_blocks * block
        es = 8 if self.prec == _native.SG_F64 else 4
        d_info = _native.DeviceBuffer(B * c.K)
        d_x = _native.DeviceBuffer(B * c.N)
        d_ch = _native.DeviceBuffer(B * c.N * es)
        for i, blk in enumerate(range(first_block, first_block + n_blocks)):
            sid = (int(point) << 32) | int(blk)
            o = i * block
            _native.check(lib.sg_rng_bits_device(self.seed, sid, block, c.K, off(d_info.ptr, o * c.K), None))
            c.encode_device(off(d_info.ptr, o * c.K), block, off(d_x.ptr, o * c.N))
            _native.check(lib.sg_bpsk_awgn_llr_device(self.prec, self.seed, sid, off(d_x.ptr, o * c.N), block, c.N,
                                                      sigma2, off(d_ch.ptr, o * c.N * es), None))
        return d_x, d_ch, B

    def __call__(self, point, first_block, n_blocks, block):
        c = self.c
        sigma2 = 1.0 / np.power(10, self.snrs[point] / 10.0)
        if self.rng == "device":
            d_x, d_ch, B = self._device_batch(point, first_block, n_blocks, block, sigma2)
            return self._decode_count(d_x, d_ch, B)
        X, LLR = [], []
        for blk in range(first_block, first_block + n_blocks):
            rng = np.random.default_rng([self.seed, point, blk])
            x = c.encode_batch(rng.integers(0, 2, (block, c.K)))
            y = (1.0 - 2.0 * x) + np.sqrt(sigma2) * rng.standard_normal(x.shape)
            X.append(x)
            LLR.append(2.0 / sigma2 * y)
        X = np.concatenate(X)
        LLR = np.concatenate(LLR)
        B = X.shape[0]
        dt = np.float64 if self.prec == _native.SG_F64 else np.float32
        d_ch = _native.DeviceBuffer.from_array(LLR.astype(dt))
        d_x = _native.DeviceBuffer.from_array(X.astype(np.uint8))
        return self._decode_count(d_x, d_ch, B)

    def _decode_count(self, d_x, d_ch, B):
        c, lib = self.c, _native.lib()
        dt = np.float64 if self.prec == _native.SG_F64 else np.float32
        g = c._device_graph()
        d_app = _native.DeviceBuffer(B * c.N * np.dtype(dt).itemsize)
        d_it = _native.DeviceBuffer(B * 4)
        _native.check(lib.sg_ldpc_decode_device(g, _native.DECTYPES[self.dectype], self.prec, d_ch.ptr, B,
                                                self.max_it, self.corr, d_app.ptr, d_it.ptr, None))
        if self.per_unit:  # one row per codeword: [1, bit errors, frame error, iterations, 0]
            d_be = _native.DeviceBuffer(B * 4)
            _native.check(lib.sg_ldpc_codeword_errors_device(g, self.prec, d_app.ptr, d_x.ptr, B, d_be.ptr, None))
            _native.synchronize()
            be = d_be.download(np.zeros(B, np.int32)).astype(np.int64)
            it = d_it.download(np.zeros(B, np.int32)).astype(np.int64)
            return np.stack([np.ones(B, np.int64), be, (be > 0).astype(np.int64), it, np.zeros(B, np.int64)], 1)
        d_cnt = _native.DeviceBuffer(32)
        d_cnt.zero()
        _native.check(lib.sg_ldpc_count_errors_device(g, self.prec, d_app.ptr, d_x.ptr, d_it.ptr, B, c.K,
                                                      d_cnt.ptr, None))
        _native.synchronize()
        cnt = d_cnt.download(np.zeros(4, np.int64))
        return np.array([B, cnt[0], cnt[1], cnt[3], 0], dtype=np.int64)


class SparcTrial:
    """Regular SPARC with the sub-sampled DCT design over AWGN, generated and
    decoded on the GPU (throughput mode): Philox bits ->
    section indices -> x = A beta0 (sparc.py:17-53) -> y = x + N(0, awgn_var)
    (sparc_sim.py:179-204) -> AMP (sparc.py:883-999) -> errors.  Counters
    [codewords, bit errors, codeword errors, AMP iterations, section errors];
    the Philox stream of block b at point p is (p, b), so results do not
    depend on the rank count.  op: sparc.DesignOperator (shared design)."""

    def __init__(self, op, awgn_vars, t_max=25, rtol=1e-6, phi_method=1, precision="f32", seed=0):
        self.op, self.vars = op, list(awgn_vars)
        self.t_max, self.rtol, self.phi = int(t_max), float(rtol), int(phi_method)
        self.prec = {"f64": _native.SG_F64, "f32": _native.SG_F32}[precision]
        self.seed = int(seed)
        self.logM = int(np.log2(op.M))

    def __call__(self, point, first_block, n_blocks, block):
        op, lib, off = self.op, _native.lib(), _native.offset
        L, n, logM = op.L, op.n, self.logM
        es = 8 if self.prec == _native.SG_F64 else 4
        B = n_blocks * block
        plan = op.plan(self.prec)
        d_bits = _native.DeviceBuffer(B * L * logM)
        d_true = _native.DeviceBuffer(B * L * 4)
        d_x = _native.DeviceBuffer(B * n * es)
        d_y = _native.DeviceBuffer(B * n * es)
        sigma = float(np.sqrt(self.vars[point]))
        for i, blk in enumerate(range(first_block, first_block + n_blocks)):
            sid = (int(point) << 32) | int(blk)
            o = i * block
            _native.check(lib.sg_rng_bits_device(self.seed, sid, block, L * logM, off(d_bits.ptr, o * L * logM), None))
        _native.check(lib.sg_bits_to_sections_device(d_bits.ptr, B, L, logM, d_true.ptr, None))
        _native.check(lib.sg_amp_encode_device(plan, d_true.ptr, B, d_x.ptr, None))
        for i, blk in enumerate(range(first_block, first_block + n_blocks)):
            sid = (int(point) << 32) | int(blk)
            o = i * block
            _native.check(lib.sg_awgn_device(self.prec, self.seed, sid, off(d_x.ptr, o * n * es), block, n, sigma,
                                             off(d_y.ptr, o * n * es), None))
        d_map = _native.DeviceBuffer(B * L * 4)
        d_tf = _native.DeviceBuffer(B * 4)
        d_cnt = _native.DeviceBuffer(4 * 8)
        d_cnt.zero()
        _native.check(lib.sg_amp_decode_device(plan, d_y.ptr, B, d_true.ptr, float(self.vars[point]), self.t_max,
                                               self.rtol, self.phi, d_map.ptr, d_tf.ptr, None, None, None))
        _native.check(lib.sg_amp_count_errors_device(d_map.ptr, d_true.ptr, d_tf.ptr, B, L, logM, d_cnt.ptr, None))
        cnt = d_cnt.download(np.zeros(4, np.int64))
        return np.array([B, cnt[1], cnt[2], cnt[3], cnt[0]], dtype=np.int64)


class ConcatTrial:
    """Concatenated SPARC + LDPC codewords (sparc_sim_new.sparc_ldpc_sim,
    sparc_new.py:15-82) at the points' AWGN variances,
    generated and decoded in batches by pipeline.ConcatPipeline (dense AMP ->
    glue -> batched BP -> device counters).  Block b of point p draws its user
    bits and noise from Philox keyed (seed, p << 32 | b) on the GPU (rng
    "device", with the LDPC encoder on the GPU too) or from
    default_rng([seed, p, b]) on the host (rng "host"), so results do not
    depend on the rank count.  Counters [codewords, user-bit errors, codeword errors,
    unprotected-bit errors, protected-bit errors]; per-block BERs of this
    rank are kept in block_ber[point]."""

    def __init__(self, pipe, awgn_vars, seed=0, rng="device"):
        self.pipe, self.vars, self.seed = pipe, list(awgn_vars), int(seed)
        self.user_bits = pipe.L_unp * pipe.logM + pipe.mults * pipe.c.K
        self.block_ber = {}
        if rng not in ("host", "device"):
            raise ValueError("rng must be 'host' (numpy default_rng([seed, point, block])) or 'device' (Philox)")
        self.rng = rng

    def __call__(self, point, first_block, n_blocks, block):
        tot = np.zeros(NC, dtype=np.int64)
        for b in range(first_block, first_block + n_blocks):
            if self.rng == "device":  # throughput mode: no host encode or host RNG in the loop
                self.pipe.make_batch_device(block, self.vars[point], self.seed, (int(point) << 32) | int(b))
            else:
                self.pipe.make_batch(block, self.vars[point], np.random.default_rng([self.seed, int(point), int(b)]))
            self.pipe.reset_counts()
            self.pipe.decode()
            c = self.pipe.counts()
            tot += c
            self.block_ber.setdefault(point, []).append(float(c[1]) / (c[0] * self.user_bits))
        return tot


def concat_ber_sweep(L, M, n, P, L_unprotected, mults, ebn0_db, *, codewords, block=256, blocks_per_round=None,
                     rank=0, world=1, agg=None, design_seed=0, seed=0, t_max=25, bp_its=200, precision="f32",
                     ldpc=("802.11n", "1/2", 81), min_errors=None, checkpoint_dir=None, npz_file=None, rng="device",
                     trial=None, max_rounds=None, on_point=None):
    """BER / FER of concatenated SPARC + LDPC against Eb/N0 (the experiment of
    ldpc_sparc/performance_plots_general.py:100-138 for the plain concatenated
    decoder), `codewords` per point sharded over the ranks.  Eb/N0 to noise as
    the bench: awgn_var = P / (2 R_overall 10^(Eb/N0 / 10)), R_overall = user
    bits / n.  Returns one dict per point; rank 0 writes `npz_file` in the
    layout of performance_plots_general.py:138 (ber_store_averages, _max,
    _min over the blocks rank 0 decoded, and snr_store = Eb/N0 in dB), plus a
    `complete` flag per point; a sweep that `max_rounds` interrupted writes
    `<npz_file>.partial.npz` instead, so it never overwrites a final file.
    `trial(point, first_block, n_blocks, block)` (counters as ConcatTrial's)
    replaces the GPU pipeline (CPU rehearsals: tools/c5_sweep.py --rehearsal); `max_rounds`
    interrupts every point after that many rounds (run_point); `on_point(dict)`
    is called with each point's result as soon as it is done."""
    from .ldpc import code
    agg = agg or Aggregator()
    logM = int(np.log2(M))
    user_bits = L_unprotected * logM + mults * code(*ldpc).K
    r_overall = user_bits / n
    vars_ = [P / (2 * r_overall * 10 ** (e / 10)) for e in ebn0_db]
    if trial is None:
        from .pipeline import ConcatPipeline
        pipe = ConcatPipeline(L, M, n, P, L_unprotected, mults, ldpc=ldpc, design_seed=design_seed,
                              precision=precision, t_max=t_max, bp_its=bp_its)
        assert pipe.L_unp * pipe.logM + pipe.mults * pipe.c.K == user_bits
        trial = ConcatTrial(pipe, vars_, seed, rng)
    bpr = blocks_per_round or max(1, world)
    out = []
    for point, e in enumerate(ebn0_db):
        params = {"P": P, "L_unprotected": L_unprotected, "mults": mults, "ebn0_db": float(e),
                  "seed": seed, "design_seed": design_seed, "t_max": t_max, "bp_its": bp_its,
                  "precision": precision, "ldpc": list(ldpc), "codewords": codewords, "rng": rng,
                  "min_errors": min_errors}
        if min_errors is not None:
            # the counters stop at round granularity, so with an error target
            # the round size is part of the experiment (without one the point
            # ends at `codewords`, a multiple of the block, at any round size)
            params["blocks_per_round"] = bpr
        tot = run_point(trial, point, block=block, blocks_per_round=bpr, rank=rank, world=world, agg=agg,
                        min_errors=min_errors, max_units=codewords, checkpoint_dir=checkpoint_dir,
                        tag=f"concat_L{L}_M{M}_n{n}", params=params, max_rounds=max_rounds)
        out.append({"ebn0_db": float(e), "awgn_var": vars_[point], "codewords": int(tot[0]),
                    "ber": float(tot[1]) / (tot[0] * user_bits) if tot[0] else None,
                    "fer": float(tot[2]) / tot[0] if tot[0] else None,
                    "unprotected_bit_errors": int(tot[3]), "protected_bit_errors": int(tot[4]),
                    "R_overall": r_overall,
                    # False when max_rounds interrupted the point before its target
                    "complete": bool(tot[0] >= codewords or (min_errors is not None and tot[2] >= min_errors))})
        if on_point is not None:
            on_point(out[-1])
    if npz_file and rank == 0:
        complete = np.array([o["complete"] for o in out])
        if not complete.all():  # an interrupted sweep never overwrites a final file
            npz_file = (npz_file[:-4] if npz_file.endswith(".npz") else npz_file) + ".partial.npz"
        avg = np.array([[o["ber"] for o in out]], dtype=float)
        bb = [getattr(trial, "block_ber", {}).get(p, [np.nan]) for p in range(len(ebn0_db))]
        np.savez(npz_file, ber_store_averages=avg, ber_store_max=np.array([[np.max(b) for b in bb]]),
                 ber_store_min=np.array([[np.min(b) for b in bb]]), snr_store=np.asarray(ebn0_db, dtype=float),
                 complete=complete)
    return out


def ldpc_awgn_campaign(standard, rate, z, ptype="A", *, rank=0, world=1, agg=None, N_MEASUREMENTS=24,
                       C_AWGN_OFFSET=1.0, P_STEP=100.0, MIN_ERRORS=100, MAX_BLOCKS=400000, block=256,
                       blocks_per_round=16, dectype="sumprod2", max_it=200, precision="f32", seed=0,
                       results_file=None, checkpoint_dir=None, trial=None):
    """The BER/FER campaign of ldpc_awgn.sim (ldpc_awgn.py:60-114) on the GPU(s):
    same starting SNR, stopping rule (each point ends at the codeword whose
    frame error is the MIN_ERRORS-th, or at MAX_BLOCKS codewords, counted in
    block order whatever the rank count) and SNR-step heuristic; returns and
    (rank 0) appends the result tuples (standard, rate, z, ptype, SNR, nblocks,
    nblockerrors, nblocks*K, nbiterrors, nit_total) -- the 11-field form that
    results2csv.c parses (results2csv.c:47-48).  `trial` replaces the GPU
    trial (tests)."""
    from .ldpc import code
    Rv = {"1/2": .5, "2/3": 0.6667, "3/4": 0.75, "5/6": 0.83333}
    if rate not in Rv:
        raise NameError("Rate unsupported")
    agg = agg or Aggregator()
    c = code(standard, rate, z, ptype)
    snr = 10.0 * np.log10(np.power(2, Rv[rate]) - 1.0) + C_AWGN_OFFSET
    res = []
    trial = trial or LdpcTrial(c, [], dectype, max_it, 0.7, precision, seed, per_unit=True)
    for point in range(N_MEASUREMENTS):
        trial.snrs.append(snr)
        params = {"seed": seed, "dectype": dectype, "max_it": max_it, "precision": precision, "snr": float(snr),
                  "min_errors": MIN_ERRORS, "max_blocks": MAX_BLOCKS}
        tot = run_point(trial, point, block=block, blocks_per_round=blocks_per_round, rank=rank, world=world,
                        agg=agg, min_errors=MIN_ERRORS, max_units=MAX_BLOCKS, checkpoint_dir=checkpoint_dir,
                        tag=f"ldpc_{standard}_{rate.replace('/', '')}_{z}_{ptype}", params=params)
        nblocks = int(tot[0])
        out = (standard, rate, z, ptype, snr, nblocks, int(tot[2]), nblocks * c.K, int(tot[1]), int(tot[3]))
        res.append(out)
        if results_file and rank == 0:
            with open(results_file, "a") as f:
                f.write(str(out) + "\n")
        snr += np.sqrt(P_STEP / nblocks)
    return res


def results_to_csv(lines):
    """The conversion of results2csv.c:47-72 (standard code, rate, type, z, SNR,
    nblocks, nblockerrors, nbits, nbiterrors, nit) for result tuples."""
    out = []
    for (std, rate, z, ptype, snr, nb, nbe, nbits, nber, nit) in lines:
        num, den = (int(v) for v in rate.split("/"))
        out.append(f"{'16' if std[5] == '6' else '11'}, {num / den:g}, {0 if ptype == 'A' else 1}, {z}, "
                   f"{snr:g}, {nb}, {nbe}, {nbits}, {nber}, {nit}")
    return out
