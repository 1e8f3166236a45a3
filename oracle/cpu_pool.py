"""TEST INFRASTRUCTURE ONLY -- the CPU baseline on every host core.

SURVEY.md 8(d): the CPU baseline runs one process per host core with
OMP_NUM_THREADS=1 (the reference's own parallelism is one independent process
per sim_id, ldpc_jossy/py/ldpc_awgn.py:125-131).  This module fans the CPU
restatements out over such a pool:

  * amp -- oracle/sparc_ref.amp (sparc_public/sparc.py:883-999, scipy fftpack
    DCT operators, float128 softmax), one codeword per task;
  * bp  -- oracle/bp_oracle.c (ldpc_jossy/src/c_ldpc.c:138-206/:339-381 with
    the min-sum loop index corrected), a chunk of codewords per task.

Used by bench.py's cpu_baseline legs and by tests/ as the checker.  The
product never imports it.  Workers start with the 'spawn' method: each is a
fresh interpreter that imports only numpy/scipy and the oracle, so no child
inherits GPU state even though the parent (bench.py's CPU legs) has already
initialised and used the GPU when it builds the pool.
"""
import multiprocessing as mp
import os
import time

import numpy as np

_THREAD_VARS = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS", "NUMEXPR_NUM_THREADS")
_S = {}


def host_cores(cap=16):
    """Cores this process may run on, capped at `cap` (the GPU box's CPU share
    for one GPU is 16; os.cpu_count() there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(n, cap))


def _init_amp(W, L, M, n, o0, o1, Y, true, t_max):
    from oracle import sparc_ref
    Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
    _S.update(kind="amp", W=W, L=L, M=M, n=n, Y=Y, true=true, t_max=t_max, Ab=Ab, Az=Az)


def _amp_task(b):
    from oracle import sparc_ref
    L, M = _S["L"], _S["M"]
    beta0 = np.zeros(L * M)
    beta0[np.arange(L) * M + _S["true"][b]] = 1.0
    psi = []
    bh, tf, nmse, _ = sparc_ref.amp(_S["Y"][b], _S["W"], L, M, _S["n"], 1.0, _S["t_max"], _S["Ab"], _S["Az"], beta0,
                                    trace=lambda t, d: psi.append(float(np.asarray(d["psi"]).ravel()[0])))
    return (b, np.argmax(bh.reshape(L, M), 1).astype(np.int32), int(tf), np.asarray(nmse, np.float64),
            np.asarray(psi, np.float64))


def _init_bp(kind, ch, vdeg, cdeg, intrlv, max_it, factor):
    _S.update(kind=kind, ch=ch, vdeg=vdeg, cdeg=cdeg, intrlv=intrlv, max_it=max_it, factor=factor)


def _bp_task(rng):
    from oracle import bp
    a, b = rng
    app, it = bp.decode_batch(_S["kind"], _S["ch"][a:b], _S["vdeg"], _S["cdeg"], _S["intrlv"], _S["max_it"],
                              _S["factor"])
    return a, app, it


def _ready(_):
    return os.getpid()


class CpuPool:
    """A pool of `procs` single-threaded worker processes holding one
    workload.  run(tasks, deadline_s) returns (results in completion order,
    wall seconds from the first task to the last result); tasks still
    pending at the deadline are dropped, so the sample is bounded."""

    def __init__(self, procs, initializer, initargs):
        self.procs = procs
        saved = {k: os.environ.get(k) for k in _THREAD_VARS}
        for k in _THREAD_VARS:
            os.environ[k] = "1"
        try:
            self.pool = mp.get_context("spawn").Pool(procs, initializer=initializer, initargs=initargs)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        # wait until every worker has started and run its initializer
        self.pool.map(_ready, range(procs), chunksize=1)

    def run(self, fn, tasks, deadline_s):
        out = []
        t0 = time.perf_counter()
        it = self.pool.imap_unordered(fn, tasks, chunksize=1)
        for r in it:
            out.append(r)
            if time.perf_counter() - t0 >= deadline_s:
                break
        el = time.perf_counter() - t0
        return out, el

    def close(self):
        self.pool.terminate()
        self.pool.join()


def amp_pool(procs, W, L, M, n, o0, o1, Y, true, t_max):
    return CpuPool(procs, _init_amp, (np.asarray(W, float), L, M, n, o0, o1, np.asarray(Y, np.float64),
                                      np.asarray(true, np.int32), t_max))


def amp_decode(procs, W, L, M, n, o0, o1, Y, true, t_max, deadline_s=1e9, order=None):
    """Decode the rows `order` (default: all) of Y with the CPU restatement on
    `procs` processes.  Returns (dict b -> (map_idx, t_final, nmse, psi), wall s);
    psi[t] is psi after iteration t + 1 (sparc.py:973-979), so the stop rule
    compared psi[t] with psi[t - 1]."""
    pool = amp_pool(procs, W, L, M, n, o0, o1, Y, true, t_max)
    try:
        res, el = pool.run(_amp_task, list(order if order is not None else range(len(Y))), deadline_s)
    finally:
        pool.close()
    return {b: (m, tf, nm, ps) for b, m, tf, nm, ps in res}, el


def bp_decode(procs, kind, ch, vdeg, cdeg, intrlv, max_it, factor, chunk=64, deadline_s=1e9):
    """BP decode of every row of ch in chunks over `procs` processes.  Returns
    (app [done rows], it, done mask, wall s)."""
    pool = CpuPool(procs, _init_bp, (kind, np.ascontiguousarray(ch, np.float64), vdeg, cdeg, intrlv, max_it,
                                     factor))
    B = len(ch)
    try:
        res, el = pool.run(_bp_task, [(a, min(a + chunk, B)) for a in range(0, B, chunk)], deadline_s)
    finally:
        pool.close()
    app = np.zeros((B, ch.shape[1]))
    it = np.zeros(B, np.int64)
    done = np.zeros(B, bool)
    for a, ap, i in res:
        app[a:a + len(ap)] = ap
        it[a:a + len(ap)] = i
        done[a:a + len(ap)] = True
    return app, it, done, el
