"""C5 (BASELINE.json configs[4]): concatenated SPARC(L=1024, M=512, n=6144) +
4 x LDPC 802.11n r1/2 z=81 (160 unprotected sections) BER sweep over Eb/N0,
codewords sharded over the GPUs of one node with one RCCL all-reduce of the
error counters per round (montecarlo.concat_ber_sweep).

  python tools/c5_sweep.py --codewords 10000000 --ebn0 1 2 3 4 5 6
  python -m ldpc_sparc_amd.launch --nproc 8 tools/c5_sweep.py --codewords 10000000

Prints one JSON line per point on rank 0; --npz writes the arrays in the
layout of ldpc_sparc/performance_plots_general.py:138.

--rehearsal runs the same sharding, counter all-reduce (the host rendezvous group instead of RCCL),
checkpointing and npz output on the CPU with a synthetic trial in place of the
GPU pipeline (deterministic counters per (seed, point, block), so the totals
do not depend on the rank count); --max-rounds interrupts every point after
that many rounds, leaving the checkpoint for a resumed run
(tests/test_montecarlo_dist.py rehearses 8 ranks with kill and resume)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpc_sparc_amd import _native, montecarlo  # noqa: E402
from ldpc_sparc_amd.rendezvous import HostGroup  # noqa: E402


class SyntheticConcatTrial:
    """Rehearsal stand-in for montecarlo.ConcatTrial: counters [codewords,
    user-bit errors, codeword errors, unprotected, protected bit errors] of
    block b at point p drawn from default_rng([seed, p, b]), with error rates
    falling with Eb/N0 like a waterfall; per-block BERs kept like ConcatTrial."""

    def __init__(self, ebn0_db, user_bits, seed=0):
        self.ebn0, self.user_bits, self.seed = list(ebn0_db), int(user_bits), int(seed)
        self.block_ber = {}

    def __call__(self, point, first_block, n_blocks, block):
        tot = np.zeros(montecarlo.NC, dtype=np.int64)
        p_cw = 1.0 / (1.0 + np.exp(3.0 * (self.ebn0[point] - 4.5)))
        for b in range(first_block, first_block + n_blocks):
            rng = np.random.default_rng([self.seed, int(point), int(b)])
            fe = rng.binomial(1, p_cw, block)
            unp = fe * rng.integers(0, 40, block)
            prot = fe * rng.integers(1, 200, block)
            c = np.array([block, (unp + prot).sum(), fe.sum(), unp.sum(), prot.sum()], dtype=np.int64)
            tot += c
            self.block_ber.setdefault(point, []).append(float(c[1]) / (block * self.user_bits))
        return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ebn0", type=float, nargs="+", default=[1, 2, 3, 4, 5, 6])
    ap.add_argument("--codewords", type=float, default=1e7, help="per Eb/N0 point, over all GPUs")
    ap.add_argument("--block", type=int, default=256)
    ap.add_argument("--blocks-per-round", type=int, default=None)
    ap.add_argument("--min-errors", type=int, default=None, help="stop a point early at this many codeword errors")
    ap.add_argument("--design-seed", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--npz", default=None)
    ap.add_argument("--L", type=int, default=1024)
    ap.add_argument("--M", type=int, default=512)
    ap.add_argument("--n", type=int, default=6144)
    ap.add_argument("--P", type=float, default=15.0)
    ap.add_argument("--L-unprotected", type=int, default=160)
    ap.add_argument("--mults", type=int, default=4)
    ap.add_argument("--rehearsal", action="store_true",
                    help="CPU only: host-rendezvous counters and a synthetic trial instead of RCCL and the GPU pipeline")
    ap.add_argument("--max-rounds", type=int, default=None, help="interrupt every point after this many rounds")
    args = ap.parse_args()
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    agg = montecarlo.Aggregator()
    trial = None
    group = HostGroup(rank, world) if world > 1 else None  # stdlib TCP rendezvous (no PyTorch)
    if args.rehearsal:
        from ldpc_sparc_amd.ldpc import code
        user_bits = args.L_unprotected * int(np.log2(args.M)) + args.mults * code("802.11n", "1/2", 81).K
        trial = SyntheticConcatTrial(args.ebn0, user_bits, args.seed)
        if world > 1:
            agg = montecarlo.Aggregator("host", group=group)
    else:
        _native.require_gpu()
        _native.check(_native.lib().sg_set_device(local % max(_native.device_count(), 1)))
        if world > 1:
            uid = group.bcast_bytes(_native.Comm.unique_id() if rank == 0 else b"")
            agg = montecarlo.Aggregator("rccl", _native.Comm(world, rank, uid))
    t0 = time.perf_counter()
    res = montecarlo.concat_ber_sweep(args.L, args.M, args.n, args.P, args.L_unprotected, args.mults, args.ebn0,
                                      codewords=int(args.codewords), block=args.block,
                                      blocks_per_round=args.blocks_per_round, rank=rank, world=world,
                                      agg=agg, design_seed=args.design_seed, seed=args.seed,
                                      min_errors=args.min_errors, checkpoint_dir=args.checkpoint, npz_file=args.npz,
                                      trial=trial, max_rounds=args.max_rounds,
                                      on_point=(lambda r: print(json.dumps(r), flush=True)) if rank == 0 else None)
    el = time.perf_counter() - t0
    if rank == 0:
        tot = sum(r["codewords"] for r in res)
        print(json.dumps({"codewords": tot, "seconds": el, "codewords_per_s": tot / el, "gpus": world,
                          "rehearsal": bool(args.rehearsal)}), flush=True)
    if group is not None:
        group.barrier()
        group.close()


if __name__ == "__main__":
    main()
