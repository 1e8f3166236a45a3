"""C5 (BASELINE.json configs[4]): concatenated SPARC(L=1024, M=512, n=6144) +
4 x LDPC 802.11n r1/2 z=81 (160 unprotected sections) BER sweep over Eb/N0,
codewords sharded over the GPUs of one node with one RCCL all-reduce of the
error counters per round (montecarlo.concat_ber_sweep).

  python tools/c5_sweep.py --codewords 10000000 --ebn0 1 2 3 4 5 6
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
      tools/c5_sweep.py --codewords 10000000

Prints one JSON line per point on rank 0; --npz writes the arrays in the
layout of ldpc_sparc/performance_plots_general.py:138."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpc_sparc_amd import _native, montecarlo  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ebn0", type=float, nargs="+", default=[1, 2, 3, 4, 5, 6])
    ap.add_argument("--codewords", type=float, default=1e7, help="per Eb/N0 point, over all GPUs")
    ap.add_argument("--block", type=int, default=256)
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
    args = ap.parse_args()
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    _native.require_gpu()
    _native.check(_native.lib().sg_set_device(local % max(_native.device_count(), 1)))
    agg = montecarlo.Aggregator()
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        obj = [_native.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        agg = montecarlo.Aggregator("rccl", _native.Comm(world, rank, obj[0]))
    t0 = time.perf_counter()
    res = montecarlo.concat_ber_sweep(args.L, args.M, args.n, args.P, args.L_unprotected, args.mults, args.ebn0,
                                      codewords=int(args.codewords), block=args.block, rank=rank, world=world,
                                      agg=agg, design_seed=args.design_seed, seed=args.seed,
                                      min_errors=args.min_errors, checkpoint_dir=args.checkpoint, npz_file=args.npz)
    el = time.perf_counter() - t0
    if rank == 0:
        for r in res:
            print(json.dumps(r), flush=True)
        tot = sum(r["codewords"] for r in res)
        print(json.dumps({"codewords": tot, "seconds": el, "codewords_per_s": tot / el, "gpus": world}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
