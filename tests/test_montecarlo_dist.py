"""CPU tests of the multi-GPU Monte-Carlo layer (montecarlo.py): sharding,
the counter all-reduce (gloo, world_size 2, the same code path that uses RCCL
between GPUs), invariance of a campaign's result to the number of ranks,
checkpoint/resume, and the results.txt -> CSV conversion of results2csv.c."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ldpc_sparc_amd import montecarlo as mc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def fake_trial(point, first_block, n_blocks, block):
    """Deterministic per-block counters (stands in for a GPU decoder)."""
    out = np.zeros(mc.NC, dtype=np.int64)
    for b in range(first_block, first_block + n_blocks):
        rng = np.random.default_rng([7, point, b])
        errs = rng.binomial(1, 0.1 + 0.2 * point, block)
        out += [block, errs.sum() * 3, errs.sum(), b, 1]
    return out


def test_shard_range_partitions():
    for total in (0, 1, 7, 16, 1000):
        for world in (1, 2, 3, 8):
            parts = [mc.shard_range(total, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in parts) - min(b - a for a, b in parts) <= 1


def _worker(rank, world, port, q, ckpt):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    agg = mc.Aggregator("gloo")
    res = []
    for pt in range(3):
        res.append(mc.run_point(fake_trial, pt, block=64, blocks_per_round=5, rank=rank, world=world, agg=agg,
                                min_errors=200, max_units=5000, checkpoint_dir=ckpt).tolist())
    s = agg.allreduce(np.array([rank + 1, 10], dtype=np.int64)).tolist()
    q.put((rank, res, s))
    dist.destroy_process_group()


def _run(world, ckpt=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, ckpt)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
    return sorted(out)


def test_campaign_world2_equals_world1(tmp_path):
    single = [mc.run_point(fake_trial, pt, block=64, blocks_per_round=5, rank=0, world=1, agg=mc.Aggregator(),
                           min_errors=200, max_units=5000).tolist() for pt in range(3)]
    out = _run(2)
    assert out[0][1] == single and out[1][1] == single  # every rank sees the global counts
    assert out[0][2] == [3, 20] and out[1][2] == [3, 20]
    for r in single:
        assert r[2] >= 200 or r[0] >= 5000


def test_checkpoint_resume(tmp_path):
    d = str(tmp_path)
    first = mc.run_point(fake_trial, 0, block=64, blocks_per_round=5, rank=0, world=1, agg=mc.Aggregator(),
                         min_errors=30, max_units=None, checkpoint_dir=d)
    # resuming with a higher target continues from the stored counters
    resumed = mc.run_point(fake_trial, 0, block=64, blocks_per_round=5, rank=0, world=1, agg=mc.Aggregator(),
                           min_errors=200, max_units=None, checkpoint_dir=d)
    fresh = mc.run_point(fake_trial, 0, block=64, blocks_per_round=5, rank=0, world=1, agg=mc.Aggregator(),
                         min_errors=200, max_units=None)
    assert first[2] >= 30
    assert resumed.tolist() == fresh.tolist()


def test_results_csv_format():
    line = ('802.11n', '1/2', 81, 'A', 1.7134004857467928, 400000, 91, 388800000, 8741, 6220937)
    assert mc.results_to_csv([line]) == ["11, 0.5, 0, 81, 1.7134, 400000, 91, 388800000, 8741, 6220937"]
    line = ('802.16', '2/3', 3, 'B', -1.3103816364765377, 100, 100, 4800, 1439, 20000)
    assert mc.results_to_csv([line]) == ["16, 0.666667, 1, 3, -1.31038, 100, 100, 4800, 1439, 20000"]
