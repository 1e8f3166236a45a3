"""Multi-rank runs on the GPU box's single GPU (ranks share it; their counters
meet through the stdlib host rendezvous group, the code path that uses RCCL when each rank has
its own GPU): bench.py's own launcher at --gpus 2, and a Monte-Carlo campaign
whose trials really decode on the GPU, whose per-point results must not depend
on the number of ranks (the reference's campaign, ldpc_awgn.py:60-114, run as
one process per sim_id, :125-131)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAMPAIGN = dict(N_MEASUREMENTS=3, MIN_ERRORS=30, MAX_BLOCKS=6000, block=64, blocks_per_round=5, dectype="minsum",
                max_it=50, precision="f32", seed=11)


def test_bench_two_ranks_rehearsal():
    env = {k: v for k, v in os.environ.items() if not k.startswith("SG_AMP_")}
    env["BENCH_REHEARSAL"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-bp", "--no-sc",
                        "--no-concat", "--no-r13", "--cpu-seconds", "0", "--steps", "2", "--warmup", "1",
                        "--batch", "64"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["counter_allreduce"].startswith("host")
    assert out["value"] > 0
    full = json.load(open(os.path.join(REPO, out["detail"])))  # the full record rank 0 wrote
    assert full["amp"]["codeword_errors"] >= 0 and full["n_gpus"] == 2


def test_bench_two_ranks_under_torchrun():
    """The driver's launch form (python -m torch.distributed.run ... bench.py --gpus N): the ranks find rank 0's
    host rendezvous through the run-keyed port file, not through the agent's MASTER_PORT store."""
    env = {k: v for k, v in os.environ.items() if not k.startswith("SG_AMP_") and k != "SG_RDZV_PORT"}
    env["BENCH_REHEARSAL"] = "1"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-bp", "--no-sc", "--no-sc-notebook",
                        "--no-concat", "--no-r13", "--no-f64", "--cpu-seconds", "0", "--steps", "2", "--warmup", "1",
                        "--batch", "64"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["counter_allreduce"].startswith("host") and out["value"] > 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path.insert(0, REPO)
    from ldpc_sparc_amd import montecarlo as mc
    from ldpc_sparc_amd.rendezvous import HostGroup
    group = HostGroup(rank, world, "127.0.0.1", port)
    res = mc.ldpc_awgn_campaign("802.11n", "1/2", 27, rank=rank, world=world,
                                agg=mc.Aggregator("host", group=group), **CAMPAIGN)
    q.put((rank, res))
    group.barrier()
    group.close()


def test_ldpc_campaign_two_ranks_equals_one():
    from ldpc_sparc_amd import montecarlo as mc
    single = mc.ldpc_awgn_campaign("802.11n", "1/2", 27, **CAMPAIGN)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=200) for _ in range(2))
    for p in procs:
        p.join(60)
    assert out[0][1] == single and out[1][1] == single
    for row in single:  # every point stopped exactly at MIN_ERRORS frame errors (or MAX_BLOCKS)
        assert row[6] == 30 or row[5] == 6000
