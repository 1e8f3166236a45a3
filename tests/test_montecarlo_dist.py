"""CPU tests of the multi-GPU Monte-Carlo layer (montecarlo.py): sharding,
the counter all-reduce (the stdlib host rendezvous group, world_size 2, the
same code path that uses RCCL between GPUs), invariance of a campaign's result to the number of ranks,
checkpoint/resume, and the results.txt -> CSV conversion of results2csv.c."""
import json
import os
import socket

import numpy as np
import pytest
import multiprocessing as mp

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


class FakeUnitTrial:
    """Per-codeword counter rows [1, bit errors, frame error, iterations, 0]
    in block order (stands in for LdpcTrial(per_unit=True))."""
    per_unit = True

    def __init__(self, snrs=()):
        self.snrs = list(snrs)

    def rows(self, point, b, block):
        snr = self.snrs[point] if self.snrs else point
        rng = np.random.default_rng([11, point, b])
        fe = rng.binomial(1, 1.0 / (2.0 + abs(snr)), block)
        be = fe * rng.integers(1, 9, block)
        return np.stack([np.ones(block, np.int64), be, fe, rng.integers(0, 50, block), np.zeros(block, np.int64)],
                        1).astype(np.int64)

    def __call__(self, point, first_block, n_blocks, block):
        return np.concatenate([self.rows(point, b, block) for b in range(first_block, first_block + n_blocks)])


def sequential_sim(trial, min_errors, max_blocks, block, n_points, snr0, p_step):
    """Restatement of ldpc_awgn.sim's loop (ldpc_awgn.py:84-114): codewords one
    by one in block order, stop at the MIN_ERRORS-th frame error or at
    MAX_BLOCKS, then SNR += sqrt(P_STEP / nblocks)."""
    snr, out = snr0, []
    for point in range(n_points):
        trial.snrs.append(snr)
        nbiterrors = nblockerrors = nblocks = nit = 0
        b = 0
        rows = trial.rows(point, b, block)
        while nblockerrors < min_errors:
            r = rows[nblocks - b * block]
            nbiterrors += int(r[1])
            nblockerrors += int(r[2])
            nit += int(r[3])
            nblocks += 1
            if nblocks >= max_blocks:
                break
            if nblocks % block == 0:
                b += 1
                rows = trial.rows(point, b, block)
        out.append((snr, nblocks, nblockerrors, nbiterrors, nit))
        snr += np.sqrt(p_step / nblocks)
    return out


def _worker(rank, world, port, q, ckpt):
    from ldpc_sparc_amd.rendezvous import HostGroup
    group = HostGroup(rank, world, "127.0.0.1", port)
    agg = mc.Aggregator("host", group=group)
    res = []
    for pt in range(3):
        res.append(mc.run_point(fake_trial, pt, block=64, blocks_per_round=5, rank=rank, world=world, agg=agg,
                                min_errors=200, max_units=5000, checkpoint_dir=ckpt).tolist())
    s = agg.allreduce(np.array([rank + 1, 10], dtype=np.int64)).tolist()
    camp = mc.ldpc_awgn_campaign("802.11n", "1/2", 27, rank=rank, world=world, agg=agg, N_MEASUREMENTS=4,
                                 MIN_ERRORS=37, MAX_BLOCKS=3000, block=32, blocks_per_round=3, trial=FakeUnitTrial())
    q.put((rank, res, s, camp))
    group.barrier()
    group.close()


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
    camp1 = mc.ldpc_awgn_campaign("802.11n", "1/2", 27, N_MEASUREMENTS=4, MIN_ERRORS=37, MAX_BLOCKS=3000,
                                  block=32, blocks_per_round=3, trial=FakeUnitTrial())
    assert out[0][3] == camp1 and out[1][3] == camp1  # the exact stopping rule does not depend on the ranks
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


def test_exact_stopping_rule_matches_sequential_sim():
    """ldpc_awgn_campaign stops every point at the same codeword as the
    reference's sequential loop, so nblocks, the counts and the SNR sequence
    agree (ldpc_awgn.py:84-114), whatever the round size."""
    for bpr in (1, 3, 16):
        camp = mc.ldpc_awgn_campaign("802.11n", "1/2", 27, N_MEASUREMENTS=5, MIN_ERRORS=25, MAX_BLOCKS=400,
                                     block=16, blocks_per_round=bpr, trial=FakeUnitTrial())
        snr0 = 10.0 * np.log10(2 ** 0.5 - 1.0) + 1.0
        ref = sequential_sim(FakeUnitTrial(), 25, 400, 16, 5, snr0, 100.0)
        for c, r in zip(camp, ref):
            assert c[4] == r[0] and (c[5], c[6], c[8], c[9]) == r[1:], (bpr, c, r)


def test_exact_stop_at_max_blocks():
    t = FakeUnitTrial([100.0])  # ~1 % frame errors: MAX_BLOCKS ends the point
    tot = mc.run_point(t, 0, block=16, blocks_per_round=4, rank=0, world=1, agg=mc.Aggregator(), min_errors=1000,
                       max_units=50)
    assert tot[0] == 50 and tot[2] == t(0, 0, 4, 16)[:50, 2].sum()


def test_checkpoint_refuses_other_parameters(tmp_path):
    d = str(tmp_path)
    mc.run_point(fake_trial, 0, block=64, blocks_per_round=5, rank=0, world=1, agg=mc.Aggregator(), min_errors=30,
                 checkpoint_dir=d, params={"seed": 1})
    with pytest.raises(ValueError):
        mc.run_point(fake_trial, 0, block=64, blocks_per_round=5, rank=0, world=1, agg=mc.Aggregator(),
                     min_errors=60, checkpoint_dir=d, params={"seed": 2})
    with pytest.raises(ValueError):  # another block size is another experiment too
        mc.run_point(fake_trial, 0, block=32, blocks_per_round=5, rank=0, world=1, agg=mc.Aggregator(),
                     min_errors=60, checkpoint_dir=d, params={"seed": 1})


def test_results_csv_format():
    line = ('802.11n', '1/2', 81, 'A', 1.7134004857467928, 400000, 91, 388800000, 8741, 6220937)
    assert mc.results_to_csv([line]) == ["11, 0.5, 0, 81, 1.7134, 400000, 91, 388800000, 8741, 6220937"]
    line = ('802.16', '2/3', 3, 'B', -1.3103816364765377, 100, 100, 4800, 1439, 20000)
    assert mc.results_to_csv([line]) == ["16, 0.666667, 1, 3, -1.31038, 100, 100, 4800, 1439, 20000"]


def _c5_rehearsal(world, ckpt, extra=(), env=None):
    """tools/c5_sweep.py --rehearsal at `world` ranks (ldpc_sparc_amd.launch,
    the host rendezvous group on the CPU); the JSON lines rank 0 prints."""
    import subprocess
    import sys
    tool = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "c5_sweep.py")
    args = ["--rehearsal", "--ebn0", "1", "3", "4.5", "6", "--codewords", "40960", "--block", "256",
            "--blocks-per-round", "8", "--min-errors", "3000", "--checkpoint", ckpt] + list(extra)
    if world == 1:
        cmd = [sys.executable, tool] + args
    else:
        cmd = [sys.executable, "-m", "ldpc_sparc_amd.launch", "--nproc", str(world), tool] + args
    env = {k: v for k, v in (env or os.environ).items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = env.get("PYTHONPATH", "") + os.pathsep + repo
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


def test_c5_sweep_rehearsal_world8_kill_and_resume(tmp_path):
    """The C5 sweep driver at 8 ranks (host-rendezvous rehearsal of the RCCL
    path), with torch not importable: interrupted after 2 rounds of every
    point, then resumed from rank 0's checkpoints, it ends with the same
    per-point counts as one uninterrupted rank; the interrupted run stopped
    short of them."""
    stub = tmp_path / "notorch" / "torch"
    stub.mkdir(parents=True)
    (stub / "__init__.py").write_text("raise ImportError('torch is blocked in this test')\n")
    env = dict(os.environ, PYTHONPATH=str(tmp_path / "notorch"))
    one = _c5_rehearsal(1, str(tmp_path / "one"), env=env)
    part = _c5_rehearsal(8, str(tmp_path / "eight"), ["--max-rounds", "2"], env=env)
    full = _c5_rehearsal(8, str(tmp_path / "eight"), env=env)
    keys = ("codewords", "ber", "fer", "unprotected_bit_errors", "protected_bit_errors")
    assert [[p[k] for k in keys] for p in full[:-1]] == [[p[k] for k in keys] for p in one[:-1]]
    assert full[-1]["gpus"] == 8 and full[-1]["rehearsal"]
    assert any(p["codewords"] < f["codewords"] for p, f in zip(part[:-1], full[:-1]))
    assert all(p["codewords"] <= 2 * 8 * 256 for p in part[:-1])
    # the error target ends the low-Eb/N0 points early; the high ones run to the codeword cap
    assert full[0]["codewords"] < 40960 and full[-2]["codewords"] == 40960


def test_checkpoint_without_min_errors_key_resumes(tmp_path):
    """A checkpoint written before min_errors was recorded (round 3) resumes
    a run whose min_errors is None, the value it implies; another value is
    still refused."""
    d = str(tmp_path)
    mc.run_point(fake_trial, 0, block=64, blocks_per_round=5, rank=0, world=1, agg=mc.Aggregator(),
                 max_units=640, checkpoint_dir=d, params={"seed": 1}, max_rounds=1)
    path = mc._ckpt_path(d, "campaign", 0)
    st = json.load(open(path))
    assert "min_errors" not in st["params"]
    tot = mc.run_point(fake_trial, 0, block=64, blocks_per_round=5, rank=0, world=1, agg=mc.Aggregator(),
                       max_units=640, checkpoint_dir=d, params={"seed": 1, "min_errors": None})
    assert tot[0] == 640
    with pytest.raises(ValueError):
        mc.run_point(fake_trial, 0, block=64, blocks_per_round=5, rank=0, world=1, agg=mc.Aggregator(),
                     max_units=640, checkpoint_dir=d, params={"seed": 1, "min_errors": 10})


def test_interrupted_sweep_writes_partial_npz(tmp_path):
    """concat_ber_sweep with max_rounds: the per-point dicts say complete=False
    and the arrays go to <npz>.partial.npz, never over the final file."""
    import numpy as np
    npz = str(tmp_path / "c5.npz")
    kw = dict(codewords=4096, block=256, blocks_per_round=2, trial=lambda p, a, n, b: np.array(
        [n * b, 3 * n, n, 2 * n, n], dtype=np.int64), npz_file=npz)
    part = mc.concat_ber_sweep(1024, 512, 9216, 15.0, 160, 4, [5.0, 6.0], max_rounds=1, **kw)
    assert not any(p["complete"] for p in part)
    assert os.path.exists(str(tmp_path / "c5.partial.npz")) and not os.path.exists(npz)
    full = mc.concat_ber_sweep(1024, 512, 9216, 15.0, 160, 4, [5.0, 6.0], **kw)
    assert all(p["complete"] for p in full)
    assert np.load(npz)["complete"].all()
