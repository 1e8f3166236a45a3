"""CPU tests of bench.py's launcher (no GPU): --gpus N starts N ranks through
torch.distributed.run before any GPU call (the reference's own parallelism is
one process per sim_id, ldpc_jossy/py/ldpc_awgn.py:125-131), a mismatched
WORLD_SIZE or engine knobs in the environment are refused, and the CPU
baseline pool (oracle/cpu_pool.py) decodes like the serial restatement."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if not k.startswith("SG_AMP_") and k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_gpus_two_spawns_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--rendezvous-check"], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    out = json.loads(lines[0])
    assert out["n_ranks"] == 2 and out["ranks"] == [0, 1] and out["world_size"] == 2


def test_world_size_mismatch_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--rendezvous-check"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


@pytest.mark.parametrize("knob", ["SG_AMP_SKIP", "SG_AMP_ENGINE", "SG_AMP_HANDOVER"])
def test_engine_knobs_refused(knob):
    r = subprocess.run([sys.executable, BENCH, "--steps", "1"], env=_env(**{knob: "1"}), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 3 and knob in r.stderr


def test_more_gpus_than_visible_refused():
    # no GPU in this container: --gpus 2 must exit non-zero, never fall back to one rank
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"], env=_env(), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 2 and "GPU" in r.stderr


_LAUNCH_PROBE = r'''
import subprocess, sys, types
fake = types.ModuleType("amdsmi")
class _F:
    INIT_AMD_GPUS = 1
fake.AmdSmiInitFlags = _F
fake.amdsmi_init = lambda flags: None
fake.amdsmi_get_processor_handles = lambda: list(range(8))
fake.amdsmi_shut_down = lambda: None
sys.modules["amdsmi"] = fake
calls = []
class _R:
    returncode = 0
subprocess.run = lambda cmd, env=None: (calls.append(cmd), _R())[1]
sys.argv = ["bench.py", "--gpus", "8"]
import bench
code = None
try:
    bench.maybe_spawn(bench.parse())
except SystemExit as e:
    code = e.code
import json
print(json.dumps({"code": code, "torch_loaded": "torch" in sys.modules,
                  "hip_loaded": any("amdhip" in l for l in open("/proc/self/maps")),
                  "cmd": calls[0] if calls else None}))
'''


def test_launcher_counts_gpus_without_hip():
    """--gpus 8 with 8 GPUs visible (amdsmi stubbed): the parent starts
    torch.distributed.run with 8 processes per node and exits with its code,
    without importing torch or mapping the HIP runtime (so no GPU call can
    precede the launch)."""
    env = {k: v for k, v in _env().items() if not k.endswith("_VISIBLE_DEVICES")}
    r = subprocess.run([sys.executable, "-c", _LAUNCH_PROBE], env=env, capture_output=True, text=True,
                       timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["code"] == 0 and not out["torch_loaded"] and not out["hip_loaded"], out
    assert "torch.distributed.run" in out["cmd"] and "--nproc-per-node=8" in out["cmd"]


def test_visible_devices_mask_narrows_count():
    r = subprocess.run([sys.executable, "-c", _LAUNCH_PROBE], env=_env(HIP_VISIBLE_DEVICES="0,1"),
                       capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["code"] == 2 and out["cmd"] is None, out


def test_cpu_pool_matches_serial_oracle():
    """Two-process pool = the serial CPU restatement, codeword for codeword."""
    from oracle import bp, cpu_pool, sparc_ref
    from ldpc_sparc_amd import sparc
    from ldpc_sparc_amd.ldpc import code
    L, M, n = 16, 64, 96
    W = np.array(15.0)
    o0, o1 = sparc.generate_ordering(W, n, L * M, 5)
    Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
    rs = np.random.RandomState(3)
    true = rs.randint(0, M, (4, L))
    Y = []
    for b in range(4):
        beta0 = np.zeros(L * M)
        beta0[np.arange(L) * M + true[b]] = 1
        Y.append(Ab(beta0) + rs.randn(n))
    Y = np.array(Y)
    res, _ = cpu_pool.amp_decode(2, W, L, M, n, o0, o1, Y, true, 10)
    assert sorted(res) == [0, 1, 2, 3]
    for b in range(4):
        beta0 = np.zeros(L * M)
        beta0[np.arange(L) * M + true[b]] = 1
        bh, tf, nm, _ = sparc_ref.amp(Y[b], W, L, M, n, 1.0, 10, Ab, Az, beta0)
        assert np.array_equal(res[b][0], np.argmax(bh.reshape(L, M), 1)) and res[b][1] == tf
        np.testing.assert_array_equal(res[b][2], nm)
    c = code("802.11n", "1/2", 27)
    rng = np.random.default_rng(1)
    X = c.encode_batch(rng.integers(0, 2, (40, c.K)))
    ch = 2 * ((1 - 2 * X) + 0.8 * rng.standard_normal(X.shape)) / 0.64
    app, it, done, _ = cpu_pool.bp_decode(2, "minsum", ch, c.vdeg, c.cdeg, c.intrlv, 20, 0.7, chunk=16)
    oapp, oit = bp.decode_batch("minsum", ch, c.vdeg, c.cdeg, c.intrlv, 20, 0.7)
    assert done.all() and np.array_equal(app, oapp) and np.array_equal(it, oit)
