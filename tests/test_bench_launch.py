"""CPU tests of bench.py's launcher (no GPU): --gpus N starts N ranks
(ldpc_sparc_amd.launch, no PyTorch) before any GPU call (the reference's own parallelism is
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
class _P:
    def __init__(self, cmd, env=None):
        calls.append((cmd, {k: env[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "SG_RDZV_PORT")}))
    def poll(self):
        return 0
    def send_signal(self, s):
        pass
    def kill(self):
        pass
    def wait(self):
        return 0
subprocess.Popen = _P
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
                  "calls": calls}))
'''


def test_launcher_counts_gpus_without_hip():
    """--gpus 8 with 8 GPUs visible (amdsmi stubbed): the parent starts 8 ranks
    of bench.py (ldpc_sparc_amd.launch: RANK 0..7, one rendezvous port) and
    exits with the job's code, without importing torch or mapping the HIP
    runtime (so no GPU call can precede the launch)."""
    env = {k: v for k, v in _env().items() if not k.endswith("_VISIBLE_DEVICES")}
    r = subprocess.run([sys.executable, "-c", _LAUNCH_PROBE], env=env, capture_output=True, text=True,
                       timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["code"] == 0 and not out["torch_loaded"] and not out["hip_loaded"], out
    assert len(out["calls"]) == 8
    assert [c[1]["RANK"] for c in out["calls"]] == [str(r) for r in range(8)]
    assert all(c[1]["WORLD_SIZE"] == "8" for c in out["calls"])
    assert len({c[1]["SG_RDZV_PORT"] for c in out["calls"]}) == 1
    assert all(c[0][1].endswith("bench.py") and "--gpus" in c[0] for c in out["calls"])


def test_visible_devices_mask_narrows_count():
    r = subprocess.run([sys.executable, "-c", _LAUNCH_PROBE], env=_env(HIP_VISIBLE_DEVICES="0,1"),
                       capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["code"] == 2 and out["calls"] == [], out


def _no_torch_env(tmp_path):
    """An environment in which `import torch` fails (a stub package first on
    PYTHONPATH): the multi-rank paths must not need PyTorch (north_star)."""
    stub = tmp_path / "notorch" / "torch"
    stub.mkdir(parents=True)
    (stub / "__init__.py").write_text("raise ImportError('torch is blocked in this test')\n")
    env = _env()
    env["PYTHONPATH"] = str(tmp_path / "notorch") + os.pathsep + env.get("PYTHONPATH", "")
    return env


def test_rendezvous_without_torch(tmp_path):
    """--gpus 4 --rendezvous-check with torch not importable: four ranks
    started by the stdlib launcher meet over the stdlib rendezvous."""
    env = _no_torch_env(tmp_path)
    chk = subprocess.run([sys.executable, "-c", "import torch"], env=env, capture_output=True, text=True)
    assert chk.returncode != 0 and "blocked" in chk.stderr
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--rendezvous-check"], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["ranks"] == [0, 1, 2, 3] and out["torch_loaded"] is False


def test_rendezvous_under_torchrun_file_discovery():
    """The driver launches N > 1 through torch.distributed.run, whose agent
    holds MASTER_PORT: the ranks then find rank 0's relay through the temp
    file keyed by the run (no SG_RDZV_PORT)."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr", "127.0.0.1", f"--master-port={port}", BENCH, "--gpus", "3", "--rendezvous-check"]
    env = {k: v for k, v in _env().items() if k != "SG_RDZV_PORT"}
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["ranks"] == [0, 1, 2]


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


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_summary_is_compact_and_last_key_material():
    """The line's closing "summary" repeats every configuration's value,
    roofline fraction and CPU decision match in a few hundred bytes (a log that
    keeps only the line's tail still shows C3-C5)."""
    b = _bench_module()
    out = {"value": 10900.5, "roofline": {"frac": 0.1834, "bound": "valu-f32", "valu_issue_frac": 0.55,
                                          "flops_per_lane_instr": 1.4},
           "cpu_baseline": {"ber_match": {"identical_section_decisions": 0.99998}},
           "amp_r13": {"value": 13100.0, "roofline": {}, "cpu_baseline": {"ber_match": {
               "identical_section_decisions": 1.0}}},
           "bp": {"value": 4.5e6, "roofline": {"frac": 0.59, "bound": "lds"},
                  "cpu_baseline": {"ber_match": {"identical_codeword_decisions": 1.0}}},
           "concat": {"value": 270.0, "roofline": {"frac": 0.85, "bound": "mfma"},
                      "decision_match": {"identical_block_decisions_where_oracle_decodes": 1.0}}}
    s = b.summary(out)
    assert s["C2"] == {"value": 10900.5, "frac": 0.1834, "bound": "valu-f32", "cpu_match": 0.99998}
    assert s["C3"]["cpu_match"] == 1.0 and s["C5"]["frac"] == 0.85 and s["C5"]["cpu_match"] == 1.0
    assert s["C2_factors"] == {"valu_issue": 0.55, "flops_per_lane": 1.4}
    assert "C4" not in s and len(json.dumps(s)) < 700


def test_pmc_files_only_for_this_build(tmp_path, monkeypatch):
    """bench.py reports PMC traffic / SQ figures only from a summary whose
    lib_sha256 is the running library's."""
    b = _bench_module()
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(b, "REPO", str(tmp_path))
    dig = b.lib_digest()
    (prof / "r09_pmc_traffic_bench_old.json").write_text(json.dumps({"lib_sha256": "0" * 16, "amp": {
        "kernel": "cw2_ab", "hbm_bytes_per_codeword_iteration": 1.0}}))
    assert b.pmc_traffic("amp", "hbm_bytes_per_codeword_iteration", "cw2_") == (None, None)
    (prof / "r09_pmc_traffic_bench_new.json").write_text(json.dumps({"lib_sha256": dig, "amp": {
        "kernel": "cw2_ab+cw2_az", "hbm_bytes_per_codeword_iteration": 2.0}}))
    assert b.pmc_traffic("amp", "hbm_bytes_per_codeword_iteration", "cw2_") == (2.0, "r09_pmc_traffic_bench_new.json")
    (prof / "r09_pmc_sq_bench.json").write_text(json.dumps({"lib_sha256": dig, "amp": {
        "valu_wave_insts_per_codeword_iteration": 5.0}}))
    assert b.pmc_sq("amp")[0]["valu_wave_insts_per_codeword_iteration"] == 5.0


def test_compact_line_fits_the_driver(tmp_path):
    """The printed line is built from the full record (here round 5's, whose
    23 KB line the driver could not ingest): under 8 KB, with the contract keys,
    the C2 roofline and cpu_baseline, and one short entry per companion."""
    b = _bench_module()
    with open(os.path.join(REPO, "tests", "data", "bench_out_r05.json")) as f:
        out = json.load(f)
    line = b.compact_line(out, "profiles/bench_detail_0123456789abcdef.json")
    s = json.dumps(line, separators=(",", ":"))
    assert len(s) < b.LINE_MAX_BYTES and len(s) < 4096, len(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "cpu_baseline", "higher_is_better", "scaling", "vs_baseline", "data"):
        assert k in line, k
    rf = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "valu_issue_frac", "lds_bank_conflict_frac"):
        assert rf[k] is not None, k
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    cb = line["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample", "port_over_reference_speed", "ber_match"):
        assert cb[k] is not None, k
    comp = line["companions"]
    for k in ("C2_R1.3", "C2_f64", "C3", "C4", "C4_notebook", "C5"):
        assert k in comp and len(json.dumps(comp[k])) <= 150, (k, comp.get(k))
    assert line["value"] == out["value"] and line["ms_per_step"] == out["ms_per_step"]
    assert line["detail"].startswith("profiles/bench_detail_")
    # the detail file holds the full record
    p = b.write_detail(out, str(tmp_path))
    assert json.load(open(os.path.join(REPO, p))) == out


def test_rendezvous_survives_silent_and_foreign_peers():
    """A peer that connects to the relay and never says hello, and one with the wrong key, are dropped; the
    real ranks still meet (rendezvous.py handshake timeouts)."""
    import socket as _so
    import threading
    from ldpc_sparc_amd.rendezvous import HostGroup, free_port
    port = free_port()
    out = {}

    def rank(r):
        g = HostGroup(r, 2, "127.0.0.1", port, timeout=60)
        out[r] = g.allreduce_sum_i64([r + 1, 10 * r])
        g.close()

    t0 = threading.Thread(target=rank, args=(0,))
    t0.start()
    silent = None
    for _ in range(200):  # the relay is up once rank 0 listens
        try:
            silent = _so.create_connection(("127.0.0.1", port), timeout=1.0)
            break
        except OSError:
            import time
            time.sleep(0.05)
    assert silent is not None
    foreign = _so.create_connection(("127.0.0.1", port), timeout=1.0)
    body = b'{"key": "not-this-run", "rank": 1}'
    foreign.sendall(len(body).to_bytes(8, "little") + body)
    t1 = threading.Thread(target=rank, args=(1,))
    t1.start()
    t0.join(30)
    t1.join(30)
    silent.close()
    foreign.close()
    assert not t0.is_alive() and not t1.is_alive()
    assert out[0].tolist() == [3, 10] and out[1].tolist() == [3, 10]


def test_launcher_stops_siblings_of_a_failed_rank(tmp_path, monkeypatch):
    """Rank 1 exits 3; rank 0 ignores SIGTERM and would wait for it forever: the launcher returns 3 and
    kills rank 0 after the grace period (ldpc_sparc_amd.launch.spawn)."""
    import time
    from ldpc_sparc_amd import launch
    script = tmp_path / "rank.py"
    script.write_text("import os, signal, sys, time\n"
                      "if os.environ['RANK'] == '1':\n"
                      "    time.sleep(0.5); sys.exit(3)\n"
                      "signal.signal(signal.SIGTERM, signal.SIG_IGN)\n"
                      "time.sleep(120)\n")
    monkeypatch.setattr(launch, "GRACE_S", 1.0)
    t0 = time.monotonic()
    assert launch.spawn(2, [sys.executable, str(script)]) == 3
    assert time.monotonic() - t0 < 30
