"""Per-launch kernel times of the split C2 engine with every codeword active
(rtol = 0: no early stop), for phase-ablation variants built with
tools/mk_variant.sh (their results are garbage; only the times matter).

usage: python tools/c2_ablate.py [B] [t_max] [reps] [R] [f32|f64]
prints one JSON line: ms per launch of cw2_ab / cw2_az / ctrl, and the
decode's wall time."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpc_sparc_amd import _native, sparc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
t_max = int(sys.argv[2]) if len(sys.argv) > 2 else 10
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
R = float(sys.argv[4]) if len(sys.argv) > 4 else 1.5
PREC = _native.SG_F64 if len(sys.argv) > 5 and sys.argv[5] == "f64" else _native.SG_F32
L, M = 1024, 512
n = int(round(L * 9 / R))
W = np.array(15.0)
o0, o1 = sparc.generate_ordering(W, n, L * M, 0)
op = sparc.DesignOperator(W, L, M, n, o0, o1)
plan = op.plan(PREC)
rng = np.random.default_rng(1)
true = rng.integers(0, M, (B, L)).astype(np.int32)
beta0 = np.zeros((B, L * M))
beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
Y = op.apply(beta0, False, _native.SG_F32) + rng.standard_normal((B, n))
lib = _native.lib()
d_y = _native.DeviceBuffer.from_array(Y.astype(np.float64 if PREC == _native.SG_F64 else np.float32))
d_true = _native.DeviceBuffer.from_array(true)
d_map = _native.DeviceBuffer(B * L * 4)
d_tf = _native.DeviceBuffer(B * 4)


def decode():
    _native.check(lib.sg_amp_decode_device(plan, d_y.ptr, B, d_true.ptr, 1.0, t_max, 1e-30, 1,
                                           d_map.ptr, d_tf.ptr, None, None, None))


decode()
_native.synchronize()
prof = _native.Profiler(1)
t0 = time.perf_counter()
for _ in range(reps):
    decode()
_native.synchronize()
wall = time.perf_counter() - t0
ph = prof.stop()
tf = d_tf.download(np.zeros(B, np.int32))
out = {"lib": os.environ.get("LDPC_SPARC_AMD_LIB", "default"), "prec": "f64" if PREC == _native.SG_F64 else "f32", "B": B, "t_max": t_max, "reps": reps,
       "t_final_mean": float(tf.mean()), "wall_ms_per_decode": 1e3 * wall / reps}
for k, (ms, cnt) in sorted(ph.items()):
    out[k] = {"ms_per_launch": ms / max(cnt, 1), "launches": cnt}
print(json.dumps(out), flush=True)
