"""Quick probe: C2 AMP decode (L=1024, M=512, n=6144, B codewords) timed on the
library stream.  Used under rocprofv3 to get the kernel breakdown."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from ldpc_sparc_amd import _native, sparc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
R = float(sys.argv[3]) if len(sys.argv) > 3 else 1.5
PREC = _native.SG_F64 if len(sys.argv) > 4 and sys.argv[4] == "f64" else _native.SG_F32
L, M = 1024, 512
n = int(round(L * 9 / R))
W = np.array(15.0)
t0 = time.time()
o0, o1 = sparc.generate_ordering(W, n, L * M, 0)
op = sparc.DesignOperator(W, L, M, n, o0, o1)
plan = op.plan(PREC)
print("plan", time.time() - t0, flush=True)
rng = np.random.default_rng(1)
true = rng.integers(0, M, (B, L)).astype(np.int32)
beta0 = np.zeros((B, L * M))
beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
Y = op.apply(beta0, False, PREC) + rng.standard_normal((B, n))
lib = _native.lib()
d_y = _native.DeviceBuffer.from_array(Y.astype(np.float64 if PREC == _native.SG_F64 else np.float32))
d_true = _native.DeviceBuffer.from_array(true)
d_map = _native.DeviceBuffer(B * L * 4)
d_tf = _native.DeviceBuffer(B * 4)
d_cnt = _native.DeviceBuffer(4 * 8)
for r in range(reps):
    d_cnt.zero()
    _native.synchronize()
    t0 = time.time()
    _native.check(lib.sg_amp_decode_device(plan, d_y.ptr, B, d_true.ptr, 1.0, 25, 1e-6, 1,
                                           d_map.ptr, d_tf.ptr, None, None, None))
    _native.check(lib.sg_amp_count_errors_device(d_map.ptr, d_true.ptr, d_tf.ptr, B, L, 9,
                                                 d_cnt.ptr, None))
    _native.synchronize()
    dt = time.time() - t0
    cnt = d_cnt.download(np.zeros(4, np.int64))
    print(f"rep {r}: {dt*1e3:.1f} ms  {B/dt:.1f} cw/s  sec_err={cnt[0]} bit_err={cnt[1]} "
          f"cw_err={cnt[2]} iters={cnt[3]/B:.2f}", flush=True)
    total_cwit = total_cwit + int(cnt[3]) if r else int(cnt[3])
if len(sys.argv) > 4:
    import json
    with open(sys.argv[4], "w") as f:
        json.dump({"B": B, "reps": reps, "codeword_iterations": total_cwit}, f)
