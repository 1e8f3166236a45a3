"""In-process A/B of two plan variants selected by an environment knob read at
plan creation (e.g. SG_AMP_WAVEFFT=1 vs 0): same inputs, decodes interleaved,
HIP-event timing on the library stream.
usage: python tools/ab_env.py VAR VALUE_A VALUE_B [B] [reps]"""
import ctypes as ct
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from ldpc_sparc_amd import _native, sparc  # noqa: E402

var, va, vb = sys.argv[1], sys.argv[2], sys.argv[3]
B = int(sys.argv[4]) if len(sys.argv) > 4 else 256
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 4
L, M, R = 1024, 512, 1.5
n = int(round(L * 9 / R))
W = np.array(15.0)
lib = _native.lib()
o0, o1 = sparc.generate_ordering(W, n, L * M, 0)
plans = {}
for v in (va, vb):
    os.environ[var] = v
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    plans[v] = (op, op.plan(_native.SG_F32))
d_bits = _native.DeviceBuffer(B * L * 9)
d_true = _native.DeviceBuffer(B * L * 4)
d_x = _native.DeviceBuffer(B * n * 4)
d_y = _native.DeviceBuffer(B * n * 4)
p0 = plans[va][1]
_native.check(lib.sg_rng_bits_device(1, 0, B, L * 9, d_bits.ptr, None))
_native.check(lib.sg_bits_to_sections_device(d_bits.ptr, B, L, 9, d_true.ptr, None))
_native.check(lib.sg_amp_encode_device(p0, d_true.ptr, B, d_x.ptr, None))
_native.check(lib.sg_awgn_device(_native.SG_F32, 1, 0, d_x.ptr, B, n, 1.0, d_y.ptr, None))
d_map = _native.DeviceBuffer(B * L * 4)
d_tf = _native.DeviceBuffer(B * 4)
d_cnt = _native.DeviceBuffer(4 * 8)
res = {va: [], vb: []}
for r in range(reps + 1):
    for v in (va, vb):
        d_cnt.zero()
        _native.synchronize()
        t0 = time.perf_counter()
        _native.check(lib.sg_amp_decode_device(plans[v][1], d_y.ptr, B, d_true.ptr, 1.0, 25, 1e-6, 1,
                                               d_map.ptr, d_tf.ptr, None, None, None))
        _native.check(lib.sg_amp_count_errors_device(d_map.ptr, d_true.ptr, d_tf.ptr, B, L, 9, d_cnt.ptr, None))
        _native.synchronize()
        dt = time.perf_counter() - t0
        cnt = d_cnt.download(np.zeros(4, np.int64))
        if r:
            res[v].append(dt)
        print(f"{var}={v} rep {r}: {dt*1e3:.2f} ms  {B/dt:.1f} cw/s  sec_err={cnt[0]} bit_err={cnt[1]} "
              f"iters={cnt[3]/B:.3f}", flush=True)
for v in (va, vb):
    a = np.array(res[v])
    print(f"{var}={v}: median {np.median(a)*1e3:.2f} ms  min {a.min()*1e3:.2f} ms  -> {B/np.median(a):.1f} cw/s")
