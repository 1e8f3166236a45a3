"""Phase timing of the stage-1 kernels (SG_AMP_TPROF=1): mean shader-clock
cycles per phase, per workgroup, for the C2 decode at B codewords
(usage: amp_tprof.py [B] [f32|f64])."""
import ctypes as ct
import os
import sys

import numpy as np

os.environ["SG_AMP_TPROF"] = "1"
sys.path.insert(0, ".")
from ldpc_sparc_amd import _native, sparc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
prec = _native.SG_F64 if len(sys.argv) > 2 and sys.argv[2] == "f64" else _native.SG_F32
es = 8 if prec == _native.SG_F64 else 4
L, M, R = 1024, 512, 1.5
n = int(round(L * 9 / R))
W = np.array(15.0)
lib = _native.lib()
o0, o1 = sparc.generate_ordering(W, n, L * M, 0)
op = sparc.DesignOperator(W, L, M, n, o0, o1)
plan = op.plan(prec)
d_bits = _native.DeviceBuffer(B * L * 9)
d_true = _native.DeviceBuffer(B * L * 4)
d_x = _native.DeviceBuffer(B * n * es)
d_y = _native.DeviceBuffer(B * n * es)
_native.check(lib.sg_rng_bits_device(1, 0, B, L * 9, d_bits.ptr, None))
_native.check(lib.sg_bits_to_sections_device(d_bits.ptr, B, L, 9, d_true.ptr, None))
_native.check(lib.sg_amp_encode_device(plan, d_true.ptr, B, d_x.ptr, None))
_native.check(lib.sg_awgn_device(prec, 1, 0, d_x.ptr, B, n, 1.0, d_y.ptr, None))
d_map = _native.DeviceBuffer(B * L * 4)
d_tf = _native.DeviceBuffer(B * 4)
for rep in range(2):
    _native.check(lib.sg_amp_decode_device(plan, d_y.ptr, B, d_true.ptr, 1.0, 6, 1e-6, 1, d_map.ptr, d_tf.ptr,
                                           None, None, None))
_native.synchronize()
names = {0: ["setup", "gather+scatter", "FFT", "rows out", "-", "-", "-"],
         1: ["setup", "rows in", "FFT", "s update", "compact", "statistics", "s store"]}
for k, kn in ((0, "ab_stage1"), (1, "az_stage2")):
    cyc = (ct.c_double * 8)()
    nph = ct.c_int()
    _native.check(lib.sg_amp_stage_profile(plan, k, cyc, ct.byref(nph)))
    v = list(cyc)[1:]
    tot = sum(v)
    print(kn, "total %.0f cycles (%.2f us at 2.4 GHz)" % (tot, tot / 2400.0))
    for nm, c in zip(names[k], v):
        if nm != "-":
            print("   %-16s %8.0f cycles  %5.1f %%" % (nm, c, 100 * c / tot))

# occupancy: sum of workgroup durations over the span of the launch (both in
# shader-clock cycles); 256 = every CU busy with one workgroup all the time
items = ct.c_size_t()
for k, kn in ((0, "ab_stage1"), (1, "az_stage2")):
    _native.check(lib.sg_amp_stage_raw(plan, k, None, ct.byref(items)))
    raw = np.zeros((items.value, 10), np.uint64)
    _native.check(lib.sg_amp_stage_raw(plan, k, raw.ctypes.data, ct.byref(items)))
    ok = (raw[:, 8] > 0) & (raw[:, 9] > 0)
    r = raw[ok].astype(np.float64)
    st, en = r[:, 8] * 10.0, r[:, 9] * 10.0  # ns (100 MHz realtime clock)
    span = en.max() - st.min()
    dur = en - st
    cyc = r[:, 7] - r[:, 0]
    print("%s: %d workgroups, span %.1f us, duration mean %.2f us, p10/p50/p90 %.2f/%.2f/%.2f us, "
          "concurrency %.1f, shader clock %.2f GHz"
          % (kn, len(r), span / 1e3, dur.mean() / 1e3, *(np.percentile(dur, [10, 50, 90]) / 1e3),
             dur.sum() / span, cyc.sum() / dur.sum()))
