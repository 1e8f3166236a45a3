"""Throughput of the C2 decode (L=1024, M=512, R=1.5, t_max=25) at B
codewords and the given precision, under whatever engine knobs the
environment sets (bench.py refuses them): codewords/s and mean iterations.
usage: amp_probe.py [B] [f32|f64]"""
import sys
import time

import numpy as np

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
op = sparc.DesignOperator(W, L, M, n, o0, o1)  # (owns the plan: keep it alive)
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


def run():
    _native.check(lib.sg_amp_decode_device(plan, d_y.ptr, B, d_true.ptr, 1.0, 25, 1e-6, 1, d_map.ptr, d_tf.ptr,
                                           None, None, None))


run()
_native.synchronize()
reps = 3
t0 = time.perf_counter()
for _ in range(reps):
    run()
_native.synchronize()
el = time.perf_counter() - t0
tf = d_tf.download(np.zeros(B, np.int32))
mp = d_map.download(np.zeros(B * L, np.int32))
print("cw/s %.1f  iterations %.2f  ms/decode %.2f  map-digest %d" % (B * reps / el, tf.mean(), el / reps * 1e3,
                                                                   int(mp.astype(np.int64).sum())))
