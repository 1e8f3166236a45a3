"""C4 (spatially coupled, omega=6, Lambda=32, L=1024, M=512, R=1.5) in-process
A/B of two engines selected by SG_AMP_ENGINE at plan creation: same inputs,
decodes interleaved; reports timing and decision agreement.
usage: python tools/c4_ab.py ENGINE_A ENGINE_B [B] [reps] [t_max]   ('' = default engine)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from ldpc_sparc_amd import _native, sparc  # noqa: E402

ea, eb = sys.argv[1], sys.argv[2]
B = int(sys.argv[3]) if len(sys.argv) > 3 else 64
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
t_max = int(sys.argv[5]) if len(sys.argv) > 5 else 40
L, M, P, omega, Lam, R = 1024, 512, 15.0, 6, 32, 1.5
W = sparc.sc_basic(np.array(P), omega, Lam)
Lr, Lc = W.shape
n = int(round(L * 9 / R))
Mr = int(round(n / Lr))
n = Mr * Lr
o0, o1 = sparc.generate_ordering(W, Mr, L * M // Lc, 0)
plans = {}
for e in (ea, eb):
    if e:
        os.environ["SG_AMP_ENGINE"] = e
    else:
        os.environ.pop("SG_AMP_ENGINE", None)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    plans[e] = (op, op.plan(_native.SG_F32))
lib = _native.lib()
d_bits = _native.DeviceBuffer(B * L * 9)
d_true = _native.DeviceBuffer(B * L * 4)
d_x = _native.DeviceBuffer(B * n * 4)
d_y = _native.DeviceBuffer(B * n * 4)
_native.check(lib.sg_rng_bits_device(1, 0, B, L * 9, d_bits.ptr, None))
_native.check(lib.sg_bits_to_sections_device(d_bits.ptr, B, L, 9, d_true.ptr, None))
_native.check(lib.sg_amp_encode_device(plans[eb][1], d_true.ptr, B, d_x.ptr, None))
_native.check(lib.sg_awgn_device(_native.SG_F32, 1, 0, d_x.ptr, B, n, 1.0, d_y.ptr, None))
out = {}
for r in range(reps):
    for e in (ea, eb):
        d_map = _native.DeviceBuffer(B * L * 4)
        d_tf = _native.DeviceBuffer(B * 4)
        d_nm = _native.DeviceBuffer(B * t_max * Lc * 8)
        _native.synchronize()
        t0 = time.perf_counter()
        _native.check(lib.sg_amp_decode_device(plans[e][1], d_y.ptr, B, d_true.ptr, 1.0, t_max, 1e-6, 1,
                                               d_map.ptr, d_tf.ptr, d_nm.ptr, None, None))
        _native.synchronize()
        dt = time.perf_counter() - t0
        mp = d_map.download(np.zeros((B, L), np.int32))
        tf = d_tf.download(np.zeros(B, np.int32))
        nm = d_nm.download(np.zeros((B, t_max, Lc)))
        tr = d_true.download(np.zeros((B, L), np.int32))
        out[e] = (mp, tf, nm)
        print(f"engine={e or 'default'} rep {r}: {dt*1e3:.1f} ms  {B/dt:.1f} cw/s  iters={tf.mean():.2f} "
              f"sec_err={(mp != tr).sum()} cw_err={(mp != tr).any(1).sum()}", flush=True)
(ma, ta, na), (mb, tb_, nb) = out[ea], out[eb]
print("t_final equal:", np.array_equal(ta, tb_), " max |dt|:", np.abs(ta - tb_).max(),
      " map equal:", np.array_equal(ma, mb), " sections differing:", int((ma != mb).sum()))
k = min(5, t_max)
print("nmse[:5] max abs diff:", float(np.abs(na[:, :k] - nb[:, :k]).max()))
