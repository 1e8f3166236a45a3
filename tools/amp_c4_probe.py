"""C4: spatially coupled SPARC (omega=6, Lambda=32, L=1024, M=512, R=1.5,
P=15, awgn_var=1, t_max=40; sparc_demo_sc_decode_wave) decoded on the GPU.
args: B reps [R] [L]  (L = 2048: the notebook geometry, w = 2^16, the two-class block engine)"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from ldpc_sparc_amd import _native, sparc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
R = float(sys.argv[3]) if len(sys.argv) > 3 else 1.5
L = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
M, P, omega, Lam = 512, 15.0, 6, 32
W = sparc.sc_basic(np.array(P), omega, Lam)
Lr, Lc = W.shape
n = int(round(L * 9 / R))
Mr = int(round(n / Lr))
n = Mr * Lr
t0 = time.time()
o0, o1 = sparc.generate_ordering(W, Mr, L * M // Lc, 0)
op = sparc.DesignOperator(W, L, M, n, o0, o1)
plan = op.plan(_native.SG_F32)
print(f"W {Lr}x{Lc}, n={n}, plan {time.time() - t0:.1f} s", flush=True)
lib = _native.lib()
d_bits = _native.DeviceBuffer(B * L * 9)
d_true = _native.DeviceBuffer(B * L * 4)
d_x = _native.DeviceBuffer(B * n * 4)
d_y = _native.DeviceBuffer(B * n * 4)
_native.check(lib.sg_rng_bits_device(1, 0, B, L * 9, d_bits.ptr, None))
_native.check(lib.sg_bits_to_sections_device(d_bits.ptr, B, L, 9, d_true.ptr, None))
_native.check(lib.sg_amp_encode_device(plan, d_true.ptr, B, d_x.ptr, None))
_native.check(lib.sg_awgn_device(_native.SG_F32, 1, 0, d_x.ptr, B, n, 1.0, d_y.ptr, None))
d_map = _native.DeviceBuffer(B * L * 4)
d_tf = _native.DeviceBuffer(B * 4)
d_cnt = _native.DeviceBuffer(32)
for r in range(reps):
    d_cnt.zero()
    _native.synchronize()
    t0 = time.time()
    _native.check(lib.sg_amp_decode_device(plan, d_y.ptr, B, d_true.ptr, 1.0, 40, 1e-6, 1, d_map.ptr, d_tf.ptr,
                                           None, None, None))
    _native.check(lib.sg_amp_count_errors_device(d_map.ptr, d_true.ptr, d_tf.ptr, B, L, 9, d_cnt.ptr, None))
    _native.synchronize()
    dt = time.time() - t0
    cnt = d_cnt.download(np.zeros(4, np.int64))
    print(f"rep {r}: {dt*1e3:.1f} ms  {B/dt:.1f} cw/s  sec_err={cnt[0]} cw_err={cnt[2]} iters={cnt[3]/B:.2f}",
          flush=True)
