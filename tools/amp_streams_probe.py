"""C2 AMP decode split into NS concurrent batches (own plan workspace, own HIP
stream, own host thread) on one GPU: does stream concurrency fill the
serialized phases of the stage kernels?  args: B NS reps"""
import ctypes as ct
import sys
import threading
import time

import numpy as np

sys.path.insert(0, ".")
from ldpc_sparc_amd import _native, sparc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
NS = int(sys.argv[2]) if len(sys.argv) > 2 else 2
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
L, M, R = 1024, 512, 1.5
n = int(round(L * 9 / R))
W = np.array(15.0)
lib = _native.lib()
o0, o1 = sparc.generate_ordering(W, n, L * M, 0)
ops = [sparc.DesignOperator(W, L, M, n, o0, o1) for _ in range(NS)]
plans = [op.plan(_native.SG_F32) for op in ops]
streams = []
for _ in range(NS):
    s = ct.c_void_p()
    _native.check(lib.sg_stream_create(ct.byref(s)))
    streams.append(s)
Bs = B // NS
work = []
for k in range(NS):
    d_bits = _native.DeviceBuffer(Bs * L * 9)
    d_true = _native.DeviceBuffer(Bs * L * 4)
    d_x = _native.DeviceBuffer(Bs * n * 4)
    d_y = _native.DeviceBuffer(Bs * n * 4)
    _native.check(lib.sg_rng_bits_device(1, k, Bs, L * 9, d_bits.ptr, None))
    _native.check(lib.sg_bits_to_sections_device(d_bits.ptr, Bs, L, 9, d_true.ptr, None))
    _native.check(lib.sg_amp_encode_device(plans[k], d_true.ptr, Bs, d_x.ptr, None))
    _native.check(lib.sg_awgn_device(_native.SG_F32, 1, k, d_x.ptr, Bs, n, 1.0, d_y.ptr, None))
    work.append(dict(y=d_y, true=d_true, map=_native.DeviceBuffer(Bs * L * 4), tf=_native.DeviceBuffer(Bs * 4)))
_native.synchronize()


def run(k):
    w = work[k]
    _native.check(lib.sg_amp_decode_device(plans[k], w["y"].ptr, Bs, w["true"].ptr, 1.0, 25, 1e-6, 1, w["map"].ptr,
                                           w["tf"].ptr, None, None, streams[k]))
    _native.check(lib.sg_stream_synchronize(streams[k]))


for r in range(reps):
    _native.device_synchronize()
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(k,)) for k in range(NS)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    _native.device_synchronize()
    dt = time.perf_counter() - t0
    its = sum(int(w["tf"].download(np.zeros(Bs, np.int32)).sum()) for w in work)
    print(f"NS={NS} B={B} rep {r}: {dt*1e3:.1f} ms  {B/dt:.1f} cw/s  avg it {its/B:.2f}", flush=True)
