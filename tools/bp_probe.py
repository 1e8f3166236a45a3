"""C3 BP probe for counter runs: the bench's C3 batch (802.11n r1/2 z=81,
4096 codewords, Eb/N0 2.0 dB, f32 min-sum, 50 iterations) decoded `reps`
times on the device, printing the kernel name and the time per launch.

  python tools/bp_probe.py [reps] [ebn0]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpc_sparc_amd import _native  # noqa: E402
from ldpc_sparc_amd.ldpc import code  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
ebn0 = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
c = code("802.11n", "1/2", 81)
B = 4096
rng = np.random.default_rng(2000)
X = c.encode_batch(rng.integers(0, 2, (B, c.K)))
s2 = 1 / (2 * (c.K / c.N) * 10 ** (ebn0 / 10))
ch = 2 * ((1 - 2 * X) + np.sqrt(s2) * rng.standard_normal(X.shape)) / s2
lib = _native.lib()
g = c._device_graph()
d_ch = _native.DeviceBuffer.from_array(ch.astype(np.float32))
d_app, d_it = _native.DeviceBuffer(B * c.N * 4), _native.DeviceBuffer(B * 4)


def run():
    _native.check(lib.sg_ldpc_decode_device(g, _native.SG_MINSUM, _native.SG_F32, d_ch.ptr, B, 50, 0.7,
                                            d_app.ptr, d_it.ptr, None))


run()
_native.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    run()
_native.synchronize()
el = time.perf_counter() - t0
its = d_it.download(np.zeros(B, np.int32))
_ = el = time.perf_counter() - t0
ex = np.where(its < 50, its + 1, 50)
print(c.decode_kernel("minsum"), f"{el / reps * 1e3:.3f} ms per launch (host clock)",
      f"avg executed iterations {ex.mean():.2f}", flush=True)
