"""Quick BP throughput probe (802.11n r1/2 z=81, random codewords)."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from ldpc_sparc_amd import _native
from ldpc_sparc_amd.ldpc import code

c = code("802.11n", "1/2", 81)
L = _native.lib()
g = c._device_graph()
rng = np.random.default_rng(0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
for ebn0 in (1.0, 2.0):
    R = c.K / c.N; s2 = 1 / (2 * R * 10 ** (ebn0 / 10))
    X = c.encode_batch(rng.integers(0, 2, (B, c.K)))
    ch = (2 * ((1 - 2 * X) + np.sqrt(s2) * rng.standard_normal(X.shape)) / s2)
    for prec, dt, nm in ((_native.SG_F32, np.float32, "f32"), (_native.SG_F64, np.float64, "f64")):
        for kind in ("minsum", "sumprod2"):
            d_ch = _native.DeviceBuffer.from_array(ch.astype(dt))
            d_app = _native.DeviceBuffer(ch.size * np.dtype(dt).itemsize)
            d_it = _native.DeviceBuffer(B * 4)
            e0, e1 = _native.Event(), _native.Event()
            for rep in range(3):
                e0.record()
                _native.check(L.sg_ldpc_decode_device(g, _native.DECTYPES[kind], prec, d_ch.ptr, B, 50, 0.7, d_app.ptr, d_it.ptr, None))
                e1.record()
                ms = e0.elapsed_ms(e1)
            it = d_it.download(np.zeros(B, np.int32))
            app = d_app.download(np.zeros(ch.shape, dt))
            fer = np.mean(np.any((app < 0) != X, axis=1))
            execd = np.where(it < 50, it + 1, 50).sum()
            print(f"EbN0={ebn0} {nm} {kind}: {ms:.3f} ms  {B/ms*1e3:.0f} cw/s  {execd/ms*1e3/1e6:.2f} M cw-it/s  avg_it={it.mean():.2f} FER={fer:.4f}")
