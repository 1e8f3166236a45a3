"""C3 A/B probe: bench.py's C3 workload (802.11n r1/2 z=81, 4096 codewords, f32
min-sum, 50 iterations; LLRs of bench.py bp_setup) at 1.0 / 1.5 / 2.0 dB,
median kernel time per launch over `reps` launches (HIP events on the library
stream) and a hash of (app, it) so that variants can be checked bit for bit.
One JSON line per run; the library is whatever LDPC_SPARC_AMD_LIB names."""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpc_sparc_amd import _native  # noqa: E402
from ldpc_sparc_amd.ldpc import code  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = 4096
c = code("802.11n", "1/2", 81)
lib = _native.lib()
g = c._device_graph()
out = {"lib": os.environ.get("LDPC_SPARC_AMD_LIB", "default"),
       "kernel": None}
for ebn0 in (1.0, 1.5, 2.0):
    rng = np.random.default_rng(2000)
    X = c.encode_batch(rng.integers(0, 2, (B, c.K)))
    R = c.K / c.N
    s2 = 1 / (2 * R * 10 ** (ebn0 / 10))
    ch = 2 * ((1 - 2 * X) + np.sqrt(s2) * rng.standard_normal(X.shape)) / s2
    d_ch = _native.DeviceBuffer.from_array(ch.astype(np.float32))
    d_app = _native.DeviceBuffer(B * c.N * 4)
    d_it = _native.DeviceBuffer(B * 4)
    ms = []
    for r in range(reps + 2):
        e0, e1 = _native.Event(), _native.Event()
        e0.record()
        _native.check(lib.sg_ldpc_decode_device(g, _native.SG_MINSUM, _native.SG_F32, d_ch.ptr, B, 50, 0.7,
                                                d_app.ptr, d_it.ptr, None))
        e1.record()
        if r >= 2:
            ms.append(e0.elapsed_ms(e1))
    app = d_app.download(np.zeros((B, c.N), np.float32))
    it = d_it.download(np.zeros(B, np.int32))
    h = hashlib.sha256(app.tobytes() + it.tobytes()).hexdigest()[:16]
    cwit = int(np.where(it < 50, it + 1, 50).sum())
    med = float(np.median(ms))
    out[f"{ebn0}"] = {"ms": med, "ms_min": float(np.min(ms)), "codewords_per_s": B / med * 1e3,
                      "codeword_iterations": cwit, "hash": h,
                      "lds_bound_frac": cwit * 16 * c.Nmsg / (med * 1e-3) / 52.4e12}
print(json.dumps(out), flush=True)
