"""C5 GEMM probe: the dense-design AMP of bench.py's concat line (L=1024, M=512,
n=9216, B=256, f32 matrix cores) for `t` iterations, per-launch time of the
two GEMM kinds (HIP events around every launch, Profiler phase dense_gemm) and a
hash of the final (beta, s) so that variants can be checked bit for bit.
One JSON line; the library is whatever LDPC_SPARC_AMD_LIB names."""
import ctypes as ct
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpc_sparc_amd import _native  # noqa: E402
from ldpc_sparc_amd.pipeline import ConcatPipeline  # noqa: E402

t_max = int(sys.argv[1]) if len(sys.argv) > 1 else 4
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
B = 256
pipe = ConcatPipeline(1024, 512, 9216, 15.0, 160, 4, ldpc=("802.11n", "1/2", 81), design_seed=0, precision="f32",
                      t_max=t_max, bp_its=200)
pipe.make_batch_device(B, 0.5, 2024, 7)
lib = _native.lib()
lib.sg_dense_amp_device(pipe.plan, pipe.d_y.ptr, B, t_max, None, None, None)
_native.synchronize()
prof = _native.Profiler(1)
t0 = time.perf_counter()
for _ in range(reps):
    _native.check(lib.sg_dense_amp_device(pipe.plan, pipe.d_y.ptr, B, t_max, None, None, None))
_native.synchronize()
wall = time.perf_counter() - t0
ph = prof.stop()
d_beta, d_s = ct.c_void_p(), ct.c_void_p()
_native.check(lib.sg_dense_state_device(pipe.plan, ct.byref(d_beta), ct.byref(d_s)))
h = hashlib.sha256()
for d in (d_beta, d_s):
    a = np.empty((8, 1024 * 512), np.float32)
    _native.check(lib.sg_memcpy_d2h(_native.ptr(a), d, a.nbytes, None))
    h.update(a.tobytes())
out = {"lib": os.environ.get("LDPC_SPARC_AMD_LIB", "default"), "t_max": t_max, "reps": reps,
       "wall_ms_per_decode": 1e3 * wall / reps, "hash_rows0_7": h.hexdigest()[:16]}
for k, (ms, cnt) in sorted(ph.items()):
    out[k] = {"ms_per_launch": ms / max(cnt, 1), "launches": cnt}
g = ph.get("dense_gemm")
if g:
    flops = 2.0 * B * 9216 * 1024 * 512
    out["gemm_tflops"] = flops / (g[0] / g[1] * 1e-3) / 1e12
    out["gemm_frac_of_157.3"] = out["gemm_tflops"] / 157.3
pipe.design.release()
print(json.dumps(out), flush=True)
