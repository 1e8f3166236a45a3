"""Per-phase shader-clock stamps of the split per-codeword engine
(amp_cw2.hip C2_TP points, SG_AMP_TPROF): one C2 batch decode (bench design,
B = 256), then the mean / max cycles between the stamps of the last
iteration's third class of every workgroup half, and the kernels' per-class
cycles (entry to exit over the half's classes).  The stamps are compiled in
only in a diagnostic library (make -C ldpc_sparc_amd/csrc DIAG=1, or a variant
built with -DC2_STAMPS=1 loaded through LDPC_SPARC_AMD_LIB)."""
import ctypes as ct
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SG_AMP_TPROF"] = "1"
from ldpc_sparc_amd import _native, sparc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
R = float(sys.argv[2]) if len(sys.argv) > 2 else 1.5
L, M = 1024, 512
n = int(round(L * 9 / R))
W = np.array(15.0)
o0, o1 = sparc.generate_ordering(W, n, L * M, 0)
op = sparc.DesignOperator(W, L, M, n, o0, o1)
rng = np.random.default_rng(1)
true = rng.integers(0, M, (B, L))
beta0 = np.zeros((B, L * M))
beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
Y = op.apply(beta0, False) + rng.standard_normal((B, n))
lib = _native.lib()
plan = op.plan(_native.SG_F32)
sparc.amp_decode_batch(Y, op, 1.0, 6, true_idx=true, precision=_native.SG_F32)
items = ct.c_size_t()
_native.check(lib.sg_amp_stage_raw(plan, 0, None, ct.byref(items)))
out = np.zeros((items.value, 10), np.uint64)
_native.check(lib.sg_amp_stage_raw(plan, 0, out.ctypes.data_as(ct.POINTER(ct.c_uint64)), ct.byref(items)))
st = out[:, :8].reshape(-1)[:2 * B * 64].reshape(2 * B, 64).astype(np.int64)
Qh = 32
names = {(0, 8): "Ab: loads + prev accumulate + barrier", (8, 1): "Ab: scatter chunk 0",
         (1, 2): "Ab: scatter chunk 1", (2, 3): "Ab: barrier", (3, 6): "Ab: FFT", (0, 6): "Ab: class (to FFT end)",
         (32, 33): "Az: rows", (33, 34): "Az: barrier", (34, 35): "Az: FFT (inverse)", (35, 36): "Az: s_new",
         (36, 37): "Az: s store", (37, 38): "Az: barrier", (38, 39): "Az: class copy + barrier",
         (39, 40): "Az: section stats", (40, 41): "Az: closing barrier", (32, 41): "Az: class total"}
for (a, b), nm in names.items():
    dlt = st[:, b] - st[:, a]
    ok = (st[:, a] > 0) & (st[:, b] > 0) & (dlt > 0)
    if ok.any():
        print(f"{nm:30s} {dlt[ok].mean():10.0f} cycles  (min {dlt[ok].min()}, max {dlt[ok].max()}, n {ok.sum()})")
for (a, b), nm in {(10, 11): "cw2_ab per class", (42, 43): "cw2_az per class"}.items():
    dlt = (st[:, b] - st[:, a]) / Qh
    ok = (st[:, a] > 0) & (st[:, b] > 0) & (dlt > 0)
    if ok.any():
        print(f"{nm:30s} {dlt[ok].mean():10.0f} cycles  (min {dlt[ok].min():.0f}, max {dlt[ok].max():.0f})")
