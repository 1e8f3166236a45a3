"""Per-phase shader-clock stamps of the per-codeword AMP engine (SG_AMP_TPROF):
one C2 batch decode, then the mean cycles between the stamps of the last
iteration over the workgroups (amp_cw.hip CW_TP points)."""
import ctypes as ct
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SG_AMP_TPROF"] = "1"
from ldpc_sparc_amd import _native, sparc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
L, M, R = 1024, 512, 1.5
n = int(round(L * 9 / R))
W = np.array(15.0)
o0, o1 = sparc.generate_ordering(W, n, L * M, 0)
op = sparc.DesignOperator(W, L, M, n, o0, o1)
rng = np.random.default_rng(1)
true = rng.integers(0, M, (B, L))
beta0 = np.zeros((B, L * M), np.float32)
beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
Y = op.apply(beta0.astype(np.float64), False) + rng.standard_normal((B, n))
print("engine", _native.lib().sg_amp_plan_engine(op.plan(_native.SG_F32), B))
sparc.amp_decode_batch(Y, op, 1.0, 6, true_idx=true, precision=_native.SG_F32)
lib = _native.lib()
items = ct.c_size_t()
plan = op.plan(_native.SG_F32)
_native.check(lib.sg_amp_stage_raw(plan, 0, None, ct.byref(items)))
out = np.zeros((items.value, 10), np.uint64)
_native.check(lib.sg_amp_stage_raw(plan, 0, out.ctypes.data_as(ct.POINTER(ct.c_uint64)), ct.byref(items)))
st = out[:, :8].reshape(-1)[:B * 32].reshape(B, 32).astype(np.int64)
names = {(0, 1): "Ab loop", (1, 2): "control+G", (2, 3): "Az loop", (3, 4): "merge",
         (8, 9): "Ab: zero+tw sync", (9, 10): "Ab: scatter+issue next", (10, 11): "Ab: FFT",
         (11, 12): "Ab: accumulate+sync",
         (16, 17): "Az: zero+tw sync", (17, 18): "Az: U rows+issue", (18, 19): "Az: FFT (inverse)",
         (19, 20): "Az: s_new", (20, 21): "Az: class copy", (21, 22): "Az: section stats",
         (22, 23): "Az: s store+sync"}
for (a, b), nm in names.items():
    dlt = st[:, b] - st[:, a]
    ok = (st[:, a] > 0) & (st[:, b] > 0)
    print(f"{nm:26s} {dlt[ok].mean():12.0f} cycles  (min {dlt[ok].min()}, max {dlt[ok].max()})")
