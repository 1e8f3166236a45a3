"""Section errors of the per-codeword, staged and f64 engines on one C2-size batch."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpc_sparc_amd import _native, sparc  # noqa: E402

P = float(sys.argv[1]) if len(sys.argv) > 1 else 31.0
R = float(sys.argv[2]) if len(sys.argv) > 2 else 1.5
L = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
M = 512
n = int(round(L * 9 / R))
W = np.array(P)
o0, o1 = sparc.generate_ordering(W, n, L * M, 21)
rng = np.random.default_rng(9)
B = 4
true = rng.integers(0, M, (B, L))
beta0 = np.zeros((B, L * M))
beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
op = sparc.DesignOperator(W, L, M, n, o0, o1)
Y = op.apply(beta0, False) + rng.standard_normal((B, n))
m64, t64, n64, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true)
print("f64   ", (m64 != true).sum(1), t64, n64[:, :6].round(4).tolist())
os.environ["SG_AMP_ENGINE"] = "staged"
os_ = sparc.DesignOperator(W, L, M, n, o0, o1)
ms, ts, ns, _ = sparc.amp_decode_batch(Y, os_, 1.0, 25, true_idx=true, precision=_native.SG_F32)
print("staged", (ms != true).sum(1), ts, ns[:, :6].round(4).tolist())
os.environ["SG_AMP_ENGINE"] = "cw"
oc = sparc.DesignOperator(W, L, M, n, o0, o1)
mc, tc, nc, _ = sparc.amp_decode_batch(Y, oc, 1.0, 25, true_idx=true, precision=_native.SG_F32)
print("cw", _native.lib().sg_amp_plan_engine(oc.plan(_native.SG_F32), B), (mc != true).sum(1), tc,
      nc[:, :6].round(4).tolist())
# operator check at the cw plan's P (staged kernels on the P = 8192 tables)
x = rng.standard_normal(L * M)
a = oc.apply(x, False, _native.SG_F32)
b = op.Ab(x)
print("Ab rel err (P=8192 tables)", np.abs(a - b).max() / np.abs(b).max())
