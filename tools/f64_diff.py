"""Max |NMSE difference| per iteration between the f64 split engine (forced) and the staged f64 engine on
one C2 batch (B=48, R=1.5): python tools/f64_diff.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpc_sparc_amd import _native, sparc  # noqa: E402

L, M, R, B = 1024, 512, 1.5, 48
n = int(round(L * 9 / R))
W = np.array(15.0)
o0, o1 = sparc.generate_ordering(W, n, L * M, 41)
op = sparc.DesignOperator(W, L, M, n, o0, o1)
rng = np.random.default_rng(5)
true = rng.integers(0, M, (B, L)).astype(np.int32)
beta0 = np.zeros((B, L * M))
beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
Y = op.apply(beta0, False) + rng.standard_normal((B, n))
res = {}
for eng in ("cw", "staged"):
    os.environ["SG_AMP_ENGINE"] = eng
    res[eng] = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true)
d = np.abs(res["cw"][2][:, :, 0] - res["staged"][2][:, :, 0]).max(0)
print(os.environ.get("LDPC_SPARC_AMD_LIB", "cur"), "t_final equal", bool(np.array_equal(res["cw"][1], res["staged"][1])),
      "max |dNMSE| per iteration:", " ".join("%.1e" % x for x in d[:25]))
