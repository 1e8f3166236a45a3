"""f32 vs reference t_final / psi for every golden SPARC seed (diagnostic)."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from ldpc_sparc_amd import _native, sparc  # noqa: E402
from sparc_cases import all_seeds, design  # noqa: E402

g = np.load("tests/golden/sparc_golden.npz")
for name, cp, dp, var, si in all_seeds():
    key = f"{name}_s{si}"
    W, L, M, n, o0, o1 = design(g, name, si, cp, var)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    dp = dict(dp)
    sparc.check_decode_params(dp)
    true = sparc.bin_arr_2_msg_vector(g[key + "_bits"], M).reshape(L, M).argmax(1)
    out = {}
    for prec in (_native.SG_F64, _native.SG_F32):
        mi, tf, nmse, psi = sparc.amp_decode_batch(g[key + "_y"][None], op, var, dp['t_max'], dp['rtol'],
                                                   dp['phi_est_method'], true[None], precision=prec)
        out[prec] = (int(tf[0]), np.asarray(psi[0]).ravel(), np.asarray(nmse[0]).ravel())
    print(key, "ref", int(g[key + "_t_final"]), "f64", out[_native.SG_F64][0], "f32", out[_native.SG_F32][0],
          "psi64", np.array2string(out[_native.SG_F64][1][:3], precision=9),
          "psi32", np.array2string(out[_native.SG_F32][1][:3], precision=9),
          "nmse32 tail", np.array2string(out[_native.SG_F32][2][-3:], precision=3), flush=True)
