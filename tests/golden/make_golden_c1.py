"""C1 fixture (BASELINE.json configs[0]): the reference's dense Gaussian-design
simulation at L=32, M=512, R=1.5, P=15, AWGN variance 1, 10 codewords
(sparc_sophie/sparc_sim_new.py:12-23 with ldpc_bool=False: sparc_new.py:15-51
encode, :885-912 AMP with t_max=25, :1099-1116 MAP, :1319-1341 bits), written to
tests/golden/c1_golden.npz.

Build-container only (imports /root/reference via ref_harness).  The 192 x 16384
design matrix of each seed is NOT stored: tests regenerate it from the seed with
numpy's default_rng (create_design_matrix, sparc_new.py:1284-1294), which is
what the reference does.  Stored per seed: the seed, the received word y, the
user bits, the decoded bits and the BER; for the first two seeds also the
reference's final (beta, s) of sparc_amp.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402

SP = {'P': 15.0, 'R': 1.5, 'L': 32, 'M': 512}
DP = {'t_max': 25}
AWGN_VAR = 1.0
SEEDS = [[101 + k, 32] for k in range(10)]


def make_c1():
    ldpc, sparc, sparc_sim, sparc_new, sim_new, param_calc = ref_harness.import_reference()
    out = {"sp": np.array([SP['P'], SP['R'], SP['L'], SP['M']]), "awgn_var": np.array(AWGN_VAR),
           "t_max": np.array(DP['t_max'])}
    for k, seed in enumerate(SEEDS):
        bi, bo, ber = sim_new.sparc_ldpc_sim(dict(SP), None, None, False, dict(DP), AWGN_VAR, seed)
        # the same encode/channel again for the received word and the AMP state
        ub, tb, beta0, x, A = sparc_new.sparc_ldpc_encode(dict(SP), None, None, False, seed)
        y = sim_new.awgn_channel(x, AWGN_VAR, seed)
        key = f"c1_s{k}"
        out[key + "_seed"] = np.array(seed)
        out[key + "_y"] = y
        out[key + "_bits_in"] = np.asarray(bi).astype(np.uint8)
        out[key + "_bits_out"] = np.asarray(bo).astype(np.uint8)
        out[key + "_ber"] = np.array(ber)
        if k < 2:
            beta, s = sparc_new.sparc_amp(y, dict(SP), dict(DP), A)
            out[key + "_beta"] = beta
            out[key + "_s"] = s
        print(key, "n", len(y), "ber", ber)
    np.savez_compressed(os.path.join(HERE, "c1_golden.npz"), **out)
    print("wrote c1_golden.npz", sum(v.nbytes for v in out.values()) / 1e6, "MB raw")


if __name__ == "__main__":
    make_c1()
