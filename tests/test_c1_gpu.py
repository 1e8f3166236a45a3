"""C1 (BASELINE.json configs[0]) at its own size: dense Gaussian design,
L=32, M=512, R=1.5, P=15, AWGN variance 1, 10 codewords
(sparc_sim_new.sparc_ldpc_sim with ldpc_bool=False, sparc_new.py:15-82,885-912,
1284-1294), against tests/golden/c1_golden.npz, written by the reference itself
(tests/golden/make_golden_c1.py).  The 192 x 16384 design of each seed is
regenerated from the seed with numpy's default_rng, as the reference does.

Bars: the CPU restatement (oracle/sparc_ref.dense_amp) reproduces the fixture's
decisions and final state (pins the oracle at this size); the drop-in's f64
path gives the fixture's user bits, decoded bits and BER exactly, and beta / s
within 1e-9 (relative to sqrt(n P_l) / max|s|); the f32 matrix-core path decodes
the same sections wherever its final s separates the section maximum by more
than 1e-3 (relative) -- every codeword fails at this rate, so near-ties decide
the rest -- and its BER lies within 0.02 of the fixture's."""
import os

import numpy as np
import pytest

from ldpc_sparc_amd import sparc_new, sparc_sim_new
from oracle import sparc_ref

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def c1():
    return np.load(os.path.join(HERE, "golden", "c1_golden.npz"))


def _params(g):
    P, R, L, M = (float(v) for v in g["sp"])
    return {'P': P, 'R': R, 'L': int(L), 'M': int(M)}


def _seeds(g):
    return [k for k in range(10) if f"c1_s{k}_seed" in g.files]


def test_c1_oracle_pinned_to_reference(c1):
    """CPU: the restatement of sparc_new.py:885-912 on the fixture's y and the
    regenerated A gives the reference's (beta, s) and decoded bits."""
    sp = _params(c1)
    L, M = sp['L'], sp['M']
    for k in _seeds(c1):
        seed = [int(v) for v in c1[f"c1_s{k}_seed"]]
        y = c1[f"c1_s{k}_y"]
        A = sparc_new.create_design_matrix(L, M, len(y), seed)
        beta, s = sparc_ref.dense_amp(y, A, sp['P'], L, M, int(c1["t_max"]))
        if f"c1_s{k}_s" in c1.files:
            np.testing.assert_allclose(s, c1[f"c1_s{k}_s"], rtol=0, atol=1e-12 * np.abs(s).max())
            np.testing.assert_allclose(beta, c1[f"c1_s{k}_beta"], rtol=0, atol=1e-12 * np.abs(beta).max())
        idx = s.reshape(L, M).argmax(1)
        bits = ((idx[:, None] >> np.arange(9)[::-1]) & 1).ravel()
        assert np.array_equal(bits, c1[f"c1_s{k}_bits_out"])


@pytest.mark.gpu
def test_c1_f64_equals_reference(c1):
    sp = _params(c1)
    for k in _seeds(c1):
        seed = [int(v) for v in c1[f"c1_s{k}_seed"]]
        bi, bo, ber = sparc_sim_new.sparc_ldpc_sim(dict(sp), None, None, False, {'t_max': int(c1["t_max"])},
                                                   float(c1["awgn_var"]), seed)
        assert np.array_equal(np.asarray(bi, np.uint8), c1[f"c1_s{k}_bits_in"])
        assert np.array_equal(np.asarray(bo, np.uint8), c1[f"c1_s{k}_bits_out"]), k
        assert ber == float(c1[f"c1_s{k}_ber"])
        if f"c1_s{k}_s" in c1.files:
            y = c1[f"c1_s{k}_y"]
            A = sparc_new.create_design_matrix(sp['L'], sp['M'], len(y), seed)
            beta, s = sparc_new.sparc_amp(y, dict(sp), {'t_max': int(c1["t_max"])}, A)
            snp = np.sqrt(len(y) * sp['P'] / sp['L'])
            np.testing.assert_allclose(beta, c1[f"c1_s{k}_beta"], rtol=0, atol=1e-9 * snp)
            np.testing.assert_allclose(s, c1[f"c1_s{k}_s"], rtol=0, atol=1e-9 * np.abs(c1[f"c1_s{k}_s"]).max())


@pytest.mark.gpu
def test_c1_f32_matrix_cores(c1):
    sp = _params(c1)
    L, M = sp['L'], sp['M']
    for k in _seeds(c1):
        seed = [int(v) for v in c1[f"c1_s{k}_seed"]]
        y = c1[f"c1_s{k}_y"]
        A = sparc_new.create_design_matrix(L, M, len(y), seed)
        beta, s = sparc_new.sparc_amp(y, dict(sp), {'t_max': int(c1["t_max"]), 'precision': 'f32'}, A)
        ref_bits = c1[f"c1_s{k}_bits_out"].reshape(L, 9)
        ref_idx = ref_bits.astype(np.int64) @ (1 << np.arange(9)[::-1])
        ss = s.reshape(L, M)
        top2 = np.sort(ss, axis=1)[:, -2:]
        clear = (top2[:, 1] - top2[:, 0]) > 1e-3 * np.abs(ss).max()
        idx = ss.argmax(1)
        assert np.array_equal(idx[clear], ref_idx[clear]), k
        bits = ((idx[:, None] >> np.arange(9)[::-1]) & 1).ravel()
        ber = np.mean(bits != c1[f"c1_s{k}_bits_in"])
        print(f"  seed {k}: {int(clear.sum())} of {L} sections clear, BER {ber:.4f} vs {float(c1[f'c1_s{k}_ber']):.4f}",
              flush=True)
        assert abs(ber - float(c1[f"c1_s{k}_ber"])) < 0.02, (k, ber)
