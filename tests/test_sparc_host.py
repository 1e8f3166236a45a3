"""CPU tests of the SPARC host layer (parameter handling, bits and message
vectors, base matrices, orderings, channel) against reference fixtures."""
import numpy as np
import pytest

from ldpc_sparc_amd import sparc, sparc_sim
from sparc_cases import SPARC_CASES, all_seeds


def test_check_code_params_rewrites_dict():
    cp = {'P': 15.0, 'R': 1.5, 'L': 32, 'M': 512, 'junk': 1}
    sparc.check_code_params(cp)
    assert cp == {'complex': False, 'modulated': False, 'power_allocated': False,
                  'spatially_coupled': False, 'P': 15.0, 'R': 1.5, 'L': 32, 'M': 512}
    with pytest.raises(Exception, match="Need code parameters"):
        sparc.check_code_params({'P': 15.0, 'R': 1.5, 'L': 32})
    with pytest.raises(AssertionError):
        sparc.check_code_params({'P': 15.0, 'R': 1.5, 'L': 32, 'M': 500})
    with pytest.raises(AssertionError, match="B must divide L"):
        sparc.check_code_params({'P': 15.0, 'R': 1.5, 'L': 30, 'M': 64, 'power_allocated': True,
                                 'B': 4, 'R_PA_ratio': 1.0})


def test_check_decode_params_defaults():
    dp = {'t_max': 25}
    sparc.check_decode_params(dp)
    assert dp == {'t_max': 25, 'rtol': 1e-6, 'phi_est_method': 1}
    with pytest.raises(AssertionError):
        sparc.check_decode_params({'t_max': 1})


def test_bits_round_trip_golden(sparc_golden):
    for k, M in ((9216, 512), (96, 4)):
        bits = sparc.rnd_bin_arr(k, [11, 22])
        assert np.array_equal(bits, sparc_golden[f"rt_{k}_{M}_bits"])
        mv = sparc.bin_arr_2_msg_vector(bits, M)
        assert np.array_equal(np.flatnonzero(mv), sparc_golden[f"rt_{k}_{M}_idx"])
        assert np.array_equal(sparc.msg_vector_2_bin_arr(mv, M), bits)
    sparc.test_bin_arr_msg_vector()
    for i in (0, 1, 5, 511):
        assert sparc.bin_arr_2_int(sparc.int_2_bin_arr(i, 9)) == i
    assert sparc.int_2_bin_arr(5, 4).tolist() == [False, True, False, True]


def test_base_matrices_golden(sparc_golden):
    assert np.array_equal(sparc.pa_iterative(15.0, 1.0, 16, 1.4), sparc_golden["pa_16"])
    assert np.array_equal(sparc.sc_basic(np.array(15.0), 6, 32), sparc_golden["sc_6_32"])
    assert np.array_equal(sparc.sc_basic(sparc.pa_iterative(15.0, 1.0, 2, 0.96), 2, 4),
                          sparc_golden["scpa_2_4_q"])


@pytest.mark.parametrize("name,cp,dp,var,si", list(all_seeds()))
def test_orderings_and_channel_golden(sparc_golden, name, cp, dp, var, si):
    """generate_ordering reproduces the reference's RandomState draws block by
    block; bits and AWGN noise come from the same seeds (sparc.py:27-45,
    sparc_sim.py:194-198)."""
    key = f"{name}_s{si}"
    seed = [int(v) for v in sparc_golden[key + "_seed"]]
    sparc.check_code_params(cp)
    L, M, R = cp['L'], cp['M'], cp['R']
    tmp = cp.copy()
    tmp.update({'awgn_var': var})
    W = sparc.create_base_matrix(**tmp)
    bit_len = int(round(L * np.log2(M)))
    bits = sparc.rnd_bin_arr(bit_len, seed)
    assert np.array_equal(bits, sparc_golden[key + "_bits"])
    n = int(round(bit_len / R))
    if W.ndim == 2:
        n = int(round(n / W.shape[0])) * W.shape[0]
    assert n == int(sparc_golden[key + "_n"])
    if W.ndim == 0:
        Mr, Mc = n, L * M
    elif W.ndim == 1:
        Mr, Mc = n, L * M // W.size
    else:
        Mr, Mc = n // W.shape[0], L * M // W.shape[1]
    o0, o1 = sparc.generate_ordering(W, Mr, Mc, seed)
    g0, g1 = sparc_golden[key + "_order0"], sparc_golden[key + "_order1"]
    if W.ndim == 0:
        assert np.array_equal(o0, g0[0]) and np.array_equal(o1, g1[0])
    elif W.ndim == 1:
        assert np.array_equal(o0, g0) and np.array_equal(o1, g1)
    else:
        nz = [(r, c) for r in range(W.shape[0]) for c in range(W.shape[1]) if W[r, c] != 0]
        assert np.array_equal(np.stack([o0[rc] for rc in nz]), g0)
        assert np.array_equal(np.stack([o1[rc] for rc in nz]), g1)
    x = sparc_golden[key + "_x"]
    y = sparc_sim.awgn_channel(x, var, seed)
    assert np.array_equal(y, sparc_golden[key + "_y"])


def test_calc_ber_ser():
    b0 = np.zeros(12); b0[[1, 5, 8]] = 1
    b1 = np.zeros(12); b1[[1, 6, 8]] = 1
    ser, loc, num = sparc_sim.calc_ser(b0, b1, 3)
    assert ser == 1 / 3 and loc.tolist() == [1] and num == 1
    assert sparc_sim.calc_ber(np.array([1, 0, 1], bool), np.array([1, 1, 1], bool)) == 1 / 3
