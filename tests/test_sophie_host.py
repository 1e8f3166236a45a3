"""CPU tests of the sparc_new / sparc_sim_new / param_calc host layer against
the reference's fixtures (tests/golden/sophie_golden.npz, made by
tests/golden/make_golden_sparc.py from the reference itself) and its own KATs
(sparc_sophie/testing/test_S_k_mapping.py)."""
import numpy as np

from ldpc_sparc_amd import param_calc, sparc_new, sparc_sim_new


def test_param_calc_golden(sophie_golden):
    g = sophie_golden
    r = param_calc.param_calc_semi_protected(1.5, 4, 0.8, 512, '802.11n', '1/2', 1 / 2, 81)
    got = [r[0], r[1], r[2], r[3]['k_ldpc'], r[3]['mults'], r[3]['L_unprotected'], r[4]]
    np.testing.assert_array_equal(np.array(got, dtype=float), g["semi_params"])
    ovr, Ls, Lsl, lengths = param_calc.param_calc(1, 6, '802.11n', '1/2', 1 / 2, 27, 1.0)
    assert Lsl == int(g["cat_L"])
    assert [lengths['k_ldpc'], lengths['mults'], lengths['L_unprotected']] == g["cat_lengths"].tolist()


def test_S_k_mapping_kat():
    """sparc_sophie/testing/test_S_k_mapping.py:31-39."""
    assert sparc_new.S_k_mapping(4) == [[0, 1], [0, 2]]
    assert sparc_new.S_k_mapping(8) == [[0, 1, 2, 3], [0, 1, 4, 5], [0, 2, 4, 6]]
    assert sparc_new.S_k_mapping(16) == [[0, 1, 2, 3, 4, 5, 6, 7], [0, 1, 2, 3, 8, 9, 10, 11],
                                         [0, 1, 4, 5, 8, 9, 12, 13], [0, 2, 4, 6, 8, 10, 12, 14]]


def test_bits_and_message_vectors():
    rng = np.random.default_rng(0)
    bits = rng.integers(0, 2, 9 * 20).astype(bool)
    mv = sparc_new.bin_arr_2_msg_vector(bits, 512, 100, 0.25)
    assert np.allclose(mv[mv != 0], np.sqrt(100 * 0.25)) and np.count_nonzero(mv) == 20
    assert np.array_equal(sparc_new.msg_vector_2_bin_arr(mv, 512), bits)
    for i in (0, 3, 255):
        assert sparc_new.bin_arr_2_int(sparc_new.int_2_bin_arr(i, 8)) == i
    assert sparc_new.bit_err_rate(np.array([0, 1, 1, 0]), np.array([0, 1, 0, 0])) == 0.25


def test_encoder_and_channel_reproduce_reference(sophie_golden):
    """sparc_ldpc_encode + awgn_channel draw the same bits, design and noise
    as the reference for the same seed (uncoded and LDPC-coded)."""
    g = sophie_golden
    for si, (L, M, R) in enumerate(((16, 64, 1.0), (32, 16, 0.8))):
        sp = {'P': 15.0, 'R': R, 'L': L, 'M': M}
        seed = [int(v) for v in g[f"dense{si}_seed"]]
        ub, tb, beta0, x, A = sparc_new.sparc_ldpc_encode(sp, None, None, False, seed)
        y = sparc_sim_new.awgn_channel(x, 1.0, seed)
        assert np.array_equal(ub, g[f"dense{si}_user_bits"])
        np.testing.assert_allclose(y, g[f"dense{si}_y"], rtol=0, atol=1e-12)
    lengths = dict(zip(['k_ldpc', 'mults', 'L_unprotected'], [int(v) for v in g["cat_lengths"]]))
    sp = {'P': 15.0, 'R': 1.0, 'L': int(g["cat_L"]), 'M': 64}
    lp = {'standard': '802.11n', 'rate': '1/2', 'z': 27, 'int_rate': 0.5, 'mults': 1}
    for si in range(2):
        seed = [int(v) for v in g[f"cat{si}_seed"]]
        ub, tb, beta0, x, A = sparc_new.sparc_ldpc_encode(sp, lp, lengths, True, seed)
        assert np.array_equal(ub, g[f"cat{si}_bits_in"])
        from ldpc_sparc_amd.ldpc import code
        c = code('802.11n', '1/2', 27)
        H = c.pcmat()
        cw = tb.reshape(-1, c.N).astype(int)
        assert not np.any((cw @ H.T) % 2)  # every protected block is a codeword
