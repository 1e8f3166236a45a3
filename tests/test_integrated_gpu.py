"""GPU parity tests of the AMP <-> BP integrated decoders (integrated.hip,
sg_integrated_decode) against the reference's outputs
(tests/golden/integrated_golden.npz, made by running the reference) and the
CPU restatement oracle/integrated_ref.py.

Bars (stated tolerances):
  * bp_output_to_beta_estimate: bit-exact in double (same product order);
  * update_using_bp_probs: within 1e-13 relative;
  * differentiated_eta_calc(_posteriors): within 1e-11 of the largest
    magnitude (closed form vs the reference's loops);
  * the four decoders in double: information bits identical to the
    reference on every fixture, tau^2 of every iteration within 1e-9;
  * batched decoding equals one-at-a-time decoding;
  * float: same bits as double on the fixture the reference decodes.
"""
import numpy as np
import pytest

from ldpc_sparc_amd import _native, sparc_new, sparc_sim_new
from ldpc_sparc_amd.ldpc import code
from oracle import integrated_ref
from test_oracle_pin import integrated_case

pytestmark = pytest.mark.gpu

MODES = {"naive": "naive", "naivepost": "naive_posteriors", "integ": "integrated", "integpost": "integrated_posteriors"}


def test_bp_output_to_beta_exact(integrated_golden):
    g = integrated_golden
    out = sparc_new.bp_output_to_beta_estimate(g["bpb_probs"], 72, 512, 2.5)
    np.testing.assert_array_equal(out, g["bpb_beta"])


def test_update_using_bp_probs(integrated_golden):
    g = integrated_golden
    out = sparc_new.update_using_bp_probs(g["upd_gamma"], g["upd_alpha"], 2.5, 512)
    np.testing.assert_allclose(out, g["upd_beta"], rtol=1e-13, atol=1e-300)


@pytest.mark.parametrize("post", [False, True])
def test_differentiated_eta(integrated_golden, post):
    g = integrated_golden
    L, M, n, P_l, tau2 = g["deta_cfg"]
    L, M, n = int(L), int(M), int(n)
    S_k = sparc_new.S_k_mapping(M)
    if post:
        out = sparc_new.differentiated_eta_calc_posteriors(g["deta_gamma"], g["deta_beta"], g["deta_vk"],
                                                           g["deta_vk0"], g["deta_alpha"], tau2, L, M, S_k, n, P_l)
        ref = g["deta_post_out"]
    else:
        out = sparc_new.differentiated_eta_calc(g["deta_beta"], g["deta_vk"], g["deta_vk0"], g["deta_alpha"], tau2, L,
                                                M, S_k, n, P_l)
        ref = g["deta_out"]
    assert np.max(np.abs(out - ref)) <= 1e-11 * np.max(np.abs(ref))


@pytest.mark.parametrize("key", ["naive", "naivepost", "integ", "integpost"])
@pytest.mark.parametrize("ci", [0, 1])
def test_decoder_matches_reference(integrated_golden, key, ci):
    k = f"{key}{ci}"
    y, A, L, M, P, graph, N, K, t_max = integrated_case(integrated_golden, k)
    design = sparc_new.DenseDesign(A, P, L, M)
    c = code('802.11n', '1/2', 27)
    bits, tau2 = sparc_new.integrated_decode_batch(y[None], design, c, MODES[key], t_max)
    np.testing.assert_allclose(tau2[0], integrated_golden[k + "_tau2"], rtol=1e-9)
    assert np.array_equal(bits[0], integrated_golden[k + "_bits_out"]), k
    design.release()


def test_sim_dropins_match_reference(integrated_golden):
    """The sparc_sim_new simulations (the reference's call surface) end to end."""
    g = integrated_golden
    L, M, P, R, k_ldpc, mults, t_max = [v.item() for v in g["dec_cfg"]]
    sp = {'P': P, 'R': R, 'L': int(L), 'M': int(M)}
    lp = {'standard': '802.11n', 'rate': '1/2', 'z': 27, 'int_rate': 0.5, 'mults': int(mults)}
    lengths = {'k_ldpc': int(k_ldpc), 'mults': int(mults), 'L_unprotected': 0}
    sims = {"naive": sparc_sim_new.sparc_ldpc_naive_sim, "naivepost": sparc_sim_new.sparc_ldpc_naive_sim_posteriors,
            "integ": sparc_sim_new.sparc_ldpc_integrated_sim,
            "integpost": sparc_sim_new.sparc_ldpc_integrated_posteriors_sim}
    for key, sim in sims.items():
        k = f"{key}0"
        seed = [int(v) for v in g[k + "_seed"]]
        bi, bo, ber = sim(sp, lp, lengths, True, {'t_max': int(t_max)}, float(g[k + "_var"]), seed)
        assert np.array_equal(np.asarray(bo).astype(np.uint8), g[k + "_bits_out"]), key
        assert ber == float(g[k + "_ber"]), key


@pytest.mark.parametrize("key", ["naivepost", "integ"])
def test_batched_equals_single(integrated_golden, key):
    cases = [integrated_case(integrated_golden, f"{key}{ci}") for ci in (0, 1)]
    y0, A, L, M, P, graph, N, K, t_max = cases[0]
    c = code('802.11n', '1/2', 27)
    design = sparc_new.DenseDesign(A, P, L, M)
    rng = np.random.default_rng(3)
    Y = np.stack([y0, y0 + 0.3 * rng.standard_normal(y0.size), y0 + 0.6 * rng.standard_normal(y0.size)])
    bits, tau2 = sparc_new.integrated_decode_batch(Y, design, c, MODES[key], t_max)
    for b in range(3):
        b1, t1 = sparc_new.integrated_decode_batch(Y[b:b + 1], design, c, MODES[key], t_max)
        assert np.array_equal(b1[0], bits[b])
        np.testing.assert_allclose(t1[0], tau2[b], rtol=1e-12)
    design.release()


def test_oracle_agrees_on_perturbed_input(integrated_golden):
    """Beyond the fixtures: a received word the reference was not run on,
    checked against the CPU restatement."""
    y, A, L, M, P, graph, N, K, t_max = integrated_case(integrated_golden, "integ1")
    y = y + 0.2 * np.random.default_rng(9).standard_normal(y.size)
    ref_bits, ref_tau = integrated_ref.decode("integ", y, A, P, L, M, graph, N, K, t_max)
    design = sparc_new.DenseDesign(A, P, L, M)
    bits, tau2 = sparc_new.integrated_decode_batch(y[None], design, code('802.11n', '1/2', 27), "integrated", t_max)
    np.testing.assert_allclose(tau2[0], ref_tau, rtol=1e-9)
    assert np.array_equal(bits[0], ref_bits)
    design.release()


def test_float_decodes_the_decodable_fixture(integrated_golden):
    y, A, L, M, P, graph, N, K, t_max = integrated_case(integrated_golden, "integ0")
    assert float(integrated_golden["integ0_ber"]) == 0.0
    design = sparc_new.DenseDesign(A, P, L, M)
    bits, _ = sparc_new.integrated_decode_batch(y[None], design, code('802.11n', '1/2', 27), "integrated", t_max,
                                                precision=_native.SG_F32)
    assert np.array_equal(bits[0], integrated_golden["integ0_bits_out"])
    design.release()
