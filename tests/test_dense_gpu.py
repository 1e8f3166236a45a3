"""GPU parity tests of the dense Gaussian-design AMP engine (dense.hip) and the
AMP -> BP glue through the C ABI, against the reference's own outputs
(tests/golden/sophie_golden.npz), its KATs (sparc_sophie/testing/
test_beta_estimate_to_bp_probs.py) and the CPU restatement oracle/sparc_ref.py.

Bars: f64 AMP state within 1e-9 (relative to sqrt(n P_l)) of the reference and
identical decisions; f32 (matrix-core GEMMs) products within 2e-5 relative of
a float64 product, decisions identical on decodable codewords; glue
probabilities within 1e-12; BP hard decisions identical."""
import numpy as np
import pytest

from ldpc_sparc_amd import _native, sparc_new, sparc_sim_new
from ldpc_sparc_amd.ldpc import code
from oracle import sparc_ref

pytestmark = pytest.mark.gpu


def _dense_case(g, si):
    L, M, R = ((16, 64, 1.0), (32, 16, 0.8))[si]
    sp = {'P': 15.0, 'R': R, 'L': L, 'M': M}
    seed = [int(v) for v in g[f"dense{si}_seed"]]
    ub, tb, beta0, x, A = sparc_new.sparc_ldpc_encode(sp, None, None, False, seed)
    return sp, g[f"dense{si}_y"], A


@pytest.mark.parametrize("si", [0, 1])
def test_dense_amp_f64_vs_reference(sophie_golden, si):
    g = sophie_golden
    sp, y, A = _dense_case(g, si)
    beta, s = sparc_new.sparc_amp(y, sp, {'t_max': 25}, A)
    scale = np.sqrt(len(y) * sp['P'] / sp['L'])
    np.testing.assert_allclose(beta, g[f"dense{si}_beta"], rtol=0, atol=1e-9 * scale)
    np.testing.assert_allclose(s, g[f"dense{si}_s"], rtol=0, atol=1e-9 * np.abs(g[f"dense{si}_s"]).max())
    bits = sparc_new.sparc_ldpc_decode(y, sp, None, {'t_max': 25}, False, None, A)
    assert np.array_equal(bits, g[f"dense{si}_bits_out"])


@pytest.mark.parametrize("si", [0, 1])
def test_dense_amp_f32_matrix_cores(sophie_golden, si):
    g = sophie_golden
    sp, y, A = _dense_case(g, si)
    beta, s = sparc_new.sparc_amp(y, sp, {'t_max': 25, 'precision': 'f32'}, A)
    scale = np.sqrt(len(y) * sp['P'] / sp['L'])
    ref = g[f"dense{si}_beta"]
    # same section decisions; soft values within f32 accuracy
    M = sp['M']
    assert np.array_equal(s.reshape(-1, M).argmax(1), g[f"dense{si}_s"].reshape(-1, M).argmax(1))
    assert np.max(np.abs(beta - ref)) < 1e-3 * scale


def test_gemm_products_f32_vs_f64():
    """Both matrix-core GEMMs at a size with ragged tiles: s = A^T y (t_max=1,
    NN product) and one full iteration (NT split-K product A beta)."""
    rng = np.random.default_rng(3)
    L, M, n, B = 40, 64, 333, 9
    A = rng.normal(0, 1 / np.sqrt(n), (n, L * M))
    d = sparc_new.DenseDesign(A, 15.0, L, M)
    Y = rng.standard_normal((B, n)) * 2
    b1, s1 = sparc_new.dense_amp_batch(Y, d, 1, _native.SG_F32)
    ref_s1 = Y @ A
    assert np.max(np.abs(s1 - ref_s1)) < 2e-5 * np.abs(ref_s1).max()
    b2, s2 = sparc_new.dense_amp_batch(Y, d, 2, _native.SG_F32)
    b2d, s2d = sparc_new.dense_amp_batch(Y, d, 2, _native.SG_F64)
    for b in range(B):
        rb, rs = sparc_ref.dense_amp(Y[b], A, 15.0, L, M, 2)
        np.testing.assert_allclose(s2d[b], rs, rtol=0, atol=1e-10 * np.abs(rs).max())
        np.testing.assert_allclose(b2d[b], rb, rtol=0, atol=1e-10 * np.abs(rb).max())
        assert np.max(np.abs(s2[b] - rs)) < 5e-4 * np.abs(rs).max()


def test_dense_encode_device_matches_host():
    rng = np.random.default_rng(5)
    L, M, n, B = 32, 32, 200, 5
    A = rng.normal(0, 1 / np.sqrt(n), (n, L * M))
    d = sparc_new.DenseDesign(A, 15.0, L, M)
    idx = rng.integers(0, M, (B, L)).astype(np.int32)
    beta0 = np.zeros((B, L * M))
    beta0[np.arange(B)[:, None], np.arange(L) * M + idx] = np.sqrt(n * 15.0 / L)
    for prec, tol in ((_native.SG_F64, 1e-12), (_native.SG_F32, 1e-5)):
        d_idx = _native.DeviceBuffer.from_array(idx)
        d_x = _native.DeviceBuffer(B * n * (8 if prec == _native.SG_F64 else 4))
        _native.check(_native.lib().sg_dense_encode_device(d.plan(prec), d_idx.ptr, B, d_x.ptr, None))
        _native.synchronize()
        x = d_x.download(np.zeros((B, n), np.float64 if prec == _native.SG_F64 else np.float32))
        ref = beta0 @ A.T
        assert np.max(np.abs(x - ref)) < tol * np.abs(ref).max()


def test_single_iteration_vs_oracle():
    rng = np.random.default_rng(7)
    L, M, n = 16, 32, 100
    sp = {'P': 15.0, 'L': L, 'M': M, 'R': 1.0}
    A = rng.normal(0, 1 / np.sqrt(n), (n, L * M))
    y = rng.standard_normal(n) * 3
    beta = np.abs(rng.standard_normal(L * M))
    z = rng.standard_normal(n)
    tau = 1.7
    b1, z1, t1 = sparc_new.sparc_amp_single_it(sp, y, A, A.T, beta, z, tau)
    # restatement of sparc_new.py:975-990
    Ab = A @ beta
    ons = (z / tau) * (15.0 - np.sum(beta ** 2) / n)
    zr = y - Ab + ons
    s = beta + A.T @ zr
    tr = np.sum(zr ** 2) / n
    br = sparc_ref.dense_mmse_estimator(s, tr, n, 15.0 / L, M)
    np.testing.assert_allclose(z1, zr, rtol=1e-12, atol=1e-12)
    assert abs(t1 - tr) < 1e-12 * tr
    np.testing.assert_allclose(b1, br, rtol=0, atol=1e-10 * np.abs(br).max())


def test_glue_kats_and_reference(sophie_golden):
    """beta_estimate_to_bp_probs KATs (test_beta_estimate_to_bp_probs.py:27-58)
    and the reference's glue + BP outputs."""
    t1 = sparc_new.beta_estimate_to_bp_probs(np.array([1, 0, 0, 0, 0, 0, 1, 0, 1, 0, 0, 0.]), 3, 4, 1)
    assert np.array_equal(t1, np.array([1, 1, 0, 1, 1, 1.]))
    t2 = sparc_new.beta_estimate_to_bp_probs(np.array([.7, .1, .1, .1, .1, .1, .7, .1, .7, .1, .1, .1]), 3, 4, 1)
    assert np.array_equal(np.where(t2 < 0.5, 1, 0), [0, 0, 1, 0, 0, 0])
    t3 = sparc_new.beta_estimate_to_bp_probs(np.array([.5, .2, .1, .1, .1, .1, .7, .1, .2, .4, .2, .2]), 3, 4, 1)
    assert np.array_equal(np.where(t3 < 0.5, 1, 0), [0, 0, 1, 0, 0, 1])
    g = sophie_golden
    probs = sparc_new.beta_estimate_to_bp_probs(g["glue_beta"], 72, 512, 2.5)
    np.testing.assert_allclose(probs, g["glue_probs"], rtol=1e-12, atol=1e-14)
    c = code('802.11n', '1/2', 27)
    _, hard = sparc_new.ldpc_bp(g["glue_probs"], c, 200, True)
    assert np.array_equal(hard, g["glue_hard_bits"])
    soft, _ = sparc_new.ldpc_bp(g["glue_probs"], c, 6, False)
    np.testing.assert_allclose(soft, g["glue_soft_probs"], rtol=1e-9, atol=1e-12)


def test_llr_layout_for_bp():
    """Device LLRs of a section range land where the batched BP expects them."""
    rng = np.random.default_rng(2)
    B, L, M = 3, 20, 16
    beta = rng.random((B, L * M))
    beta /= beta.reshape(B, L, M).sum(-1).repeat(M, axis=1).reshape(B, L * M)
    logM = 4
    l0, nl = 5, 12
    d_b = _native.DeviceBuffer.from_array(beta)
    ld = nl * logM + 7
    d_l = _native.DeviceBuffer(B * ld * 8)
    d_l.zero()
    _native.check(_native.lib().sg_beta_to_llr_device(_native.SG_F64, d_b.ptr, B, L, M, 1.0, l0, nl, ld, 0,
                                                      d_l.ptr, None))
    _native.synchronize()
    llr = d_l.download(np.zeros((B, ld)))
    for b in range(B):
        p = sparc_ref.beta_to_bit_probs(beta[b, l0 * M:(l0 + nl) * M], nl, M, 1.0)
        p = np.clip(p, 1e-15, 1 - 1e-15)
        np.testing.assert_allclose(llr[b, :nl * logM], np.log(p) - np.log(1 - p), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("si", [0, 1])
def test_concatenated_sim_vs_reference(sophie_golden, si):
    """sparc_ldpc_sim end to end (sparc_sim_new.py:12-23): AMP, glue, BP."""
    g = sophie_golden
    lengths = dict(zip(['k_ldpc', 'mults', 'L_unprotected'], [int(v) for v in g["cat_lengths"]]))
    sp = {'P': 15.0, 'R': 1.0, 'L': int(g["cat_L"]), 'M': 64}
    lp = {'standard': '802.11n', 'rate': '1/2', 'z': 27, 'int_rate': 0.5, 'mults': 1}
    seed = [int(v) for v in g[f"cat{si}_seed"]]
    bi, bo, ber = sparc_sim_new.sparc_ldpc_sim(sp, lp, lengths, True, {'t_max': 25}, float(g[f"cat{si}_var"]),
                                               seed)
    assert np.array_equal(bi, g[f"cat{si}_bits_in"])
    assert np.array_equal(bo, g[f"cat{si}_bits_out"])
    assert ber == float(g[f"cat{si}_ber"])
