"""GPU parity tests of the SPARC AMP engine (amp_dct.hip) through the C ABI.

Bars (stated tolerances):
  * design operators Ab / Az: double plan within 1e-12 of the reference
    operator (relative to the output's max magnitude), float plan within 2e-6;
  * double-precision decode: identical t_final and MAP decision as the
    reference on every golden seed, NMSE per iteration within 1e-9;
  * float decode: identical MAP decision on seeds the reference decodes
    (BER 0), t_final within +-2, NMSE per iteration within 1e-3 absolute for
    the first iterations;
  * full size (L=1024, M=512, w=2^20): operators as above; R=1.3 codewords
    decode with BER 0; NMSE trajectory tracks the CPU restatement.
"""
import ctypes

import numpy as np
import pytest

from ldpc_sparc_amd import _native, sparc, sparc_sim
from oracle import sparc_ref
from sparc_cases import SPARC_CASES, all_seeds, design

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


@pytest.mark.parametrize("name,cp,dp,var,si", [c for c in all_seeds() if c[4] == 0])
def test_operators_vs_reference(sparc_golden, name, cp, dp, var, si):
    W, L, M, n, o0, o1 = design(sparc_golden, name, si, cp, var)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
    rng = np.random.default_rng(1)
    X = rng.standard_normal((3, L * M))
    Y = rng.standard_normal((3, n))
    for prec, tol in ((_native.SG_F64, 1e-12), (_native.SG_F32, 2e-6)):
        gx = op.apply(X, False, prec)
        gy = op.apply(Y, True, prec)
        for b in range(3):
            assert _rel(gx[b], Ab(X[b])) < tol, (name, prec)
            assert _rel(gy[b], Az(Y[b])) < tol, (name, prec)


@pytest.mark.parametrize("w_exp,Mr", [(4, 5), (5, 12), (7, 40), (10, 300), (13, 1000), (16, 6000)])
def test_operator_sizes(w_exp, Mr):
    """Transform sizes from w=16 to 2^16 with random orders (odd P/Q splits)."""
    w = 2 ** w_exp
    Mc = w // 2 + 3 if w > 16 else 9
    L, M = Mc, 1
    rng = np.random.RandomState(w_exp)
    idx0 = np.arange(1, w, dtype=np.uint32); rng.shuffle(idx0)
    idx1 = np.arange(1, w, dtype=np.uint32); rng.shuffle(idx1)
    o0, o1 = idx0[:Mr], idx1[:Mc]
    W = np.array(3.0)
    op = sparc.DesignOperator(W, L, M, Mr, o0, o1)
    assert op.w == w
    Ab, Az = sparc_ref.dct_operators(W, L, M, Mr, o0, o1)
    x = rng.standard_normal(L * M)
    y = rng.standard_normal(Mr)
    assert _rel(op.Ab(x), Ab(x)) < 1e-12
    assert _rel(op.Az(y), Az(y)) < 1e-12


@pytest.mark.parametrize("name,cp,dp,var,si", list(all_seeds()))
def test_decode_f64_matches_reference(sparc_golden, name, cp, dp, var, si):
    key = f"{name}_s{si}"
    W, L, M, n, o0, o1 = design(sparc_golden, name, si, cp, var)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    dp = dict(dp)
    sparc.check_decode_params(dp)
    true = sparc.bin_arr_2_msg_vector(sparc_golden[key + "_bits"], M).reshape(L, M).argmax(1)
    mi, tf, nmse, psi = sparc.amp_decode_batch(sparc_golden[key + "_y"][None], op, var, dp['t_max'],
                                               dp['rtol'], dp['phi_est_method'], true[None])
    assert tf[0] == int(sparc_golden[key + "_t_final"]), key
    assert np.array_equal(mi[0], sparc_golden[key + "_map"]), key
    ref_nmse = sparc_golden[key + "_nmse"]
    np.testing.assert_allclose(nmse[0].reshape(ref_nmse.shape), ref_nmse, rtol=0, atol=1e-9, err_msg=key)


@pytest.mark.parametrize("name,cp,dp,var,si", list(all_seeds()))
def test_sparc_sim_dropin_matches_reference(sparc_golden, name, cp, dp, var, si):
    """sparc_sim (the reference's call surface) end to end on the GPU."""
    key = f"{name}_s{si}"
    seed = [int(v) for v in sparc_golden[key + "_seed"]]
    res = sparc_sim.sparc_sim(dict(cp), dict(dp), var, seed)
    assert res['ber'] == float(sparc_golden[key + "_sim_ber"])
    assert res['ser'] == float(sparc_golden[key + "_sim_ser"])
    assert res['t_final'] == int(sparc_golden[key + "_sim_t"])
    assert res['detect'] == float(sparc_golden[key + "_sim_detect"])
    assert res['num_of_sec_errs'] == int(sparc_golden[key + "_sim_nsec"])
    assert np.array_equal(res['loc_of_sec_errs'], sparc_golden[key + "_sim_locs"])


@pytest.mark.parametrize("name,cp,dp,var,si", list(all_seeds()))
def test_decode_f32_tolerance(sparc_golden, name, cp, dp, var, si):
    key = f"{name}_s{si}"
    W, L, M, n, o0, o1 = design(sparc_golden, name, si, cp, var)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    dp = dict(dp)
    sparc.check_decode_params(dp)
    true = sparc.bin_arr_2_msg_vector(sparc_golden[key + "_bits"], M).reshape(L, M).argmax(1)
    mi, tf, nmse, psi = sparc.amp_decode_batch(sparc_golden[key + "_y"][None], op, var, dp['t_max'],
                                               dp['rtol'], dp['phi_est_method'], true[None],
                                               precision=_native.SG_F32)
    ref_map = sparc_golden[key + "_map"]
    ref_nmse = sparc_golden[key + "_nmse"].reshape(nmse[0].shape)
    decoded = float(sparc_golden[key + "_sim_ber"]) == 0.0
    if decoded:
        assert np.array_equal(mi[0], ref_map), key
        assert abs(int(tf[0]) - int(sparc_golden[key + "_t_final"])) <= 2, key
    k = 4
    np.testing.assert_allclose(nmse[0][:k], ref_nmse[:k], rtol=0, atol=1e-3, err_msg=key)


def test_batched_decode_equals_single():
    """A batch of codewords sharing one design decodes exactly like one-by-one."""
    cp = {'P': 15.0, 'R': 1.3, 'L': 64, 'M': 64}
    sparc.check_code_params(cp)
    L, M = cp['L'], cp['M']
    n = int(round(L * 6 / 1.3))
    W = np.array(15.0)
    o0, o1 = sparc.generate_ordering(W, n, L * M, 5)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    rng = np.random.default_rng(0)
    true = rng.integers(0, M, (9, L))
    beta0 = np.zeros((9, L * M))
    beta0[np.arange(9)[:, None], np.arange(L) * M + true] = 1
    Y = op.apply(beta0, False) + rng.standard_normal((9, n))
    for prec in (_native.SG_F64, _native.SG_F32):
        mb, tb, nb, pb = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true, precision=prec)
        for b in (0, 4, 8):
            m1, t1, n1, p1 = sparc.amp_decode_batch(Y[b:b + 1], op, 1.0, 25, true_idx=true[b:b + 1],
                                                    precision=prec)
            assert np.array_equal(m1[0], mb[b]) and t1[0] == tb[b]
            assert np.array_equal(n1[0], nb[b])


def test_standalone_estimators():
    rng = np.random.default_rng(3)
    s = rng.standard_normal(64 * 32) * 5
    tau = 0.7
    np.testing.assert_allclose(sparc.msg_vector_mmse_estimator(s, tau, 32),
                               sparc_ref.mmse_estimator(s, tau, 32), rtol=1e-12, atol=1e-300)
    assert np.array_equal(sparc.msg_vector_map_estimator(s, 32), sparc_ref.map_estimator(s, 32))


def _c2_design(seed, R=1.5, P=15.0):
    L, M = 1024, 512
    n = int(round(L * 9 / R))
    W = np.array(P)
    o0, o1 = sparc.generate_ordering(W, n, L * M, seed)
    return W, L, M, n, o0, o1


def test_full_size_operators():
    W, L, M, n, o0, o1 = _c2_design(11)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    assert op.w == 2 ** 20
    Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
    rng = np.random.default_rng(2)
    x = rng.standard_normal(L * M)
    y = rng.standard_normal(n)
    assert _rel(op.Ab(x), Ab(x)) < 1e-12
    assert _rel(op.Az(y), Az(y)) < 1e-12
    assert _rel(op.apply(x, False, _native.SG_F32), Ab(x)) < 5e-6
    assert _rel(op.apply(y, True, _native.SG_F32), Az(y)) < 5e-6


def test_full_size_decode_r13_f32_and_f64():
    """C2 geometry at R=1.3 (a decodable rate): every codeword of a batch
    decodes with zero section errors in both precisions, and the f32 NMSE
    trajectory tracks the f64 one."""
    W, L, M, n, o0, o1 = _c2_design(21, R=1.3)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    rng = np.random.default_rng(8)
    B = 4
    true = rng.integers(0, M, (B, L))
    beta0 = np.zeros((B, L * M))
    beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
    Y = op.apply(beta0, False) + rng.standard_normal((B, n))
    m64, t64, n64, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true)
    m32, t32, n32, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true, precision=_native.SG_F32)
    assert np.array_equal(m64, true)
    assert np.array_equal(m32, true)
    assert np.all(np.abs(t64 - t32) <= 2)
    np.testing.assert_allclose(n32[:, :8], n64[:, :8], atol=2e-3)


def test_full_size_decode_f64_vs_oracle():
    """One C2 codeword (R=1.5, the benchmark point) against the CPU restatement
    (float128 softmax): identical t_final and MAP decisions, NMSE within 1e-8."""
    W, L, M, n, o0, o1 = _c2_design(31)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
    rng = np.random.RandomState(4)
    true = rng.randint(0, M, L)
    beta0 = np.zeros(L * M)
    beta0[np.arange(L) * M + true] = 1
    y = Ab(beta0) + rng.randn(n)
    rb, rt, rn, rp = sparc_ref.amp(y, W, L, M, n, 1.0, 25, Ab, Az, beta0)
    mi, tf, nm, ps = sparc.amp_decode_batch(y[None], op, 1.0, 25, true_idx=true[None])
    assert tf[0] == rt
    np.testing.assert_allclose(nm[0, :, 0], rn, atol=1e-8)
    assert np.mean(mi[0] != np.argmax(rb.reshape(L, M), 1)) < 0.01


def _c4_design(seed, R=1.5, L=1024):
    """C4 geometry (sparc_demo_sc_decode_wave): spatially coupled omega=6,
    Lambda=32, L=1024, M=512 -> W 37x32, Mr=166, n=6142, Mc=16384, w=2^15."""
    M, P, omega, Lam = 512, 15.0, 6, 32
    W = sparc.sc_basic(np.array(P), omega, Lam)
    Lr, Lc = W.shape
    n = int(round(L * 9 / R))
    Mr = int(round(n / Lr))
    n = Mr * Lr
    o0, o1 = sparc.generate_ordering(W, Mr, L * M // Lc, seed)
    return W, L, M, n, o0, o1


def _c4_batch(op, B, seed):
    rng = np.random.default_rng(seed)
    true = rng.integers(0, op.M, (B, op.L))
    beta0 = np.zeros((B, op.L * op.M))
    beta0[np.arange(B)[:, None], np.arange(op.L) * op.M + true] = 1
    return op.apply(beta0, False) + rng.standard_normal((B, op.n)), true


def test_c4_block_engine_vs_oracle():
    """One C4 codeword through the f32 block engine (amp_block.hip) against
    the CPU restatement (float128 softmax): t_final within +-2, the same MAP
    decisions on all but 0.5 % of the sections, NMSE within 2e-3 over the
    first 10 iterations (f32 bar of the module docstring)."""
    W, L, M, n, o0, o1 = _c4_design(5)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    assert op.w == 2 ** 15 and W.shape == (37, 32)
    Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
    rng = np.random.RandomState(6)
    true = rng.randint(0, M, L)
    beta0 = np.zeros(L * M)
    beta0[np.arange(L) * M + true] = 1
    y = Ab(beta0) + rng.randn(n)
    rb, rt, rn, rp = sparc_ref.amp(y, W, L, M, n, 1.0, 40, Ab, Az, beta0)
    mi, tf, nm, ps = sparc.amp_decode_batch(y[None], op, 1.0, 40, true_idx=true[None], precision=_native.SG_F32)
    assert abs(int(tf[0]) - int(rt)) <= 2, (tf[0], rt)
    assert np.mean(mi[0] != np.argmax(rb.reshape(L, M), 1)) < 0.005
    np.testing.assert_allclose(nm[0, :10], np.asarray(rn).reshape(40, -1)[:10], atol=2e-3)


def test_c4_block_engine_batch_vs_oracle():
    """A 32-codeword C4 batch through the shipped block engine (the bench's sc
    line runs it at B = 256) against the CPU restatement on every codeword, the
    restatement fanned out over the host cores (oracle/cpu_pool.py): the same
    MAP decision on every section but at most 0.01 %, stopping iterations within
    one (f32 against float64 with a float128 softmax), the same decoded
    codewords."""
    from oracle import cpu_pool
    W, L, M, n, o0, o1 = _c4_design(5)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    B = 32
    rng = np.random.default_rng(17)
    true = rng.integers(0, M, (B, L)).astype(np.int32)
    beta0 = np.zeros((B, L * M))
    beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
    Y = op.apply(beta0, False) + rng.standard_normal((B, n))
    mi, tf, nm, _ = sparc.amp_decode_batch(Y, op, 1.0, 40, true_idx=true, precision=_native.SG_F32)
    res, _ = cpu_pool.amp_decode(cpu_pool.host_cores(), W, L, M, n, o0, o1, Y, true, 40)
    assert sorted(res) == list(range(B))
    cpu_map = np.stack([res[b][0] for b in range(B)])
    cpu_tf = np.array([res[b][1] for b in range(B)])
    assert np.mean(mi != cpu_map) <= 1e-4
    assert np.max(np.abs(tf.astype(int) - cpu_tf)) <= 1, (tf, cpu_tf)
    assert np.array_equal((mi == true).all(1), (cpu_map == true).all(1))


def test_c4_block_engine_vs_general_engine(monkeypatch):
    """The block engine and the general four-step engine (SG_AMP_ENGINE=general)
    decode the same C4 batch to the same decisions and stopping iterations."""
    W, L, M, n, o0, o1 = _c4_design(7)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Y, true = _c4_batch(op, 8, 9)
    mb, tb_, nb, _ = sparc.amp_decode_batch(Y, op, 1.0, 40, true_idx=true, precision=_native.SG_F32)
    monkeypatch.setenv("SG_AMP_ENGINE", "general")
    og = sparc.DesignOperator(W, L, M, n, o0, o1)
    mg, tg, ng, _ = sparc.amp_decode_batch(Y, og, 1.0, 40, true_idx=true, precision=_native.SG_F32)
    assert np.all(np.abs(tb_ - tg) <= 1)
    assert np.mean(mb != mg) < 1e-3
    np.testing.assert_allclose(nb[:, :10], ng[:, :10], atol=1e-4)
    assert np.mean(mb != true) < 0.05  # the decode wave runs through at R = 1.5


def test_c4_two_class_form_vs_single_class(monkeypatch):
    """C4 through the two-class block engine at P = 2^13 (amp_block2.hip, two
    512-thread workgroups per CU; SG_AMP_BLOCK=two-class) against the default
    single-class engine (amp_block.hip) on the same batch: stopping iterations
    within one, decisions and the first NMSE values agree (f32)."""
    W, L, M, n, o0, o1 = _c4_design(7)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Y, true = _c4_batch(op, 8, 9)
    monkeypatch.delenv("SG_AMP_BLOCK", raising=False)
    m1, t1, n1, _ = sparc.amp_decode_batch(Y, op, 1.0, 40, true_idx=true, precision=_native.SG_F32)
    monkeypatch.setenv("SG_AMP_BLOCK", "two-class")
    o2 = sparc.DesignOperator(W, L, M, n, o0, o1)
    m2, t2, n2, _ = sparc.amp_decode_batch(Y, o2, 1.0, 40, true_idx=true, precision=_native.SG_F32)
    assert _native.amp_last_decode(o2.plan(_native.SG_F32))["engine"] == 3
    assert np.all(np.abs(t1 - t2) <= 1)
    assert np.mean(m1 != m2) < 1e-3
    np.testing.assert_allclose(n1[:, :10], n2[:, :10], atol=1e-4)
    assert np.mean(m2 != true) < 0.05


def _notebook_design(seed):
    """The notebook's own geometry (sparc_demo_sc_decode_wave.ipynb cell 1):
    spatially coupled omega=6, Lambda=32, L=2048, M=512, R=1.5, P=15 ->
    W 37x32, Mr=332, n=12284, Mc=32768, w=2^16 (the general four-step path)."""
    return _c4_design(seed, L=2048)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_notebook_geometry_vs_oracle(precision):
    """The reference's only published M=512 configuration, one codeword of the
    notebook's geometry against the CPU restatement of sparc.py:883-999 (f32
    through the two-class block engine, f64 through the general path):
    f64 -- same t_final and MAP decisions, NMSE within 1e-9; f32 -- t_final
    within 2, decisions on all but 0.5 % of the sections, NMSE within 2e-3
    over the first 10 iterations."""
    W, L, M, n, o0, o1 = _notebook_design(13)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    assert op.w == 2 ** 16 and W.shape == (37, 32) and n == 12284
    prec = _native.SG_F64 if precision == "f64" else _native.SG_F32
    # f32: the two-class block engine (amp_block2.hip); f64: the general path
    assert _native.lib().sg_amp_plan_engine(op.plan(prec), 1) == (3 if precision == "f32" else 0)
    Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
    rng = np.random.RandomState(14)
    true = rng.randint(0, M, L)
    beta0 = np.zeros(L * M)
    beta0[np.arange(L) * M + true] = 1
    y = Ab(beta0) + rng.randn(n)
    rb, rt, rn, rp = sparc_ref.amp(y, W, L, M, n, 1.0, 40, Ab, Az, beta0)
    mi, tf, nm, ps = sparc.amp_decode_batch(y[None], op, 1.0, 40, true_idx=true[None], precision=prec)
    ref_map = np.argmax(rb.reshape(L, M), 1)
    rn = np.asarray(rn).reshape(40, -1)
    if precision == "f64":
        assert int(tf[0]) == int(rt)
        assert np.array_equal(mi[0], ref_map)
        np.testing.assert_allclose(nm[0], rn, atol=1e-9)
    else:
        assert abs(int(tf[0]) - int(rt)) <= 2, (tf[0], rt)
        assert np.mean(mi[0] != ref_map) < 0.005
        np.testing.assert_allclose(nm[0, :10], rn[:10], atol=2e-3)
    assert np.mean(ref_map != true) < 0.01  # the decode wave runs through at this size


def test_notebook_block2_vs_general_engine(monkeypatch):
    """The two-class block engine (amp_block2.hip) and the general four-step
    engine (SG_AMP_ENGINE=general) decode the same batch of the notebook's
    geometry to the same decisions and stopping iterations (f32)."""
    W, L, M, n, o0, o1 = _notebook_design(17)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Y, true = _c4_batch(op, 8, 19)
    monkeypatch.delenv("SG_AMP_ENGINE", raising=False)
    mb, tb_, nb, _ = sparc.amp_decode_batch(Y, op, 1.0, 40, true_idx=true, precision=_native.SG_F32)
    assert _native.amp_last_decode(op.plan(_native.SG_F32))["engine"] == 3
    monkeypatch.setenv("SG_AMP_ENGINE", "general")
    og = sparc.DesignOperator(W, L, M, n, o0, o1)
    mg, tg, ng, _ = sparc.amp_decode_batch(Y, og, 1.0, 40, true_idx=true, precision=_native.SG_F32)
    assert _native.amp_last_decode(og.plan(_native.SG_F32))["engine"] == 0
    assert np.all(np.abs(tb_ - tg) <= 1)
    assert np.mean(mb != mg) < 1e-3
    np.testing.assert_allclose(nb[:, :10], ng[:, :10], atol=1e-4)
    assert np.mean(mb != true) < 0.01


def test_notebook_block2_operators():
    """The two-class block engine's forward and adjoint operators (through
    decoding-free applications would need the general plan; here: one AMP
    iteration pair) -- checked through the first NMSE value, which depends only
    on Ab and Az of the first iteration, against the CPU restatement."""
    W, L, M, n, o0, o1 = _notebook_design(21)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
    rng = np.random.RandomState(22)
    true = rng.randint(0, M, L)
    beta0 = np.zeros(L * M)
    beta0[np.arange(L) * M + true] = 1
    y = Ab(beta0) + rng.randn(n)
    rb, rt, rn, rp = sparc_ref.amp(y, W, L, M, n, 1.0, 3, Ab, Az, beta0)
    mi, tf, nm, ps = sparc.amp_decode_batch(y[None], op, 1.0, 3, true_idx=true[None], precision=_native.SG_F32)
    np.testing.assert_allclose(nm[0], np.asarray(rn).reshape(3, -1), atol=2e-4)


# ---- per-codeword engine (amp_cw.hip): opt-in with SG_AMP_ENGINE=cw (plan
# creation builds its tables, decode runs it)

@pytest.mark.parametrize("name,cp,dp,var,si", [c for c in all_seeds() if c[1].get('M') == 512 and
                                              not c[1].get('power_allocated')])
def test_cw_engine_f32_vs_reference(sparc_golden, monkeypatch, name, cp, dp, var, si):
    """Regular designs with w >= 2^15 through the per-codeword engine, against
    the reference's own outputs (the bar of test_decode_f32_tolerance)."""
    key = f"{name}_s{si}"
    W, L, M, n, o0, o1 = design(sparc_golden, name, si, cp, var)
    if np.ndim(W) != 0:
        pytest.skip("one transform per design only")
    monkeypatch.setenv("SG_AMP_ENGINE", "cw")
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    dp = dict(dp)
    sparc.check_decode_params(dp)
    true = sparc.bin_arr_2_msg_vector(sparc_golden[key + "_bits"], M).reshape(L, M).argmax(1)
    mi, tf, nmse, psi = sparc.amp_decode_batch(sparc_golden[key + "_y"][None], op, var, dp['t_max'],
                                               dp['rtol'], dp['phi_est_method'], true[None],
                                               precision=_native.SG_F32)
    assert _native.lib().sg_amp_plan_engine(op.plan(_native.SG_F32), 1) == 2, "per-codeword engine not selected"
    ref_map = sparc_golden[key + "_map"]
    ref_nmse = sparc_golden[key + "_nmse"].reshape(nmse[0].shape)
    if float(sparc_golden[key + "_sim_ber"]) == 0.0:
        assert np.array_equal(mi[0], ref_map), key
        assert abs(int(tf[0]) - int(sparc_golden[key + "_t_final"])) <= 2, key
    np.testing.assert_allclose(nmse[0][:4], ref_nmse[:4], rtol=0, atol=1e-3, err_msg=key)


@pytest.mark.parametrize("L,R,P", [(512, 1.2, 15.0), (1024, 1.3, 15.0)])
def test_cw_engine_full_size_vs_staged_and_f64(monkeypatch, L, R, P):
    """Designs where AMP decodes (L=512, M=512, R=1.2, w=2^19; and the C2
    geometry at R=1.3, n=7089, whose 14 needed indices per thread put two X
    slots in registers; with flat power n=6144 does not decode at any P, see
    the R=1.5 test below): the per-codeword engine decodes every codeword,
    agrees with the staged engine on the decisions and tracks the f64 NMSE."""
    M = 512
    n = int(round(L * 9 / R))
    W = np.array(P)
    o0, o1 = sparc.generate_ordering(W, n, L * M, 21)
    rng = np.random.default_rng(9)
    B = 6
    true = rng.integers(0, M, (B, L))
    beta0 = np.zeros((B, L * M))
    beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Y = op.apply(beta0, False) + rng.standard_normal((B, n))
    m64, t64, n64, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true)
    monkeypatch.setenv("SG_AMP_ENGINE", "cw")
    mc, tc, nc, pc = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true, precision=_native.SG_F32)
    assert _native.lib().sg_amp_plan_engine(op.plan(_native.SG_F32), B) == 2
    monkeypatch.setenv("SG_AMP_ENGINE", "staged")
    os_ = sparc.DesignOperator(W, L, M, n, o0, o1)  # staged tables (P = 16384)
    ms, ts, ns, ps = sparc.amp_decode_batch(Y, os_, 1.0, 25, true_idx=true, precision=_native.SG_F32)
    assert np.array_equal(mc, true) and np.array_equal(ms, true)
    assert np.all(np.abs(tc - ts) <= 1) and np.all(np.abs(tc - t64) <= 2)
    np.testing.assert_allclose(nc[:, :8], n64[:, :8], atol=2e-3)
    np.testing.assert_allclose(nc[:, :8], ns[:, :8], atol=1e-4)


def test_cw_engine_rate15_matches_staged(monkeypatch):
    """C2 benchmark point (R=1.5, AMP does not decode): the two f32 engines
    reach the same section decisions on almost every section and the same
    iteration counts within one."""
    W, L, M, n, o0, o1 = _c2_design(5)
    rng = np.random.default_rng(12)
    B = 3
    true = rng.integers(0, M, (B, L))
    beta0 = np.zeros((B, L * M))
    beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Y = op.apply(beta0, False) + rng.standard_normal((B, n))
    monkeypatch.setenv("SG_AMP_ENGINE", "cw")
    mc, tc, nc, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true, precision=_native.SG_F32)
    monkeypatch.setenv("SG_AMP_ENGINE", "staged")
    os_ = sparc.DesignOperator(W, L, M, n, o0, o1)
    ms, ts, ns, _ = sparc.amp_decode_batch(Y, os_, 1.0, 25, true_idx=true, precision=_native.SG_F32)
    assert np.mean(mc == ms) > 0.97
    assert np.all(np.abs(tc - ts) <= 1)
    np.testing.assert_allclose(nc[:, :6], ns[:, :6], atol=1e-3)


@pytest.mark.parametrize("phi_method", [1, 2])
def test_cw_engine_phi_methods_match_staged(monkeypatch, phi_method):
    """Both phi estimates (sparc.py:949-955) through the per-codeword engine
    agree with the staged engine on an L=32, M=512 design (w = 2^15)."""
    L, M, R = 32, 512, 1.3
    n = int(round(L * 9 / R))
    W = np.array(15.0)
    o0, o1 = sparc.generate_ordering(W, n, L * M, 17)
    rng = np.random.default_rng(3)
    B = 5
    true = rng.integers(0, M, (B, L))
    beta0 = np.zeros((B, L * M))
    beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Y = op.apply(beta0, False) + rng.standard_normal((B, n))
    m64, t64, n64, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, 1e-6, phi_method, true)
    monkeypatch.setenv("SG_AMP_ENGINE", "cw")
    mc, tc, nc, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, 1e-6, phi_method, true, precision=_native.SG_F32)
    assert _native.lib().sg_amp_plan_engine(op.plan(_native.SG_F32), B) == 2
    assert np.array_equal(mc, m64)
    assert np.all(np.abs(tc - t64) <= 2)
    np.testing.assert_allclose(nc[:, :6], n64[:, :6], atol=1e-3)


def test_cw_engine_c2_vs_oracle(monkeypatch):
    """One C2 codeword (L=1024, M=512, n=6144, R=1.5: the benchmark point)
    through the per-codeword engine against the CPU restatement (float128
    softmax): t_final within one, section decisions identical on >= 99 %,
    NMSE per iteration within 1e-3."""
    W, L, M, n, o0, o1 = _c2_design(31)
    Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
    rng = np.random.RandomState(6)
    true = rng.randint(0, M, L)
    beta0 = np.zeros(L * M)
    beta0[np.arange(L) * M + true] = 1
    y = Ab(beta0) + rng.randn(n)
    rb, rt, rn, rp = sparc_ref.amp(y, W, L, M, n, 1.0, 25, Ab, Az, beta0)
    monkeypatch.setenv("SG_AMP_ENGINE", "cw")
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    mi, tf, nm, ps = sparc.amp_decode_batch(y[None], op, 1.0, 25, true_idx=true[None], precision=_native.SG_F32)
    assert _native.lib().sg_amp_plan_engine(op.plan(_native.SG_F32), 1) == 2
    assert abs(int(tf[0]) - int(rt)) <= 1
    assert np.mean(mi[0] == np.argmax(rb.reshape(L, M), 1)) >= 0.99
    np.testing.assert_allclose(nm[0, :, 0], rn, atol=1e-3)


@pytest.mark.parametrize("handover", [None, "0.99"])
def test_auto_engine_handover_matches_staged(monkeypatch, handover):
    """A batch that fills the CUs on a design where codewords stop early
    (L=512, R=1.2): the automatic choice starts on the per-codeword engine and
    hands the remaining iterations to the staged engine once half the batch
    has stopped; decisions, stopping iterations and NMSE agree with the staged
    engine alone."""
    L, M, R = 512, 512, 1.2
    n = int(round(L * 9 / R))
    W = np.array(15.0)
    o0, o1 = sparc.generate_ordering(W, n, L * M, 23)
    B = 256  # one per CU on MI355X
    rng = np.random.default_rng(31)
    true = rng.integers(0, M, (B, L))
    beta0 = np.zeros((B, L * M), np.float32)
    beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Y = op.apply(beta0.astype(np.float64), False) + rng.standard_normal((B, n))
    monkeypatch.delenv("SG_AMP_ENGINE", raising=False)
    if handover is None:
        monkeypatch.delenv("SG_AMP_HANDOVER", raising=False)
    else:
        monkeypatch.setenv("SG_AMP_HANDOVER", handover)
    ma, ta, na, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true, precision=_native.SG_F32)
    assert _native.lib().sg_amp_plan_engine(op.plan(_native.SG_F32), B) == 2
    last = _native.amp_last_decode(op.plan(_native.SG_F32))
    assert last["engine"] == 2 and not last["companion"]
    if handover is not None:
        # the codewords of this design stop after 8-12 iterations; the active
        # flags are copied after iterations 3, 7, ... and read one iteration
        # later, so with 99 % the hand-over follows the second copy and
        # iterations 10.. run on the staged engine
        assert last["handover_iter"] == 9 and int(ta.max()) > 9, (last, np.bincount(ta))
    monkeypatch.delenv("SG_AMP_HANDOVER", raising=False)
    monkeypatch.setenv("SG_AMP_ENGINE", "staged")
    ms, ts, ns, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true, precision=_native.SG_F32)
    assert np.array_equal(ma, true) and np.array_equal(ms, true)
    assert np.all(np.abs(ta - ts) <= 1)
    np.testing.assert_allclose(na[:, :8], ns[:, :8], atol=1e-3)


def _c2_batch(seed_design, seed_data, B, R):
    W, L, M, n, o0, o1 = _c2_design(seed_design, R=R)
    rng = np.random.default_rng(seed_data)
    true = rng.integers(0, M, (B, L)).astype(np.int32)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    beta0 = np.zeros((B, L * M))
    beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
    Y = op.apply(beta0, False) + rng.standard_normal((B, n))
    return W, L, M, n, o0, o1, op, true, Y


def _bench_c2_batch(R, seed=1, B=256, prec=None):
    """The received words bench.py times (bench.amp_setup: design seed 0,
    Philox seed 1 stream 0, encode and AWGN on the GPU, in the line's
    precision), downloaded."""
    L, M, logM = 1024, 512, 9
    n = int(round(L * logM / R))
    W = np.array(15.0)
    prec = _native.SG_F32 if prec is None else prec
    dt = np.float32 if prec == _native.SG_F32 else np.float64
    es = np.dtype(dt).itemsize
    o0, o1 = sparc.generate_ordering(W, n, L * M, 0)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    plan = op.plan(prec)
    lib = _native.lib()
    d_bits = _native.DeviceBuffer(B * L * logM)
    d_true = _native.DeviceBuffer(B * L * 4)
    d_x = _native.DeviceBuffer(B * n * es)
    d_y = _native.DeviceBuffer(B * n * es)
    _native.check(lib.sg_rng_bits_device(seed, 0, B, L * logM, d_bits.ptr, None))
    _native.check(lib.sg_bits_to_sections_device(d_bits.ptr, B, L, logM, d_true.ptr, None))
    _native.check(lib.sg_amp_encode_device(plan, d_true.ptr, B, d_x.ptr, None))
    _native.check(lib.sg_awgn_device(prec, seed, 0, d_x.ptr, B, n, 1.0, d_y.ptr, None))
    _native.synchronize()
    Y = d_y.download(np.zeros((B, n), dt)).astype(np.float64)
    true = d_true.download(np.zeros((B, L), np.int32))
    return W, L, M, n, o0, o1, op, true, Y


def _rel_change(psi, t):
    """|psi_t - psi_(t-1)| / |psi_(t-1)| at iteration t >= 2 (psi[k] = psi after
    iteration k + 1): what the stop rule of sparc.py:984-986 compares with rtol."""
    return abs(psi[t - 1] - psi[t - 2]) / abs(psi[t - 2])


@pytest.mark.parametrize("R,inputs", [(1.5, "host"), (1.3, "host"), (1.5, "bench"), (1.3, "bench")])
def test_shipped_c2_batch_vs_oracle(monkeypatch, R, inputs):
    """The path bench.py times: C2 (L=1024, M=512, n=6144 at R=1.5 / 7089 at
    R=1.3), B=256, the automatic engine choice (per-codeword engine, hand-over
    to the staged engine once half the batch stopped), f32 -- against the CPU
    restatement of sparc.py:883-999 (float128 softmax) on ALL 256 codewords,
    for a numpy-generated batch and for the bench's own Philox batch.

    f32 bar ("AMP f32"):
      * section decisions identical on >= 99 % of the sections of every
        codeword, and on all of them where the reference decodes;
      * t_final within 2 of the reference's, except for a threshold stop: the
        engine that stopped first did so where the OTHER one's relative psi
        change was within 10 % of rtol = 1e-6 (the stop rule compares a
        change of ~1e-6 relative; psi itself agrees to ~2e-7, so near the
        threshold f32 rounding decides the iteration; DESIGN.md traces the
        bench batch's one such codeword); at most 1 % of the codewords;
      * NMSE per iteration within 1e-3 over the first 6 iterations;
      * FER identical, BER within 3 binomial standard deviations."""
    from oracle import cpu_pool
    monkeypatch.delenv("SG_AMP_ENGINE", raising=False)
    monkeypatch.delenv("SG_AMP_HANDOVER", raising=False)
    B, rtol = 256, 1e-6
    if inputs == "host":
        W, L, M, n, o0, o1, op, true, Y = _c2_batch(41, 7, B, R)
    else:
        W, L, M, n, o0, o1, op, true, Y = _bench_c2_batch(R)
    plan = op.plan(_native.SG_F32)
    assert _native.lib().sg_amp_plan_engine(plan, B) == 2
    mi, tf, nm, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true, precision=_native.SG_F32)
    last = _native.amp_last_decode(plan)
    assert last["engine"] == 2
    if R == 1.3 and inputs == "host":  # codewords stop after 14-18 iterations: the hand-over fires first
        assert 0 < last["handover_iter"] < int(tf.max()), (last, np.bincount(tf))
    res, _ = cpu_pool.amp_decode(cpu_pool.host_cores(16), W, L, M, n, o0, o1, Y, true, 25)
    assert sorted(res) == list(range(B))
    gpu_psi = {}

    def gpu_rel_change(b, t):  # the GPU's psi after iterations t - 1 and t (decodes with t_max = t, t + 1)
        for tm in (t, t + 1):
            if tm not in gpu_psi:
                gpu_psi[tm] = sparc.amp_decode_batch(Y, op, 1.0, tm, true_idx=true, precision=_native.SG_F32)[3][:, 0]
        return abs(gpu_psi[t + 1][b] - gpu_psi[t][b]) / abs(gpu_psi[t][b])

    threshold_stops = []
    for b in range(B):
        cm, ct_, cn, cpsi = res[b]
        same = np.mean(mi[b] == cm)
        if np.array_equal(cm, true[b]):
            assert same == 1.0, (b, same)
        assert same >= 0.99, (b, same)
        np.testing.assert_allclose(nm[b, :6, 0], cn[:6], atol=1e-3)
        if abs(int(tf[b]) - ct_) > 2:
            if tf[b] < ct_:  # the GPU stopped first: the reference was at its threshold there
                rc = _rel_change(cpsi, int(tf[b]))
            else:
                rc = gpu_rel_change(b, ct_)
            assert rc <= 1.1 * rtol, (b, tf[b], ct_, rc)
            threshold_stops.append(b)
    assert len(threshold_stops) <= B // 100, threshold_stops
    cmap = np.stack([res[b][0] for b in range(B)])
    assert np.array_equal((cmap != true).any(1), (mi != true).any(1))  # frame errors identical
    nb = B * L * 9
    cb = np.unpackbits((cmap ^ true).astype(np.uint32).view(np.uint8)).sum() / nb
    gb = np.unpackbits((mi ^ true).astype(np.uint32).view(np.uint8)).sum() / nb
    assert abs(cb - gb) <= 3 * np.sqrt(max(cb, 1.0 / nb) * (1 - cb) / nb) + 1.0 / nb, (cb, gb)
    if R == 1.3:  # decodable rate: most codewords decode, on both sides
        assert np.mean([np.array_equal(res[b][0], true[b]) for b in range(B)]) >= 0.75


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1.5, 1.3])
def test_shipped_f64_c2_batch_vs_oracle(monkeypatch, R):
    """The bench's double-precision C2 line (bench.amp_f64: the bench's Philox
    batch generated in float64, B = 256, automatic engine choice: the f64 split
    engine amp_cw2d.hip, handing over to the staged engine once half the batch
    has stopped) against the CPU restatement of sparc.py:883-999 (float128
    softmax) on ALL 256 codewords.  f64 bar (DESIGN.md "AMP, f64"): identical
    t_final and MAP decisions on every codeword, NMSE within 1e-8 at every
    iteration (the restatement's softmax is float128, the engine's float64)."""
    from oracle import cpu_pool
    monkeypatch.delenv("SG_AMP_ENGINE", raising=False)
    monkeypatch.delenv("SG_AMP_HANDOVER", raising=False)
    B = 256
    W, L, M, n, o0, o1, op, true, Y = _bench_c2_batch(R, prec=_native.SG_F64)
    plan = op.plan(_native.SG_F64)
    assert _native.lib().sg_amp_plan_engine(plan, B) == 2
    mi, tf, nm, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true, precision=_native.SG_F64)
    last = _native.amp_last_decode(plan)
    assert last["engine"] == 2
    res, _ = cpu_pool.amp_decode(cpu_pool.host_cores(16), W, L, M, n, o0, o1, Y, true, 25)
    assert sorted(res) == list(range(B))
    for b in range(B):
        cm, ct_, cn, _ = res[b]
        assert int(tf[b]) == ct_, (b, tf[b], ct_)
        assert np.array_equal(mi[b], cm), (b, np.mean(mi[b] != cm))
        np.testing.assert_allclose(nm[b, :, 0], cn, rtol=0, atol=1e-8)
    if R == 1.3:
        assert np.mean((mi == true).all(1)) >= 0.75


@pytest.mark.gpu
def test_small_batch_runs_on_companion_plan(monkeypatch):
    """Below one wave of the CUs the automatic choice is the staged engine;
    a per-codeword plan (P = 8192) then decodes on its companion plan at
    P = 16384.  Decisions, stopping iterations and NMSE agree with the staged
    engine on the P = 8192 tables (SG_AMP_ENGINE=staged keeps the plan)."""
    L, M, R = 512, 512, 1.2
    n = int(round(L * 9 / R))
    W = np.array(15.0)
    o0, o1 = sparc.generate_ordering(W, n, L * M, 29)
    B = 24
    rng = np.random.default_rng(37)
    true = rng.integers(0, M, (B, L))
    beta0 = np.zeros((B, L * M), np.float32)
    beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Y = op.apply(beta0.astype(np.float64), False) + rng.standard_normal((B, n))
    monkeypatch.delenv("SG_AMP_ENGINE", raising=False)
    plan = op.plan(_native.SG_F32)
    P = ctypes.c_int()
    _native.lib().sg_amp_plan_info(plan, None, None, None, None, ctypes.byref(P), None)
    assert P.value == 8192
    assert _native.lib().sg_amp_plan_engine(plan, B) == 1
    ma, ta, na, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true, precision=_native.SG_F32)
    monkeypatch.setenv("SG_AMP_ENGINE", "staged")
    ms, ts, ns, _ = sparc.amp_decode_batch(Y, op, 1.0, 25, true_idx=true, precision=_native.SG_F32)
    assert np.array_equal(ma, true) and np.array_equal(ms, true)
    assert np.all(np.abs(ta - ts) <= 1)
    np.testing.assert_allclose(na[:, :8], ns[:, :8], atol=1e-3)
