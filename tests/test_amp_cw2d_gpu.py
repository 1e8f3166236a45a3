"""GPU parity of the double-precision split engine (amp_cw2d.hip) against the
staged f64 engine (amp_fused.hip, SG_AMP_ENGINE=staged) on the same plan and
against the CPU restatement of sparc.py:883-999 (oracle/sparc_ref.py, float128
softmax) on the C2 size.

Bars (the f64 bars of DESIGN.md "Oracle and parity"): against the staged
engine, identical t_final and MAP decisions on every codeword and NMSE within
1e-9 at every iteration; against the CPU restatement, the bar of
test_amp_gpu.py::test_full_size_decode_f64_vs_oracle (identical t_final, NMSE
within 1e-8, decisions on >= 99 % of the sections).  The two GPU engines
differ only in summation order and twiddle arithmetic (Horner / rotation
steps here, table products there)."""
import numpy as np
import pytest

from ldpc_sparc_amd import _native, sparc

pytestmark = pytest.mark.gpu


def _batch(L, M, R, B, seed_design, seed_data, P=15.0):
    n = int(round(L * np.log2(M) / R))
    W = np.array(P)
    o0, o1 = sparc.generate_ordering(W, n, L * M, seed_design)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    rng = np.random.default_rng(seed_data)
    true = rng.integers(0, M, (B, L)).astype(np.int32)
    beta0 = np.zeros((B, L * M))
    beta0[np.arange(B)[:, None], np.arange(L) * M + true] = 1
    Y = op.apply(beta0, False) + rng.standard_normal((B, n))
    return op, true, Y


def _decode(monkeypatch, op, Y, true, engine, t_max=25):
    if engine is None:
        monkeypatch.delenv("SG_AMP_ENGINE", raising=False)
    else:
        monkeypatch.setenv("SG_AMP_ENGINE", engine)
    out = sparc.amp_decode_batch(Y, op, 1.0, t_max, true_idx=true)
    info = _native.amp_last_decode(op.plan(_native.SG_F64))
    return out, info


@pytest.mark.parametrize("L,M,R,B", [(1024, 512, 1.5, 48), (1024, 512, 1.3, 32)])
def test_f64_split_engine_vs_staged(monkeypatch, L, M, R, B):
    op, true, Y = _batch(L, M, R, B, 41, 5)
    (ma, ta, na, pa), ia = _decode(monkeypatch, op, Y, true, "cw")
    (mb, tb, nb, pb), ib = _decode(monkeypatch, op, Y, true, "staged")
    assert ia["engine"] == 2 and ia["handover_iter"] == -1
    assert ib["engine"] == 1
    assert np.array_equal(ta, tb)
    assert np.array_equal(ma, mb)
    np.testing.assert_allclose(na, nb, rtol=0, atol=1e-9)
    np.testing.assert_allclose(pa, pb, rtol=1e-9, atol=1e-12)
    if R <= 1.3:
        assert (ma == true).all(1).mean() >= 0.75


def test_f64_split_engine_first_iterations(monkeypatch):
    """psi after 1, 2, 3 iterations (t_max = 2, 3, 4): the state after each of
    the engine's first launches (t = 0 has no Ab; t = 1 the first Ab)."""
    op, true, Y = _batch(1024, 512, 1.5, 16, 7, 9)
    for tm in (2, 3, 4):
        (_, _, na, pa), _ = _decode(monkeypatch, op, Y, true, "cw", tm)
        (_, _, nb, pb), _ = _decode(monkeypatch, op, Y, true, "staged", tm)
        np.testing.assert_allclose(pa, pb, rtol=1e-11)
        np.testing.assert_allclose(na, nb, rtol=0, atol=1e-11)


def test_f64_split_engine_vs_oracle(monkeypatch):
    """One C2 codeword through the split engine (forced) against the CPU
    restatement: the bar of test_full_size_decode_f64_vs_oracle."""
    from oracle import sparc_ref
    W, L, M = np.array(15.0), 1024, 512
    n = int(round(L * 9 / 1.5))
    o0, o1 = sparc.generate_ordering(W, n, L * M, 31)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    Ab, Az = sparc_ref.dct_operators(W, L, M, n, o0, o1)
    rng = np.random.RandomState(4)
    true = rng.randint(0, M, L)
    beta0 = np.zeros(L * M)
    beta0[np.arange(L) * M + true] = 1
    y = Ab(beta0) + rng.randn(n)
    rb, rt, rn, rp = sparc_ref.amp(y, W, L, M, n, 1.0, 25, Ab, Az, beta0)
    (mi, tf, nm, ps), info = _decode(monkeypatch, op, y[None], true[None], "cw")
    assert info["engine"] == 2
    assert tf[0] == rt
    np.testing.assert_allclose(nm[0, :, 0], rn, atol=1e-8)
    assert np.mean(mi[0] != np.argmax(rb.reshape(L, M), 1)) < 0.01


def test_f64_shipped_choice_full_batch(monkeypatch):
    """B = 256 (the bench batch size) with the automatic choice: the split
    engine, handing over to the staged engine once half the batch has stopped
    (R = 1.3: codewords stop after 14-18 iterations, so the hand-over fires; at
    R = 1.5 nearly every codeword runs to t_max and none happens); same
    decisions and stopping iterations as the staged engine throughout."""
    op, true, Y = _batch(1024, 512, 1.3, 256, 11, 3)
    (ma, ta, na, _), ia = _decode(monkeypatch, op, Y, true, None)
    (mb, tb, nb, _), ib = _decode(monkeypatch, op, Y, true, "staged")
    assert ia["engine"] == 2 and ib["engine"] == 1
    assert ia["handover_iter"] > 0  # the split -> staged state transfer ran (class-order s, stM / stI, z, tau, phi)
    assert np.array_equal(ta, tb)
    assert np.array_equal(ma, mb)
    np.testing.assert_allclose(na, nb, rtol=0, atol=1e-9)


def test_f64_outside_split_engine_bounds_takes_staged(monkeypatch):
    """A design outside the f64 split engine's bounds (M = 1024 > 512 entries per section for its
    one-wavefront statistics) at a batch that fills the CUs: the plan keeps the staged engine, and the
    decode runs (no SG_ERR_UNSUPPORTED at decode time)."""
    op, true, Y = _batch(256, 1024, 1.5, 256, 3, 4)
    (m, t, nm, _), info = _decode(monkeypatch, op, Y, true, None, t_max=6)
    assert info["engine"] == 1
    assert np.all(t >= 1) and np.isfinite(nm).all()
