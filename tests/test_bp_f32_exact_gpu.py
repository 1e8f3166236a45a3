"""Single-precision min-sum BP (the C3 kernel, bp.hip) against an exact
float32 restatement of the corrected reference min-sum (c_ldpc.c:339-381 with
the index fix of SURVEY.md 8(c); same arithmetic order: the variable sums in
port order, one multiply by the factor), bit for bit -- and every decoder on an
irregular random graph (variable degrees 1 to 11, odd and even) against the
C restatement oracle/bp_oracle.c.

The float32 restatement is oracle/bp.py minsum_numpy (test infrastructure,
pinned bit for bit against oracle/bp_oracle.c in float64 by
tests/test_ldpc_host.py)."""
import ctypes as ct

import numpy as np
import pytest

from ldpc_sparc_amd import _native
from ldpc_sparc_amd.ldpc import code
from oracle import bp

pytestmark = pytest.mark.gpu


def _awgn(c, ebn0, B, rng):
    R = c.K / c.N
    s2 = 1 / (2 * R * 10 ** (ebn0 / 10))
    X = c.encode_batch(rng.integers(0, 2, (B, c.K)))
    return X, 2 * ((1 - 2 * X) + np.sqrt(s2) * rng.standard_normal(X.shape)) / s2


@pytest.mark.parametrize("std,rate,z", [("802.11n", "1/2", 81), ("802.11n", "3/4", 27), ("802.16", "1/2", 96)])
def test_f32_minsum_bitexact_vs_float32_restatement(std, rate, z):
    c = code(std, rate, z)
    rng = np.random.default_rng(7)
    for ebn0 in (1.0, 2.0):
        X, ch = _awgn(c, ebn0, 48, rng)
        ch32 = ch.astype(np.float32).astype(np.float64)  # the f32 path's inputs, exactly
        app, it = c.decode_batch(ch32, 50, "minsum", 0.7, precision="f32")
        rapp, rit = bp.minsum_numpy(ch32, c.vdeg, c.cdeg, c.intrlv, 50, 0.7, np.float32)
        assert np.array_equal(it, rit)
        assert np.array_equal(app.astype(np.float32), rapp)


def _random_graph(nv, rng):
    """Irregular graph in the reference's decoder layout (vdeg, cdeg, intrlv):
    variable degrees cycle through 1, 2, 3, 5, 11, 2, 4; checks of degree 2-8."""
    vdeg = np.array([(1, 2, 3, 5, 11, 2, 4)[v % 7] for v in range(nv)], dtype=np.int64)
    E = int(vdeg.sum())
    cdeg = []
    left = E
    while left > 0:
        d = int(min(left, rng.integers(2, 9)))
        if left - d == 1:
            d += 1
        cdeg.append(d)
        left -= d
    cdeg = np.array(cdeg, dtype=np.int64)
    intrlv = rng.permutation(E).astype(np.int64)  # variable port -> check-ordered message
    return vdeg, cdeg, intrlv


def _decode_graph(vdeg, cdeg, intrlv, ch, max_it, dectype, factor, precision):
    L = _native.lib()
    g = ct.c_void_p()
    _native.check(L.sg_ldpc_graph_create(_native.ptr(vdeg), _native.ptr(cdeg), _native.ptr(intrlv), len(vdeg),
                                         len(cdeg), len(intrlv), ct.byref(g)))
    try:
        ch = np.ascontiguousarray(ch, dtype=np.float64)
        app = np.zeros_like(ch)
        it = np.zeros(ch.shape[0], dtype=np.int32)
        _native.check(L.sg_ldpc_decode(g, _native.DECTYPES[dectype], precision, _native.ptr(ch), ch.shape[0],
                                       int(max_it), float(factor), _native.ptr(app), _native.ptr(it)))
        return app, it
    finally:
        L.sg_ldpc_graph_destroy(g)


def test_irregular_graph_all_decoders():
    """Degree-1 and odd-degree variables, ports past a round's end: the
    variable pass's two-port rounds and register-held slots on every path."""
    rng = np.random.default_rng(3)
    vdeg, cdeg, intrlv = _random_graph(700, rng)
    ch = 1.5 + 2.0 * rng.standard_normal((32, len(vdeg)))
    for mi in (1, 7, 30):
        app, it = _decode_graph(vdeg, cdeg, intrlv, ch, mi, "minsum", 0.7, _native.SG_F64)
        oapp, oit = bp.decode_batch("minsum", ch, vdeg, cdeg, intrlv, mi, 0.7)
        assert np.array_equal(it, oit) and np.array_equal(app, oapp)
        ch32 = ch.astype(np.float32).astype(np.float64)
        app, it = _decode_graph(vdeg, cdeg, intrlv, ch32, mi, "minsum", 0.7, _native.SG_F32)
        rapp, rit = bp.minsum_numpy(ch32, vdeg, cdeg, intrlv, mi, 0.7, np.float32)
        assert np.array_equal(it, rit) and np.array_equal(app.astype(np.float32), rapp)
        for dt in ("sumprod2", "sumprod"):
            app, it = _decode_graph(vdeg, cdeg, intrlv, ch, mi, dt, 0.7, _native.SG_F64)
            oapp, oit = bp.decode_batch(dt, ch, vdeg, cdeg, intrlv, mi, 0.7)
            assert np.array_equal(it, oit), dt
            fin = np.isfinite(oapp)
            np.testing.assert_allclose(app[fin], oapp[fin], rtol=1e-9, atol=1e-9, err_msg=dt)
