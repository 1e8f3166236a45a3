"""The degree-grouped single-precision min-sum kernel (bp.hip
bp_grouped_minsum_kernel, the C3 path) against the table kernel
(SG_BP_GROUPED=0) and the float32 restatement of c_ldpc.c:339-381
(oracle/bp.py minsum_numpy), bit for bit: which graphs take it, both of its
instances (<4, 2> and <8, 4> groups per wave), degree-0/1 and degree-16
variables, partially filled groups, a negative normalisation factor, and the
iteration caps 1 and 50."""
import ctypes as ct

import numpy as np
import pytest

from ldpc_sparc_amd import _native
from ldpc_sparc_amd.ldpc import code
from oracle import bp

pytestmark = pytest.mark.gpu


def _graph(vdeg, cdeg, intrlv):
    g = ct.c_void_p()
    _native.check(_native.lib().sg_ldpc_graph_create(_native.ptr(vdeg), _native.ptr(cdeg), _native.ptr(intrlv),
                                                     len(vdeg), len(cdeg), len(intrlv), ct.byref(g)))
    return g


def _kernel(g, dectype="minsum", prec=_native.SG_F32):
    buf = ct.create_string_buffer(128)
    _native.check(_native.lib().sg_ldpc_decode_kernel(g, _native.DECTYPES[dectype], prec, buf, 128))
    return buf.value.decode()


def _decode(g, ch, max_it, factor):
    ch = np.ascontiguousarray(ch, dtype=np.float64)
    app = np.zeros_like(ch)
    it = np.zeros(ch.shape[0], dtype=np.int32)
    _native.check(_native.lib().sg_ldpc_decode(g, _native.DECTYPES["minsum"], _native.SG_F32, _native.ptr(ch),
                                               ch.shape[0], int(max_it), float(factor), _native.ptr(app),
                                               _native.ptr(it)))
    return app.astype(np.float32), it


def _random_graph(vdegs, nv, rng, cmax=8, cmin=2):
    vdeg = np.array([vdegs[v % len(vdegs)] for v in range(nv)], dtype=np.int64)
    E = int(vdeg.sum())
    cdeg, left = [], E
    while left > 0:
        d = int(min(left, rng.integers(cmin, cmax + 1)))
        if left - d == 1:
            d += 1
        cdeg.append(d)
        left -= d
    return vdeg, np.array(cdeg, dtype=np.int64), rng.permutation(E).astype(np.int64)


def _check(monkeypatch, vdeg, cdeg, intrlv, ch, max_its=(1, 50), factors=(0.7,), expect=None):
    g = _graph(vdeg, cdeg, intrlv)
    try:
        name = _kernel(g)
        if expect:
            assert name.startswith(expect), name
        ch32 = ch.astype(np.float32).astype(np.float64)
        for mi in max_its:
            for f in factors:
                monkeypatch.setenv("SG_BP_GROUPED", "1")
                app, it = _decode(g, ch32, mi, f)
                monkeypatch.setenv("SG_BP_GROUPED", "0")
                tapp, tit = _decode(g, ch32, mi, f)
                assert np.array_equal(it, tit) and np.array_equal(app.view(np.uint32), tapp.view(np.uint32)), (mi, f)
                rapp, rit = bp.minsum_numpy(ch32, vdeg, cdeg, intrlv, mi, f, np.float32)
                assert np.array_equal(it, rit) and np.array_equal(app, rapp), (mi, f)
        return name
    finally:
        _native.lib().sg_ldpc_graph_destroy(g)


def _awgn(c, ebn0, B, rng):
    R = c.K / c.N
    s2 = 1 / (2 * R * 10 ** (ebn0 / 10))
    X = c.encode_batch(rng.integers(0, 2, (B, c.K)))
    return 2 * ((1 - 2 * X) + np.sqrt(s2) * rng.standard_normal(X.shape)) / s2


@pytest.mark.parametrize("std,rate,z,expect", [("802.11n", "1/2", 81, "bp_grouped_minsum_kernel<4, 2>"),
                                               ("802.11n", "1/2", 27, "bp_grouped_minsum_kernel"),
                                               ("802.16", "1/2", 96, "bp_grouped_minsum_kernel"),
                                               ("802.11n", "5/6", 81, "bp_flood_kernel<float, 2, 24,")])
def test_standard_codes(monkeypatch, std, rate, z, expect):
    c = code(std, rate, z)
    rng = np.random.default_rng(11)
    ch = np.concatenate([_awgn(c, e, 24, rng) for e in (1.0, 2.5)])
    _check(monkeypatch, np.asarray(c.vdeg, np.int64), np.asarray(c.cdeg, np.int64), np.asarray(c.intrlv, np.int64),
           ch, expect=expect)


def test_irregular_small_groups(monkeypatch):
    """Degrees 0, 1, 16 and odd degrees; every group partially filled."""
    rng = np.random.default_rng(5)
    vdeg, cdeg, intrlv = _random_graph((1, 2, 3, 5, 16, 0, 2, 4, 7), 300, rng)
    ch = 1.0 + 2.0 * rng.standard_normal((40, len(vdeg)))
    _check(monkeypatch, vdeg, cdeg, intrlv, ch, max_its=(1, 7, 50), factors=(0.7, 1.0, -0.5),
           expect="bp_grouped_minsum_kernel<4, 2>")


def test_irregular_many_groups_takes_wide_instance(monkeypatch):
    """More than 32 variable groups: the <8, 4> instance."""
    rng = np.random.default_rng(6)
    vdeg, cdeg, intrlv = _random_graph(tuple(range(1, 9)), 2400, rng, 8, 7)
    ch = 1.5 + 2.0 * rng.standard_normal((16, len(vdeg)))
    _check(monkeypatch, vdeg, cdeg, intrlv, ch, max_its=(3, 40), expect="bp_grouped_minsum_kernel<8, 4>")


def test_graphs_outside_the_grouped_layout_take_the_table_kernel():
    rng = np.random.default_rng(8)
    for vd, cmax in (((2, 17, 3), 8), ((2, 3), 12)):  # variable degree 17; check degrees up to 12
        vdeg, cdeg, intrlv = _random_graph(vd, 200, rng, cmax)
        g = _graph(vdeg, cdeg, intrlv)
        try:
            assert _kernel(g).startswith("bp_flood_kernel<float, 2,"), _kernel(g)
            assert _kernel(g, "sumprod2", _native.SG_F64).startswith("bp_flood_kernel<double, 1,")
        finally:
            _native.lib().sg_ldpc_graph_destroy(g)
    # a degree-1 check: refused when the graph is created (sg_ldpc_graph_create
    # needs check degrees 2..255), so neither kernel ever sees one
    vdeg, cdeg, intrlv = _random_graph((2, 3), 200, rng, 8)
    k = int(np.argmax(cdeg >= 3))
    cdeg = np.concatenate([cdeg[:k], [1, cdeg[k] - 1], cdeg[k + 1:]]).astype(np.int64)
    with pytest.raises(_native.NativeError, match="check degree 1"):
        _graph(vdeg, cdeg, intrlv)


@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf])
def test_nonfinite_channel_input_takes_the_table_kernel(monkeypatch, bad):
    """The grouped kernel has no NaN semantics (built -fno-honor-nans) and
    saturates channel LLRs at +-1e30: a host batch holding a NaN or an infinity
    (a hard-known bit) decodes through the table kernel, so its results equal
    the table kernel's."""
    c = code("802.11n", "1/2", 27)
    ch = _awgn(c, 1.5, 8, np.random.default_rng(4))
    ch[3, 17] = bad
    ch[5, 3] = -bad if not np.isnan(bad) else bad
    vdeg, cdeg, intrlv = (np.asarray(a, np.int64) for a in (c.vdeg, c.cdeg, c.intrlv))
    g = _graph(vdeg, cdeg, intrlv)
    try:
        monkeypatch.setenv("SG_BP_GROUPED", "1")
        app, it = _decode(g, ch, 20, 0.7)
        monkeypatch.setenv("SG_BP_GROUPED", "0")
        tapp, tit = _decode(g, ch, 20, 0.7)
        assert np.array_equal(it, tit) and np.array_equal(app.view(np.uint32), tapp.view(np.uint32))
    finally:
        _native.lib().sg_ldpc_graph_destroy(g)


def test_overflowing_channel_input_stays_finite(monkeypatch):
    """A finite double past float's range (1e300) is a finite LLR for the
    reference (c_ldpc.c computes in double).  The f32 host path clamps it to
    +-FLT_MAX and decodes it through the grouped kernel, which saturates large
    channel LLRs at +-1e30: the results equal the same batch with +-1e30 in its
    place, hold no NaN, and take the float64 oracle's decisions on every
    codeword the oracle decodes."""
    c = code("802.11n", "1/2", 27)
    ch = _awgn(c, 2.0, 8, np.random.default_rng(4))
    ch[3, 17], ch[5, 3], ch[5, 4] = 1e300, -1e300, 1e300
    sat = ch.copy()
    sat[np.abs(sat) > 1e30] = np.sign(sat[np.abs(sat) > 1e30]) * 1e30
    vdeg, cdeg, intrlv = (np.asarray(a, np.int64) for a in (c.vdeg, c.cdeg, c.intrlv))
    g = _graph(vdeg, cdeg, intrlv)
    try:
        monkeypatch.setenv("SG_BP_GROUPED", "1")
        app, it = _decode(g, ch, 20, 0.7)
        sapp, sit = _decode(g, sat, 20, 0.7)
        assert np.isfinite(app).all()
        assert np.array_equal(it, sit) and np.array_equal(app.view(np.uint32), sapp.view(np.uint32))
        oapp, oit = bp.decode_batch("minsum", ch, vdeg, cdeg, intrlv, 20, 0.7)
        dec = oit < 20
        assert dec.any()
        assert np.array_equal((app < 0)[dec], (oapp < 0)[dec]) and np.array_equal(it[dec], oit[dec])
    finally:
        _native.lib().sg_ldpc_graph_destroy(g)


@pytest.mark.parametrize("ebn0", [1.0, 2.0])
def test_c3_batch_at_bench_size(monkeypatch, ebn0):
    """C3 at its bench size (B = 4096, BASELINE.json configs[2]): one workgroup
    per codeword (bp_grouped.hip BPG_GRID_B), 4096 workgroups through 4 slots
    per CU, so later workgroups start on LDS images and stop-flag words that
    earlier ones left behind.  Bit for bit against the float32 restatement of
    the corrected min-sum (c_ldpc.c:339-381) at iteration caps 1 and 50."""
    c = code("802.11n", "1/2", 81)
    B = 4096
    assert B > 4 * _native.cu_count()
    ch = _awgn(c, ebn0, B, np.random.default_rng(int(ebn0 * 10) + 3))
    vdeg, cdeg, intrlv = (np.asarray(a, np.int64) for a in (c.vdeg, c.cdeg, c.intrlv))
    g = _graph(vdeg, cdeg, intrlv)
    try:
        assert _kernel(g).startswith("bp_grouped_minsum_kernel<4, 2>"), _kernel(g)
        monkeypatch.setenv("SG_BP_GROUPED", "1")
        ch32 = ch.astype(np.float32).astype(np.float64)
        for mi in (1, 50):
            app, it = _decode(g, ch32, mi, 0.7)
            rapp, rit = bp.minsum_numpy(ch32, vdeg, cdeg, intrlv, mi, 0.7, np.float32)
            assert np.array_equal(it, rit), mi
            assert np.array_equal(app.view(np.uint32), rapp.view(np.uint32)), mi
    finally:
        _native.lib().sg_ldpc_graph_destroy(g)
