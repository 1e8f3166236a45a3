"""CPU tests of the degree-grouped min-sum layout (capi_ldpc.cpp grp_layout,
read through sg_ldpc_grouped_layout with no device): its invariants, and a
numpy emulation of bp_grouped_minsum_kernel's data flow over that layout --
messages at the layout's LDS byte addresses, variable groups summing their
ports in the reference's order (c_ldpc.c:171-178), check groups in 64-lane
blocks, the stopping rule of :196-197 -- which must reproduce the float32
restatement of the corrected min-sum (oracle/bp.py minsum_numpy) bit for bit.
The GPU tests (test_bp_grouped_gpu.py) then pin the kernel to the same
restatement; this one pins the layout the host builds, pairs included."""
import ctypes as ct

import numpy as np
import pytest

from ldpc_sparc_amd import _native
from ldpc_sparc_amd.ldpc import code
from oracle import bp

W = 8           # waves per workgroup (GRP_WAVES)
PAIR = 1 << 8   # GRP_PAIR
PAIR_MAXD = 3   # GRP_PAIR_MAXD


def layout(vdeg, cdeg, intrlv, pairs=True):
    vdeg, cdeg, intrlv = (np.ascontiguousarray(a, np.int64) for a in (vdeg, cdeg, intrlv))
    info = np.zeros(10, np.int32)
    args = [_native.ptr(vdeg), _native.ptr(cdeg), _native.ptr(intrlv), len(vdeg), len(cdeg), len(intrlv),
            int(pairs), _native.ptr(info)]
    _native.check(_native.lib().sg_ldpc_grouped_layout(*args, None, 0, None, 0, None, 0))
    if not info[0]:
        return None
    meta = np.zeros(info[8], np.int32)
    vmap = np.zeros(info[9], np.int32)
    vtab = np.zeros(info[6], np.uint16)
    _native.check(_native.lib().sg_ldpc_grouped_layout(*args, _native.ptr(meta), len(meta), _native.ptr(vmap),
                                                       len(vmap), _native.ptr(vtab), len(vtab)))
    kvj, kcj = int(info[3]), int(info[4])
    return {"vj": int(info[1]), "cj": int(info[2]), "kvj": kvj, "kcj": kcj, "msg_bytes": int(info[5]),
            "npairs": int(info[7]), "vtab": vtab, "vmap": vmap.reshape(W, kvj, 64),
            "vdeg": meta[:W * kvj].reshape(W, kvj), "vt": meta[W * kvj:2 * W * kvj].reshape(W, kvj) >> 1,
            "cdeg": meta[2 * W * kvj:2 * W * kvj + W * kcj].reshape(W, kcj),
            "caddr": meta[2 * W * kvj + W * kcj:2 * W * kvj + 2 * W * kcj].reshape(W, kcj),
            "cval": meta[2 * W * kvj + 2 * W * kcj:].reshape(W, kcj)}


def emulate(lay, ch, max_it, factor):
    """bp_grouped_minsum_kernel's data flow in numpy float32 over `lay`, for a
    [B, N] batch: returns (app, it) as the kernel writes them."""
    f32 = np.float32
    ch = np.asarray(ch, f32)
    B, N = ch.shape
    img = np.zeros((B, lay["msg_bytes"] // 4 + 1), f32)
    groups = [(w, j) for w in range(W) for j in range(lay["vj"])]
    app = np.zeros((B, N), f32)
    its = np.full(B, max_it, np.int32)
    live = np.ones(B, bool)
    chk = [(w, q) for w in range(W) for q in range(lay["cj"]) if lay["cdeg"][w, q] >= 2]
    for it in range(max_it):
        for w, j in groups:  # variable pass: ports in order, then the extrinsic write-backs
            d = int(lay["vdeg"][w, j]) & (PAIR - 1)
            v = lay["vmap"][w, j]
            real = v >= 0
            acc = np.where(real[None, :], ch[:, np.maximum(v, 0)], f32(0))
            slots = [lay["vtab"][lay["vt"][w, j] + 64 * k + np.arange(64)].astype(np.int64) // 4 for k in range(d)]
            m = [img[:, s] for s in slots]
            for k in range(d):
                acc = acc + m[k]
            for k in range(d):
                img[:, slots[k]] = acc - m[k]
            upd = live[:, None] & real[None, :]
            app[:, v[real]] = np.where(upd[:, real], acc[:, real], app[:, v[real]])
        unsat = np.zeros(B, bool)
        for w, q in chk:  # check pass: min-sum on each lane's dc messages (any port order)
            dc, addr, cn = int(lay["cdeg"][w, q]), int(lay["caddr"][w, q]), int(lay["cval"][w, q])
            idx = np.stack([(addr + 256 * k + 4 * np.arange(64)) // 4 for k in range(dc)], 1)  # [64, dc]
            L = img[:, idx]
            a = np.abs(L)
            sb = np.signbit(L)
            i1 = np.argmin(a, axis=2)
            m1 = np.take_along_axis(a, i1[..., None], 2)[..., 0]
            a2 = a.copy()
            np.put_along_axis(a2, i1[..., None], np.inf, 2)
            m2 = a2.min(axis=2)
            sall = np.bitwise_xor.reduce(sb, axis=2)
            u = sall | ~(m1 > 0)
            unsat |= u[:, :cn].any(axis=1)
            for k in range(dc):
                mag = np.where(i1 == k, m2, m1)
                img[:, idx[:, k]] = np.where(sall ^ sb[:, :, k], -mag, mag) * f32(factor)
        done = live & ~unsat
        its[done] = it
        live &= ~done
        if not live.any():
            break
    return app, its


def _awgn(c, ebn0, B, rng):
    R = c.K / c.N
    s2 = 1 / (2 * R * 10 ** (ebn0 / 10))
    X = c.encode_batch(rng.integers(0, 2, (B, c.K)))
    return 2 * ((1 - 2 * X) + np.sqrt(s2) * rng.standard_normal(X.shape)) / s2


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


CODES = [("802.11n", "1/2", 81), ("802.11n", "1/2", 27), ("802.16", "1/2", 96)]


@pytest.mark.parametrize("std,rate,z", CODES)
def test_layout_invariants_and_pairs(std, rate, z):
    c = code(std, rate, z)
    lay = layout(c.vdeg, c.cdeg, c.intrlv)
    assert lay is not None
    # every real port addresses a distinct slot; pairs sit at even positions, same degree <= 3
    seen = set()
    for w in range(W):
        for j in range(lay["vj"]):
            word = int(lay["vdeg"][w, j])
            d = word & (PAIR - 1)
            for l in range(64):
                if lay["vmap"][w, j, l] >= 0:
                    for k in range(d):
                        s = int(lay["vtab"][lay["vt"][w, j] + 64 * k + l])
                        assert s % 4 == 0 and s < lay["msg_bytes"] and s not in seen
                        seen.add(s)
            if word & PAIR:
                assert j % 2 == 0 and j + 1 < lay["vj"]
                assert int(lay["vdeg"][w, j + 1]) & (PAIR - 1) == d and 1 <= d <= PAIR_MAXD
    assert len(seen) == len(c.intrlv)
    if (std, rate, z) == ("802.11n", "1/2", 81):
        assert lay["npairs"] >= 8  # the C3 code: 14 degree-2 and 12 degree-3 groups over 8 waves
    assert layout(c.vdeg, c.cdeg, c.intrlv, pairs=False)["npairs"] == 0


@pytest.mark.parametrize("std,rate,z", CODES)
@pytest.mark.parametrize("pairs", [True, False])
def test_emulated_kernel_equals_f32_restatement(std, rate, z, pairs):
    c = code(std, rate, z)
    lay = layout(c.vdeg, c.cdeg, c.intrlv, pairs)
    rng = np.random.default_rng(z + 3 * int(pairs))
    ch = np.concatenate([_awgn(c, e, 12, rng) for e in (1.0, 2.5)]).astype(np.float32)
    for mi in (1, 7, 50):
        app, it = emulate(lay, ch, mi, 0.7)
        rapp, rit = bp.minsum_numpy(ch, c.vdeg, c.cdeg, c.intrlv, mi, 0.7, np.float32)
        assert np.array_equal(it, rit) and np.array_equal(app.view(np.uint32), rapp.view(np.uint32)), mi


def test_emulated_kernel_irregular_graph():
    """Degree-0/1/16 variables, partially filled groups, a negative factor."""
    rng = np.random.default_rng(5)
    vdeg, cdeg, intrlv = _random_graph((1, 2, 3, 5, 16, 0, 2, 4, 7), 300, rng)
    lay = layout(vdeg, cdeg, intrlv)
    ch = (1.0 + 2.0 * rng.standard_normal((10, len(vdeg)))).astype(np.float32)
    for mi, f in ((7, 0.7), (50, -0.5)):
        app, it = emulate(lay, ch, mi, f)
        rapp, rit = bp.minsum_numpy(ch, vdeg, cdeg, intrlv, mi, f, np.float32)
        assert np.array_equal(it, rit) and np.array_equal(app.view(np.uint32), rapp.view(np.uint32))


def test_graphs_outside_the_layout():
    rng = np.random.default_rng(8)
    vdeg, cdeg, intrlv = _random_graph((2, 17, 3), 200, rng)  # variable degree 17
    assert layout(vdeg, cdeg, intrlv) is None
    vdeg, cdeg, intrlv = _random_graph((2, 3), 200, rng, 12)  # check degrees up to 12
    assert layout(vdeg, cdeg, intrlv) is None


@pytest.mark.parametrize("bad", ["negative", "too_large", "repeated"])
def test_layout_refuses_a_bad_interleaver(bad):
    """sg_ldpc_grouped_layout runs graph creation's permutation check on intrlv
    before building the layout (which indexes msg_addr[intrlv[p]])."""
    c = code("802.11n", "1/2", 27)
    intrlv = np.array(c.intrlv, np.int64)
    intrlv[5] = {"negative": -1, "too_large": len(intrlv), "repeated": intrlv[6]}[bad]
    with pytest.raises(_native.NativeError, match="permutation"):
        layout(c.vdeg, c.cdeg, intrlv)
