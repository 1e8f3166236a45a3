"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of oracle/bp_oracle.c (the CPU
restatement of ldpc_jossy/src/c_ldpc.c) and of the reference's own c_ldpc.c
compiled into oracle/_ref/ (see oracle/Makefile)."""
import ctypes as ct
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(HERE, "_build", "libbp_oracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libc_ldpc_ref.so")

KINDS = {"sumprod": 0, "sumprod2": 1, "minsum": 2, "minsum_refbug": 3}

_dp = ct.POINTER(ct.c_double)
_lp = ct.POINTER(ct.c_int64)
_libs = {}


def _load(path, which):
    if which not in _libs:
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = ct.CDLL(path)
        _libs[which] = L
    return _libs[which]


def oracle_lib():
    L = _load(ORACLE_LIB, "oracle")
    for n in ("or_sumprod", "or_sumprod2"):
        getattr(L, n).argtypes = [_dp, _lp, _lp, _lp, ct.c_int, ct.c_int, ct.c_int, _dp, ct.c_int]
        getattr(L, n).restype = ct.c_int
    for n in ("or_minsum", "or_minsum_refbug"):
        getattr(L, n).argtypes = [_dp, _lp, _lp, _lp, ct.c_int, ct.c_int, ct.c_int, _dp,
                                  ct.c_double, ct.c_int]
        getattr(L, n).restype = ct.c_int
    L.or_lxor.argtypes = [ct.c_double, ct.c_double, ct.c_int]
    L.or_lxor.restype = ct.c_double
    L.or_lxfb.argtypes = [_dp, ct.c_int64, ct.c_int]
    L.or_lxfb.restype = ct.c_double
    L.or_decode_batch.argtypes = [ct.c_int, _dp, ct.c_int, _lp, _lp, _lp, ct.c_int, ct.c_int,
                                  ct.c_int, ct.c_double, ct.c_int, _dp,
                                  ct.POINTER(ct.c_int32)]
    L.or_decode_batch.restype = ct.c_int
    return L


def ref_available():
    return os.path.exists(REF_LIB)


def ref_lib():
    L = _load(REF_LIB, "ref")
    for n in ("sumprod", "sumprod2"):
        getattr(L, n).argtypes = [_dp, _lp, _lp, _lp, ct.c_int, ct.c_int, ct.c_int, _dp, ct.c_int]
        getattr(L, n).restype = ct.c_int
    L.minsum.argtypes = [_dp, _lp, _lp, _lp, ct.c_int, ct.c_int, ct.c_int, _dp, ct.c_double,
                         ct.c_int]
    L.minsum.restype = ct.c_int
    L.Lxor.argtypes = [ct.c_double, ct.c_double, ct.c_int]
    L.Lxor.restype = ct.c_double
    L.Lxfb.argtypes = [_dp, ct.c_int64, ct.c_int]
    L.Lxfb.restype = ct.c_double
    return L


def _graph(vdeg, cdeg, intrlv):
    return (np.ascontiguousarray(vdeg, dtype=np.int64), np.ascontiguousarray(cdeg, dtype=np.int64),
            np.ascontiguousarray(intrlv, dtype=np.int64))


def decode(kind, ch, vdeg, cdeg, intrlv, max_it=200, factor=0.7, use_ref=False):
    """One codeword: returns (app, it).  kind in KINDS.  use_ref=True runs the
    reference's own c_ldpc.c (minsum_refbug then means the shipped minsum)."""
    v, c, i = _graph(vdeg, cdeg, intrlv)
    ch = np.ascontiguousarray(ch, dtype=np.float64)
    app = np.zeros(len(v), dtype=np.float64)
    args = (ch.ctypes.data_as(_dp), v.ctypes.data_as(_lp), c.ctypes.data_as(_lp),
            i.ctypes.data_as(_lp), len(v), len(c), len(i), app.ctypes.data_as(_dp))
    if use_ref:
        L = ref_lib()
        if kind == "sumprod":
            it = L.sumprod(*args, int(max_it))
        elif kind == "sumprod2":
            it = L.sumprod2(*args, int(max_it))
        elif kind == "minsum_refbug":
            it = L.minsum(*args, float(factor), int(max_it))
        else:
            raise ValueError("the reference has no corrected minsum")
    else:
        L = oracle_lib()
        if kind in ("sumprod", "sumprod2"):
            it = getattr(L, "or_" + kind)(*args, int(max_it))
        else:
            it = getattr(L, "or_" + kind)(*args, float(factor), int(max_it))
    return app, it


def decode_batch(kind, ch, vdeg, cdeg, intrlv, max_it=200, factor=0.7):
    """[B, N] batch on one host thread with the restatement."""
    v, c, i = _graph(vdeg, cdeg, intrlv)
    ch = np.ascontiguousarray(ch, dtype=np.float64)
    B = ch.shape[0]
    app = np.zeros_like(ch)
    its = np.zeros(B, dtype=np.int32)
    r = oracle_lib().or_decode_batch(KINDS[kind], ch.ctypes.data_as(_dp), B, v.ctypes.data_as(_lp),
                                     c.ctypes.data_as(_lp), i.ctypes.data_as(_lp), len(v), len(c),
                                     len(i), float(factor), int(max_it), app.ctypes.data_as(_dp),
                                     its.ctypes.data_as(ct.POINTER(ct.c_int32)))
    if r != 0:
        raise RuntimeError("oracle decode failed")
    return app, its


def lxor(a, b, corr=1, use_ref=False):
    return (ref_lib().Lxor if use_ref else oracle_lib().or_lxor)(float(a), float(b), int(corr))


def lxfb(L, corr=1, use_ref=False):
    L = np.array(L, dtype=np.float64)
    f = ref_lib().Lxfb if use_ref else oracle_lib().or_lxfb
    agg = f(L.ctypes.data_as(_dp), len(L), int(corr))
    return agg, L


def minsum_numpy(ch, vdeg, cdeg, intrlv, max_it, factor, dtype=np.float32):
    """Flooding min-sum (c_ldpc.c:339-381 with the corrected message index of
    :364; Lxfb(corr=0) in its min / sign-parity form, c_ldpc.c:294-314) in
    `dtype`, vectorised over the codewords: the variable sums in port order
    (:171-178), one multiply of every check output by the factor (:370-371),
    the stopping rule of :196-197.  Returns (app[B, N], it int32[B]).  In
    float64 it equals or_decode_batch("minsum") bit for bit; in float32 it is
    the arithmetic of the GPU's single-precision kernel."""
    ch = np.asarray(ch, dtype=dtype)
    vdeg, cdeg, intrlv = (np.asarray(a, dtype=np.int64) for a in (vdeg, cdeg, intrlv))
    B, N = ch.shape
    Nc = len(cdeg)
    vstart = np.concatenate([[0], np.cumsum(vdeg)[:-1]])
    cstart = np.concatenate([[0], np.cumsum(cdeg)[:-1]])
    msg = np.zeros((B, len(intrlv)), dtype)
    f = dtype(factor)
    app = np.zeros((B, N), dtype)
    its = np.full(B, max_it, np.int32)
    live = np.ones(B, bool)
    vk = [(np.nonzero(vdeg > k)[0], intrlv[vstart[vdeg > k] + k]) for k in range(int(vdeg.max()))]
    ck = [(np.nonzero(cdeg > k)[0], cstart[cdeg > k] + k) for k in range(int(cdeg.max()))]
    for it in range(max_it):
        acc = ch.copy()
        for v, idx in vk:  # c_ldpc.c:171-178, ports in order
            acc[:, v] = acc[:, v] + msg[:, idx]
        for v, idx in vk:
            msg[:, idx] = acc[:, v] - msg[:, idx]
        app[live] = acc[live]
        L = np.full((B, Nc, int(cdeg.max())), np.inf, dtype)
        for k, (c, idx) in enumerate(ck):
            L[:, c, k] = msg[:, idx]
        a = np.abs(L)
        sb = np.signbit(L)
        i1 = np.argmin(a, axis=2)  # first minimum (strict '<' in the loop)
        m1 = np.take_along_axis(a, i1[..., None], 2)[..., 0]
        a2 = a.copy()
        np.put_along_axis(a2, i1[..., None], np.inf, 2)
        m2 = a2.min(axis=2)
        sall = np.bitwise_xor.reduce(sb, axis=2)
        unsat = sall | ~(m1 > 0)
        for k, (c, idx) in enumerate(ck):
            mag = np.where(i1[:, c] == k, m2[:, c], m1[:, c])
            neg = sall[:, c] ^ sb[:, c, k]
            msg[:, idx] = np.where(neg, -mag, mag) * f
        done = live & ~unsat.any(axis=1)
        its[done] = it
        live &= ~done
        if not live.any():
            break
    return app, its
