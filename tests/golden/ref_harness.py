"""Import the read-only reference (/root/reference) for fixture generation.

TEST INFRASTRUCTURE ONLY -- used by tests/golden/make_golden.py in the build
container.  Never imported by the product, never run on the GPU box (the
reference does not exist there).

Shims are applied from here, without editing any reference file
(SURVEY.md §8(c)):
  * numpy>=2 removed the aliases np.float / np.complex / np.object that
    sparc_public uses (sparc.py:415,463,465,803,839,916; sparc_sim.py:197,200);
  * int_2_bin_arr (sparc.py:191-197, sparc_new.py:1373-1378) casts a list of
    '0'/'1' characters to bool, which under numpy>=2 turns every '0' into True.
    The reference pins numpy 1.26.1 (requirements.txt) where it is correct; the
    shim restores that behaviour;
  * ldpc.code.decode (ldpc.py:463-490) dlopens a Windows DLL path and passes
    the graph as C `long` (32-bit under LLP64).  The shim calls the reference's
    own c_ldpc.c, compiled from source by oracle/Makefile into
    oracle/_ref/libc_ldpc_ref.so, with int64 graph arrays, and passes
    max_itcount to minsum (the shipped wrapper drops it, ldpc.py:487).
"""
import ctypes as ct
import os
import sys

import numpy as np

REF = os.environ.get("LDPC_SPARC_REFERENCE", "/root/reference")
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF_LIB = os.path.join(REPO, "oracle", "_ref", "libc_ldpc_ref.so")

_loaded = {}


def _int_2_bin_arr_np2(integer, arr_length):
    assert integer >= 0
    return np.array([c == "1" for c in np.binary_repr(integer, arr_length)], dtype=bool)


def ref_clib():
    if "clib" not in _loaded:
        if not os.path.exists(REF_LIB):
            raise RuntimeError("build oracle/_ref first: make -C oracle")
        lib = ct.CDLL(REF_LIB)
        dp = ct.POINTER(ct.c_double)
        lp = ct.POINTER(ct.c_long)
        for name in ("sumprod", "sumprod2"):
            f = getattr(lib, name)
            f.argtypes = [dp, lp, lp, lp, ct.c_int, ct.c_int, ct.c_int, dp, ct.c_int]
            f.restype = ct.c_int
        lib.minsum.argtypes = [dp, lp, lp, lp, ct.c_int, ct.c_int, ct.c_int, dp, ct.c_double,
                               ct.c_int]
        lib.minsum.restype = ct.c_int
        lib.Lxor.argtypes = [ct.c_double, ct.c_double, ct.c_int]
        lib.Lxor.restype = ct.c_double
        lib.Lxfb.argtypes = [dp, ct.c_long, ct.c_int]
        lib.Lxfb.restype = ct.c_double
        _loaded["clib"] = lib
    return _loaded["clib"]


def ref_decode(c, ch, max_itcount=200, dectype="sumprod2", corr_factor=0.7):
    """Reference c_ldpc.c decode with Linux-LP64 graph arrays."""
    lib = ref_clib()
    ch = np.ascontiguousarray(ch, dtype=np.float64)
    if len(ch) != len(c.vdeg):
        raise NameError("Channel inputs not consistent with variable degrees")
    vdeg = np.ascontiguousarray(c.vdeg, dtype=np.int64)
    cdeg = np.ascontiguousarray(c.cdeg, dtype=np.int64)
    intrlv = np.ascontiguousarray(c.intrlv, dtype=np.int64)
    app = np.zeros(c.Nv, dtype=np.float64)
    dp = ct.POINTER(ct.c_double)
    lp = ct.POINTER(ct.c_long)
    args = (ch.ctypes.data_as(dp), vdeg.ctypes.data_as(lp), cdeg.ctypes.data_as(lp),
            intrlv.ctypes.data_as(lp), c.Nv, c.Nc, c.Nmsg, app.ctypes.data_as(dp))
    if dectype == "sumprod":
        it = lib.sumprod(*args, int(max_itcount))
    elif dectype == "sumprod2":
        it = lib.sumprod2(*args, int(max_itcount))
    elif dectype == "minsum":
        it = lib.minsum(*args, float(corr_factor), int(max_itcount))
    else:
        raise NameError("Decoder type unknonwn")
    return app, it


def import_reference():
    """Return the reference modules: (ldpc, sparc, sparc_sim, sparc_new, sparc_sim_new, param_calc)."""
    if "mods" in _loaded:
        return _loaded["mods"]
    sys.dont_write_bytecode = True
    for name, val in (("float", float), ("complex", complex), ("object", object)):
        if not hasattr(np, name):
            setattr(np, name, val)
    for p in (REF, os.path.join(REF, "sparc_public"), os.path.join(REF, "ldpc_jossy", "py"),
              os.path.join(REF, "ldpc_sparc")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import importlib
    ldpc_mod = importlib.import_module("ldpc_jossy.py.ldpc")
    ldpc_mod.code.decode = lambda self, ch, max_itcount=200, dectype="sumprod2", corr_factor=0.7: \
        ref_decode(self, ch, max_itcount, dectype, corr_factor)
    sparc = importlib.import_module("sparc")
    sparc.int_2_bin_arr = _int_2_bin_arr_np2
    sparc_sim = importlib.import_module("sparc_sim")
    sparc_new = importlib.import_module("sparc_sophie.sparc_new")
    sparc_new.int_2_bin_arr = _int_2_bin_arr_np2
    sparc_sim_new = importlib.import_module("sparc_sophie.sparc_sim_new")
    param_calc = importlib.import_module("param_calc")
    _loaded["mods"] = (ldpc_mod, sparc, sparc_sim, sparc_new, sparc_sim_new, param_calc)
    return _loaded["mods"]
