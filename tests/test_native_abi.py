"""CPU tests of the C-ABI boundary: the library loads, exports every symbol the
public header declares, and refuses to decode without a GPU (no CPU path)."""
import ctypes as ct
import os
import re

import numpy as np
import pytest

from ldpc_sparc_amd import _native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ldpc_sparc_amd.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", src, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "while", "for", "return")))


def test_header_lists_functions():
    names = header_functions()
    for must in ("sg_ldpc_decode", "sumprod2", "minsum", "Lxfb", "sg_last_error"):
        assert must in names


def test_library_exports_every_header_symbol():
    lib = _native.lib()
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_bindings_cover_header():
    bound = {n for n, _, _ in _native.SIGNATURES}
    assert set(header_functions()) <= bound


def test_no_cpu_fallback_without_gpu():
    if _native.device_count() > 0:
        pytest.skip("GPU present")
    from ldpc_sparc_amd.ldpc import code
    c = code()
    with pytest.raises(_native.NativeError, match="no GPU"):
        c.decode(np.ones(c.N))
    # reference-compatible C entry point reports failure with a negative code
    L = _native.lib()
    ch = np.ones(c.N)
    app = np.zeros(c.N)
    v = c.vdeg.astype(np.int64); cd = c.cdeg.astype(np.int64); i = c.intrlv.astype(np.int64)
    r = L.sumprod2(ch.ctypes.data_as(_native.dp), v.ctypes.data_as(_native.lp),
                   cd.ctypes.data_as(_native.lp), i.ctypes.data_as(_native.lp),
                   c.Nv, c.Nc, c.Nmsg, app.ctypes.data_as(_native.dp), 10)
    assert r < 0
    assert b"no GPU" in L.sg_last_error()
