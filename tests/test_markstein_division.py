"""The f64 staged engine computes the softmax argument's v / tau as a
Markstein division by the staged reciprocal (amp_fused.hip sm_arg_st):
q = v r, r = RN(1 / tau), then q + fma(-q, tau, v) r.  That is the correctly
rounded quotient wherever q is within one ulp of v / tau, which RN(v r) does
not guarantee in every corner, so the claim is empirical:
tools/markstein_check.c compares it with the IEEE division over 10^8 random
pairs spanning the decoder's range (tau 2^-12 .. 2^8, |v| up to 2^12), corner
pairs (divisor significands near 1 and 2, quotients next to powers of two)
and every value of the divisor's low 16 significand bits, with the host's
fused multiply-add, which rounds as v_fma_f64 does.  The f64 split engine
(amp_cw2d.hip d_arg) uses the same form."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_markstein_division_is_correctly_rounded(tmp_path):
    exe = tmp_path / "markstein_check"
    subprocess.run(["gcc", "-O2", "-mfma", os.path.join(ROOT, "tools", "markstein_check.c"), "-o", str(exe), "-lm"],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=120).stdout
    lines = out.strip().splitlines()
    assert lines and lines[-1].startswith("total: 0 of "), out
    assert all(" 0 of " in l for l in lines), out
