"""The f64 staged engine computes the softmax argument's v / tau as a
Markstein division by the staged reciprocal (amp_fused.hip sm_arg_st):
q = v r, r = RN(1 / tau), then q + fma(-q, tau, v) r.  That is the correctly
rounded quotient, so the engine's values equal those of the IEEE division it
replaced bit for bit.  tools/markstein_check.c checks it over 10^8 random
pairs spanning the decoder's range (tau 2^-12 .. 2^8, |v| up to 2^12) with
the host's fused multiply-add, which rounds as v_fma_f64 does."""
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
    assert out.strip().endswith("0 of 100000000 differ"), out
