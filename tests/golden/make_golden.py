"""Generate the committed golden fixtures under tests/golden/ from the reference.

Runs only in the build container (it imports /root/reference through
ref_harness and the reference's own c_ldpc.c built into oracle/_ref/).  The
fixtures are data (inputs and expected outputs); tests compare the HIP path
and the CPU restatement against them.

  python tests/golden/make_golden.py [ldpc] [sparc] [sophie]
"""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402


def _ebn0_llr(c, ebn0_db, rng):
    """Random codeword, BPSK 1-2x, sigma^2 = 1/(2 R Eb/N0), LLR 2y/sigma^2
    (ldpc_awgn.py:45-56 channel model)."""
    R = c.K / c.N
    s2 = 1.0 / (2 * R * 10 ** (ebn0_db / 10))
    u = rng.integers(0, 2, c.K)
    x = c.encode(u)
    y = (1.0 - 2.0 * x) + np.sqrt(s2) * rng.standard_normal(c.N)
    return x, 2.0 * y / s2


def make_ldpc():
    ldpc = ref_harness.import_reference()[0]
    out = {}
    # --- 802.16 r1/2 z=81 graph arrays from the reference's C test header
    hdr = open(os.path.join(ref_harness.REF, "ldpc_jossy", "src", "ldpc802.16.81.h")).read()

    def arr(name):
        m = re.search(r"\b%s\s*\[[^\]]*\]\s*=\s*\{([^}]*)\}" % name, hdr)
        return np.array([int(t) for t in m.group(1).replace("\n", " ").split(",") if t.strip()],
                        dtype=np.int64)
    out["h16_81_intrlv"] = arr("intrlv")
    out["h16_81_vdeg"] = arr("vdeg")
    out["h16_81_cdeg"] = arr("cdeg")
    # --- encoder I/O and decoder vectors, reference code + reference C core
    cases = [("802.11n", "1/2", 81, 4), ("802.11n", "1/2", 27, 8), ("802.16", "2/3", 27, 4)]
    for ci, (std, rate, z, ncw) in enumerate(cases):
        c = ldpc.code(std, rate, z)
        tag = f"c{ci}"
        out[f"{tag}_meta"] = np.array([std, rate, str(z)])
        out[f"{tag}_intrlv"] = c.intrlv
        rng = np.random.default_rng(1000 + ci)
        U = rng.integers(0, 2, (4, c.K))
        out[f"{tag}_enc_u"] = U.astype(np.uint8)
        out[f"{tag}_enc_x"] = np.array([c.encode(u) for u in U], dtype=np.uint8)
        for ei, ebn0 in enumerate((1.0, 1.5, 2.0)):
            X, LLR = [], []
            for _ in range(ncw):
                x, llr = _ebn0_llr(c, ebn0, rng)
                X.append(x)
                LLR.append(llr)
            out[f"{tag}_e{ei}_x"] = np.array(X, dtype=np.uint8)
            out[f"{tag}_e{ei}_ch"] = np.array(LLR)
            for dt in ("sumprod", "sumprod2", "minsum"):
                for mi in (5, 50, 200):
                    apps, its = [], []
                    for llr in LLR:
                        a, it = c.decode(llr, mi, dt, 0.7)   # reference c_ldpc.c (shim)
                        apps.append(a)
                        its.append(it)
                    key = f"{tag}_e{ei}_{dt}_{mi}"
                    its = np.array(its, dtype=np.int32)
                    out[key + "_it"] = its
                    if mi != 200:
                        out[key + "_app"] = np.array(apps)
                    else:
                        out[key + "_hard"] = (np.array(apps) < 0).astype(np.uint8)
    np.savez_compressed(os.path.join(HERE, "ldpc_golden.npz"), **out)
    print("wrote ldpc_golden.npz", sum(v.nbytes for v in out.values()) / 1e6, "MB raw")


if __name__ == "__main__":
    which = sys.argv[1:] or ["ldpc", "sparc", "sophie"]
    if "ldpc" in which:
        make_ldpc()
    if "sparc" in which:
        from make_golden_sparc import make_sparc
        make_sparc()
    if "sophie" in which:
        from make_golden_sparc import make_sophie
        make_sophie()
