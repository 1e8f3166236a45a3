"""The polar form of the split engine's inverse coefficients (capi_amp.cpp
build_cw2, amp_cw2.hip cw2_az rows), restated in numpy and checked on every
output of the C2 design and of a w = 2^19 design (CPU; the GPU suite runs the
engine built from the same fit: tests/test_amp_cw2_gpu.py).

Output i at DCT position q reads H[a], H[b] (fwd_coef, the Makhoul packed FFT
of sparc.py:687-692) and its inverse input adds al z/phi to G[a] and be z/phi
to G[b] (inv_contrib, sparc.py:694-699).  After the pair normalisation (a mod
P the smaller row of {r, P - r}; a swap exchanges al and be) the claim is

    al = |al| e^(2 pi i A / 4N),  be = |be| e^(2 pi i (N - A) / 4N),
    A = 3a + o N/2,  o in {0, 1, 6, 7} by the output's case,

so the rows' al conj(W) and be W (W = w_N2^(m2 a)) come from one angle per
slot and class.
"""
import numpy as np
import pytest

from ldpc_sparc_amd import sparc

P = 8192


def _coefficients(q, N):
    """fwd_coef's a, b and inv_contrib's (al, be) of DCT positions q (vectorised, float64)."""
    N2 = N // 2
    q = q.astype(np.int64)
    kk = np.where(q <= N2, q, N - q)
    a, b = kk % N2, (N2 - kk) % N2
    g = 1 / np.sqrt(2.0)
    e = lambda x: np.exp(1j * np.pi * x)  # noqa: E731
    Ak = lambda k: e(k / (2 * N)) * (1 + 1j * np.exp(2j * np.pi * (k % N) / N))  # noqa: E731
    Ck = lambda k: e((k + N2) / (2 * N)) * (1 - 1j * np.exp(2j * np.pi * (k % N) / N))  # noqa: E731
    lo, hi = q < N2, q > N2
    al = np.where(lo, Ak(q) * g, np.where(hi, -1j * Ak(N - q) * g, Ck(0) * (1 - 1j) * g))
    be = np.where(lo, -1j * Ck(N2 - q) * g, np.where(hi, Ck(q - N2) * g, 0))
    return a, b, al, be


@pytest.mark.parametrize("L,M,R", [(1024, 512, 1.5), (1024, 512, 1.3), (512, 512, 1.2)])
def test_polar_fit_every_output(L, M, R):
    n = int(round(L * np.log2(M) / R))
    o0, _ = sparc.generate_ordering(np.array(15.0), n, L * M, 41)
    N = sparc.transform_size(n, L * M)
    N4 = 4 * N
    a, b, al, be = _coefficients(np.asarray(o0), N)
    r = a % P
    swap = r > (P - r) % P
    a = np.where(swap, b, a)
    al, be = np.where(swap, be, al), np.where(swap, al, be)
    best_err = np.full(len(a), np.inf)
    code = np.zeros(len(a), np.int64)
    for o in (0, 1, 6, 7):
        A = (3 * a + o * (N // 2)) % N4
        ra = al * np.exp(-2j * np.pi * A / N4)
        rb = be * np.exp(-2j * np.pi * (N - A) / N4)
        err = np.abs(ra.imag) + np.abs(rb.imag)
        better = err < best_err
        best_err[better], code[better] = err[better], o
    assert np.all(best_err <= 1e-12 * (np.abs(al) + np.abs(be)))
    # the offset is the output's case: q below / above N2, swapped or not (q = N2: o = 7, be = 0)
    q = np.asarray(o0).astype(np.int64)
    expect = np.where(q < N // 2, np.where(swap, 6, 1), np.where(swap, 0, 7))
    assert np.array_equal(code, expect)
    # one angle per slot and class gives both row values: x = ((3 + 8 m2) a + o N/2) / 4N revolutions
    mag_a = np.real(al * np.exp(-2j * np.pi * ((3 * a + code * (N // 2)) % N4) / N4))
    mag_b = np.real(be * np.exp(-2j * np.pi * ((N - 3 * a - code * (N // 2)) % N4) / N4))
    N2 = N // 2
    for m2 in (0, 1, 17, 63):
        W = np.exp(-2j * np.pi * ((m2 * a) % N2) / N2)
        x = (((3 + 8 * m2) * a + code * (N // 2)) % N4) / N4
        cs = np.exp(2j * np.pi * x)
        np.testing.assert_allclose(mag_a * cs, al * np.conj(W), atol=1e-12)
        np.testing.assert_allclose(mag_b * (cs.imag + 1j * cs.real), be * W, atol=1e-12)
