"""C5 (BASELINE.json configs[4]) at full size: SPARC(L=1024, M=512) with a
dense Gaussian design, n = 9216, semi-protected by 4 x 802.11n r1/2 z=81 blocks
(L_unprotected = 160; param_calc.py:31-58, sparc_new.py:53-82,
performance_plots_general.py:101-118), decoded by the device pipeline
(pipeline.ConcatPipeline: matrix-core AMP -> MAP -> glue -> batched f32
sumprod2 BP -> device counters), checked three ways:

(a) one full AMP iteration (sparc_new.py:901-910) against float64 products on
    the host: A is read back from the device plan in row blocks and
    s1 = A^T y, z2 = y - A beta1 + (z/tau^2)(P - |beta1|^2/n), s2 = beta1 + A^T z2
    and eta (sparc_new.py:1040-1066) are recomputed in float64 from the GPU's
    own state.  Bar: products within 2e-5 of max|s| (test_dense_gpu.py's
    matrix-core bar), beta within 2e-5 sqrt(n P_l);
(b) the glue and the 4-block BP on the GPU's final beta: LLRs against
    oracle/sparc_ref.beta_to_bit_probs + the clip/log of ldpc_bp
    (sparc_new.py:1118-1138,1167-1169) in float64, within 1e-5 (plus the
    float64 conditioning of log(1 - p), see _llr_bar); the GPU's f64 sumprod2
    on those LLRs equal to oracle/bp_oracle.c (iterations, decisions, app within
    1e-9); the shipped f32 sumprod2 with the oracle's decisions on every block
    the oracle decodes; the device error counters equal to a host recount;
(c) FER at 6.0 dB on 512 fresh codewords within 3 standard deviations of the
    committed 16384-codeword sweep (profiles/r02_c5_sweep_n9216_16384.jsonl,
    FER 0.1393), and no protected-bit error there.
"""
import ctypes as ct

import numpy as np
import pytest

from ldpc_sparc_amd import _native
from ldpc_sparc_amd.montecarlo import ConcatTrial
from ldpc_sparc_amd.pipeline import ConcatPipeline
from oracle import bp, sparc_ref

pytestmark = pytest.mark.gpu

L, M, N_CH, P, L_UNP, MULTS = 1024, 512, 9216, 15.0, 160, 4
LOGM = 9
ROWS = 256  # row block of A read back per copy (512 MB of f32)


def _awgn_var(ebn0, c):
    user_bits = L_UNP * LOGM + MULTS * c.K
    return P / (2 * (user_bits / N_CH) * 10 ** (ebn0 / 10))


@pytest.fixture(scope="module")
def pipe():
    p = ConcatPipeline(L, M, N_CH, P, L_UNP, MULTS, ldpc=("802.11n", "1/2", 81), design_seed=0, precision="f32",
                       t_max=25, bp_its=200)
    yield p
    p.design.release()


def _a_blocks(pipe):
    """Row blocks of the device plan's A as float64 (rows i0:i1)."""
    lib = _native.lib()
    dA = ct.c_void_p()
    _native.check(lib.sg_dense_plan_matrix_device(pipe.plan, ct.byref(dA)))
    LM = L * M
    buf = np.empty((ROWS, LM), np.float32)
    for i0 in range(0, N_CH, ROWS):
        r = min(ROWS, N_CH - i0)
        _native.check(lib.sg_memcpy_d2h(_native.ptr(buf), _native.offset(dA, 4 * i0 * LM), 4 * r * LM, None))
        if (i0 // ROWS) % 12 == 0:
            print(f"  A rows {i0}..{i0 + r} of {N_CH}", flush=True)  # progress (a long host pass)
        yield i0, i0 + r, buf[:r].astype(np.float64)


def _state(pipe, B):
    """(beta, s) of the first B codewords of the plan's state, as float64."""
    d_beta, d_s = ct.c_void_p(), ct.c_void_p()
    _native.check(_native.lib().sg_dense_state_device(pipe.plan, ct.byref(d_beta), ct.byref(d_s)))
    _native.synchronize()
    out = []
    for d in (d_beta, d_s):
        a = np.empty((B, L * M), np.float32)
        _native.check(_native.lib().sg_memcpy_d2h(_native.ptr(a), d, a.nbytes, None))
        out.append(a.astype(np.float64))
    return out


def _amp(pipe, B, t_max, rows=None):
    _native.check(_native.lib().sg_dense_amp_device(pipe.plan, pipe.d_y.ptr, B, t_max, None, None, None))
    return _state(pipe, B if rows is None else rows)


@pytest.mark.parametrize("ebn0", [4.5, 6.0])
def test_c5_one_amp_iteration_vs_float64(pipe, ebn0):
    B = 8
    pipe.make_batch_device(B, _awgn_var(ebn0, pipe.c), 2024, 7)
    y = pipe.d_y.download(np.empty((B, N_CH), np.float32)).astype(np.float64)
    beta1, s1 = _amp(pipe, B, 1)
    beta2, s2 = _amp(pipe, B, 2)
    _check_vs_float64(pipe, y, beta1, s1, beta2, s2)


def test_c5_shipped_wide_tile_b256(pipe):
    """The instance the C5 line times: at B = 256 both GEMMs run
    gemm_f32_mfma<*, 4> (256-row block tiles, dense.hip:160-166), at B <= 128
    the <*, 2> form.  The batch draw of codeword b depends only on (seed,
    stream, b), so codewords 0-7 of a 256-codeword batch are the received
    words of an 8-codeword batch: y (x = A beta0 through the NT GEMM), beta and
    s after one and two iterations must be bit-identical between the two
    instances (dense.hip:24: same k-order per output), and the B = 256 rows are
    checked against float64 products as in the test above
    (sparc_new.py:901-910)."""
    K = 8
    var = _awgn_var(6.0, pipe.c)
    got = {}
    for B in (256, K):
        pipe.make_batch_device(B, var, 5150, 3)
        y = pipe.d_y.download(np.empty((B, N_CH), np.float32))[:K]
        beta1, s1 = _amp(pipe, B, 1, rows=K)
        beta2, s2 = _amp(pipe, B, 2, rows=K)
        got[B] = (y, beta1, s1, beta2, s2)
    for name, a, b in zip(("y", "beta1", "s1", "beta2", "s2"), got[256], got[K]):
        assert np.array_equal(a, b), f"{name}: B = 256 (<*, 4>) differs from B = 8 (<*, 2>)"
    print("  B = 256 rows 0-7 bit-identical to the B = 8 batch (y, beta, s at t = 1, 2)", flush=True)
    y, beta1, s1, beta2, s2 = got[256]
    _check_vs_float64(pipe, y.astype(np.float64), beta1, s1, beta2, s2)


def _check_vs_float64(pipe, y, beta1, s1, beta2, s2):
    B = y.shape[0]
    Pl = P / L
    snp = np.sqrt(N_CH * Pl)
    # pass 1: s1 = A^T y (beta = 0 at t = 0) and A beta1
    s1_ref = np.zeros((B, L * M))
    ab1 = np.zeros((B, N_CH))
    for i0, i1, A in _a_blocks(pipe):
        s1_ref += y[:, i0:i1] @ A
        ab1[:, i0:i1] = beta1 @ A.T
    e1 = np.max(np.abs(s1 - s1_ref)) / np.abs(s1_ref).max()
    print(f"  s1 = A^T y: max error {e1:.2e} of max|s| (bar 2e-5)", flush=True)
    assert e1 < 2e-5
    tau1 = np.sum(y ** 2, axis=1) / N_CH
    for b in range(B):
        ref = sparc_ref.dense_mmse_estimator(s1[b], tau1[b], N_CH, Pl, M)
        assert np.max(np.abs(beta1[b] - ref)) < 2e-5 * snp, b
    # t = 1: residual with the Onsager term, then s2 = beta1 + A^T z2
    z2 = y - ab1 + (y / tau1[:, None]) * (P - np.sum(beta1 ** 2, axis=1) / N_CH)[:, None]
    s2_ref = beta1.copy()
    for i0, i1, A in _a_blocks(pipe):
        s2_ref += z2[:, i0:i1] @ A
    e2 = np.max(np.abs(s2 - s2_ref)) / np.abs(s2_ref).max()
    print(f"  s2 = beta1 + A^T z2: max error {e2:.2e} of max|s| (bar 2e-5)", flush=True)
    assert e2 < 2e-5
    tau2 = np.sum(z2 ** 2, axis=1) / N_CH
    for b in range(B):
        ref = sparc_ref.dense_mmse_estimator(s2[b], tau2[b], N_CH, Pl, M)
        assert np.max(np.abs(beta2[b] - ref)) < 2e-5 * snp, b


def _llr_bar(p):
    """|LLR_gpu - LLR_ref| allowance: 1e-5 (f32 output) plus the float64
    rounding of p amplified by 1 / min(p, 1 - p) (the device and the host sum
    the same f32 values in different orders)."""
    pc = np.clip(p, 1e-15, 1 - 1e-15)
    return 1e-5 * np.maximum(1.0, np.abs(np.log(pc) - np.log(1 - pc))) + 4e-16 / np.minimum(pc, 1 - pc)


@pytest.mark.parametrize("ebn0", [4.5, 6.0])
def test_c5_glue_and_bp_vs_oracle(pipe, ebn0):
    c = pipe.c
    B = 8
    pipe.make_batch_device(B, _awgn_var(ebn0, c), 4048, 11)
    pipe.reset_counts()
    pipe.decode()
    cnt = pipe.counts()
    beta, s = _state(pipe, B)
    snp = np.sqrt(N_CH * P / L)
    nb = B * MULTS
    llr = pipe.d_llr.download(np.empty((nb, c.N), np.float32)).astype(np.float64)
    app = pipe.d_app.download(np.empty((nb, c.N), np.float32))
    # glue: bit probabilities of the protected sections of the GPU's beta, clip, log
    for b in range(B):
        p = sparc_ref.beta_to_bit_probs(beta[b, L_UNP * M:], L - L_UNP, M, snp)
        pc = np.clip(p, 1e-15, 1 - 1e-15)
        ref = np.log(pc) - np.log(1 - pc)
        got = llr[b * MULTS:(b + 1) * MULTS].ravel()
        assert np.all(np.abs(got - ref) <= _llr_bar(p)), b
    # BP: the oracle's f64 sumprod2 on the GPU's LLRs
    oapp, oit = bp.decode_batch("sumprod2", llr, c.vdeg, c.cdeg, c.intrlv, 200)
    app64, it64 = c.decode_batch(llr, 200, "sumprod2")  # GPU, f64: the reference precision
    assert np.array_equal(it64, oit)
    assert np.array_equal(app64 < 0, oapp < 0)
    assert np.max(np.abs(app64 - oapp) / np.maximum(1.0, np.abs(oapp))) < 1e-9
    conv = oit < 200
    print(f"  BP blocks the oracle decodes: {int(conv.sum())} of {nb}; f32 decisions differing on the others: "
          f"{int(((app < 0) != (oapp < 0))[~conv].sum())} bits", flush=True)
    if ebn0 >= 6.0:
        assert conv.all(), oit
    assert np.array_equal((app < 0)[conv], (oapp < 0)[conv])  # shipped f32 BP where the oracle decodes
    # device counters against a host recount from the same decisions
    true_idx = pipe.d_true.download(np.empty((B, L), np.int32))
    info = pipe.d_info.download(np.empty((B, MULTS * c.K), np.uint8))
    map_idx = s.reshape(B, L, M).argmax(axis=2)
    assert np.array_equal(map_idx, pipe.d_idx.download(np.empty((B, L), np.int32)))
    sh = np.arange(LOGM)[::-1]
    eu = (((map_idx[:, :L_UNP, None] >> sh) & 1) != ((true_idx[:, :L_UNP, None] >> sh) & 1)).sum(axis=(1, 2))
    hard = (app.reshape(B, MULTS, c.N)[:, :, :c.K] < 0).reshape(B, -1)
    ep = (hard != info).sum(axis=1)
    assert cnt[0] == B and cnt[3] == eu.sum() and cnt[4] == ep.sum()
    assert cnt[1] == (eu + ep).sum() and cnt[2] == ((eu + ep) > 0).sum()


def test_c5_fer_at_6db_vs_committed_sweep(pipe):
    """FER at 6.0 dB on 512 codewords of a fresh seed against the committed
    sweep point (16384 codewords, FER 0.1392822, no protected-bit error)."""
    c = pipe.c
    trial = ConcatTrial(pipe, [_awgn_var(6.0, c)], seed=977, rng="device")
    tot = trial(0, 0, 2, 256)
    n = int(tot[0])
    fer = tot[2] / n
    f0, n0 = 0.1392822265625, 16384
    sig = np.sqrt(f0 * (1 - f0) * (1 / n + 1 / n0))
    print(f"  FER {fer:.4f} on {n} codewords vs {f0:.4f} (3 sigma {3 * sig:.4f})", flush=True)
    assert abs(fer - f0) < 3 * sig, (fer, f0, sig)
    assert tot[4] == 0
