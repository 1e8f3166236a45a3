"""The device-resident concatenated pipeline (pipeline.py) against the
reference-call-surface path (sparc_new.sparc_ldpc_decode per codeword, itself
pinned to the reference by test_dense_gpu.py) on the same received words."""
import numpy as np
import pytest

from ldpc_sparc_amd import param_calc, sparc_new
from ldpc_sparc_amd.pipeline import ConcatPipeline

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_pipeline_equals_per_codeword_decode(precision):
    L_sparc, R_sl, L, lengths, rate = param_calc.param_calc_semi_protected(1.0, 1, 0.8, 64, '802.11n', '1/2', 0.5,
                                                                           27)
    M, P = 64, 15.0
    n = int(L * 6 / R_sl)
    rng = np.random.default_rng(0)
    A = rng.normal(0, 1 / np.sqrt(n), (n, L * M))
    pipe = ConcatPipeline(L, M, n, P, lengths['L_unprotected'], lengths['mults'], ldpc=('802.11n', '1/2', 27),
                          precision=precision, A=A)
    B = 6
    idx, info = pipe.make_batch(B, 2.0, np.random.default_rng(1))
    pipe.reset_counts()
    pipe.decode()
    cnt = pipe.counts()
    dt = pipe.dt
    Y = pipe.d_y.download(np.empty((B, n), dt)).astype(np.float64)
    sp = {'P': P, 'R': R_sl, 'L': L, 'M': M}
    lp = {'standard': '802.11n', 'rate': '1/2', 'z': 27}
    logM = 6
    errs = 0
    cw_err = 0
    for b in range(B):
        bits = sparc_new.sparc_ldpc_decode(Y[b], sp, lp, {'t_max': 25, 'precision': precision}, True, lengths, A)
        unp = ((idx[b, :lengths['L_unprotected']][:, None] >> np.arange(logM)[::-1]) & 1).ravel()
        truth = np.concatenate([unp, info.reshape(B, -1)[b]])
        e = int(np.sum(bits != truth))
        errs += e
        cw_err += e > 0
    assert cnt[0] == B
    assert cnt[1] == errs and cnt[2] == cw_err
    assert cnt[3] + cnt[4] == cnt[1]


def test_device_batch_encodes_valid_codewords():
    """make_batch_device (throughput mode): Philox bits, the LDPC encoder on
    the GPU, MSB-first section indices and AWGN -- the protected sections carry
    the host QC encoder's codewords of the drawn information words
    (ldpc.py:400-460), the unprotected sections the drawn bits, the noise has
    the requested variance, and the draw depends only on (seed, stream)."""
    L, M, n, Lu = 80, 512, 600, 8
    pipe = ConcatPipeline(L, M, n, 15.0, Lu, 1, ldpc=("802.11n", "1/2", 27), design_seed=3)
    c = pipe.c
    B, var = 64, 0.7
    pipe.make_batch_device(B, var, 7, (3 << 32) | 5)
    idx = pipe.d_true.download(np.zeros((B, L), np.int32))
    info = pipe.d_info.download(np.zeros((B, c.K), np.uint8))
    unp = pipe.d_unp.download(np.zeros((B, Lu * 9), np.uint8))
    bits = ((idx[:, :, None] >> np.arange(9)[::-1]) & 1).reshape(B, L * 9)
    assert np.array_equal(bits[:, :Lu * 9], unp)
    assert np.array_equal(bits[:, Lu * 9:], c.encode_batch(info.astype(np.int64)))
    x = pipe.d_x.download(np.zeros((B, n), np.float32)).astype(np.float64)
    y = pipe.d_y.download(np.zeros((B, n), np.float32)).astype(np.float64)
    d = y - x
    assert abs(d.var() - var) < 0.05 * var and abs(d.mean()) < 0.02
    pipe.make_batch_device(B, var, 7, (3 << 32) | 5)
    assert np.array_equal(pipe.d_y.download(np.zeros((B, n), np.float32)), y.astype(np.float32))
    pipe.make_batch_device(B, var, 7, (3 << 32) | 6)
    assert not np.array_equal(pipe.d_true.download(np.zeros((B, L), np.int32)), idx)
