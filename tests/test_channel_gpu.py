"""GPU tests of the throughput-mode encoder and channel (channel.hip,
sg_amp_encode_device) and of the device-generated Monte-Carlo trials.

Bars:
  * LDPC encoder: bit-exact with the host QC encoder (ldpc.py:400-460
    restatement, pinned by the reference fixtures) on random words, every
    802.11n rate at z = 27 and 81; codewords satisfy every parity check;
  * bits -> section indices: exact (MSB first, sparc.py:330-364);
  * x = A beta0 on the device: within 1e-12 (f64) of the operator applied to
    the one-hot vectors;
  * Philox bits / noise: deterministic per (seed, stream), independent of the
    batch split; moments within 5 standard errors;
  * device-generated LDPC and SPARC trials agree statistically with the host
    generator (same code, same SNR), and a campaign point gives identical
    totals on 1 and 2 simulated ranks.
"""
import numpy as np
import pytest

from ldpc_sparc_amd import _native, montecarlo, sparc
from ldpc_sparc_amd.ldpc import code

pytestmark = pytest.mark.gpu


def _lib():
    return _native.lib()


@pytest.mark.parametrize("rate", ["1/2", "2/3", "3/4", "5/6"])
@pytest.mark.parametrize("z", [27, 81])
def test_device_encoder_matches_host(rate, z):
    c = code("802.11n", rate, z)
    rng = np.random.default_rng(z)
    B = 64
    info = rng.integers(0, 2, (B, c.K)).astype(np.uint8)
    d_info = _native.DeviceBuffer.from_array(info)
    d_cw = _native.DeviceBuffer(B * c.N)
    c.encode_device(d_info.ptr, B, d_cw.ptr)
    _native.synchronize()
    cw = d_cw.download(np.zeros((B, c.N), np.uint8))
    assert np.array_equal(cw, c.encode_batch(info).astype(np.uint8))
    H = c.pcmat()
    assert not np.any((cw.astype(np.int64) @ H.T) % 2)


def test_rng_bits_deterministic_and_balanced():
    lib = _lib()
    B, nb = 16, 10000
    d = _native.DeviceBuffer(B * nb)
    _native.check(lib.sg_rng_bits_device(7, 3, B, nb, d.ptr, None))
    a = d.download(np.zeros((B, nb), np.uint8))
    _native.check(lib.sg_rng_bits_device(7, 3, B, nb, d.ptr, None))
    assert np.array_equal(a, d.download(np.zeros((B, nb), np.uint8)))
    _native.check(lib.sg_rng_bits_device(7, 4, B, nb, d.ptr, None))
    b = d.download(np.zeros((B, nb), np.uint8))
    assert not np.array_equal(a, b)
    assert set(np.unique(a)) <= {0, 1}
    p = a.mean()
    assert abs(p - 0.5) < 5 * 0.5 / np.sqrt(a.size)
    # rows are independent streams (no row equals another)
    assert len({r.tobytes() for r in a}) == B


def test_bits_to_sections():
    lib = _lib()
    B, L, logM = 5, 33, 9
    rng = np.random.default_rng(1)
    bits = rng.integers(0, 2, (B, L * logM)).astype(np.uint8)
    d_b = _native.DeviceBuffer.from_array(bits)
    d_i = _native.DeviceBuffer(B * L * 4)
    _native.check(lib.sg_bits_to_sections_device(d_b.ptr, B, L, logM, d_i.ptr, None))
    idx = d_i.download(np.zeros((B, L), np.int32))
    ref = bits.reshape(B, L, logM).astype(np.int64) @ (1 << np.arange(logM)[::-1])
    assert np.array_equal(idx, ref)


@pytest.mark.parametrize("prec", [_native.SG_F64, _native.SG_F32])
def test_awgn_moments(prec):
    lib = _lib()
    B, n, sigma = 8, 100001, 0.7
    dt = np.float64 if prec == _native.SG_F64 else np.float32
    x = np.full((B, n), 0.25, dt)
    d_x = _native.DeviceBuffer.from_array(x)
    d_y = _native.DeviceBuffer(x.nbytes)
    _native.check(lib.sg_awgn_device(prec, 11, 5, d_x.ptr, B, n, sigma, d_y.ptr, None))
    g = (d_y.download(np.zeros_like(x)).astype(np.float64) - 0.25) / sigma
    N = g.size
    assert abs(g.mean()) < 5 / np.sqrt(N)
    assert abs(g.var() - 1) < 5 * np.sqrt(2 / N)
    assert abs(np.mean(g ** 4) - 3) < 5 * np.sqrt(96 / N)  # Gaussian fourth moment
    assert abs(np.corrcoef(g[:, :-1].ravel(), g[:, 1:].ravel())[0, 1]) < 5 / np.sqrt(N)


def test_bpsk_llr_statistics():
    lib = _lib()
    B, N, sigma2 = 32, 1944, 0.8
    rng = np.random.default_rng(2)
    cw = rng.integers(0, 2, (B, N)).astype(np.uint8)
    d_c = _native.DeviceBuffer.from_array(cw)
    d_l = _native.DeviceBuffer(B * N * 8)
    _native.check(lib.sg_bpsk_awgn_llr_device(_native.SG_F64, 3, 9, d_c.ptr, B, N, sigma2, d_l.ptr, None))
    llr = d_l.download(np.zeros((B, N)))
    y = llr * sigma2 / 2.0
    g = (y - (1.0 - 2.0 * cw)) / np.sqrt(sigma2)
    assert abs(g.mean()) < 5 / np.sqrt(g.size)
    assert abs(g.var() - 1) < 5 * np.sqrt(2 / g.size)


@pytest.mark.parametrize("prec,tol", [(_native.SG_F64, 1e-12), (_native.SG_F32, 2e-6)])
def test_amp_encode_device(prec, tol):
    L, M, R = 64, 64, 1.2
    n = int(round(L * 6 / R))
    W = np.array(15.0)
    o0, o1 = sparc.generate_ordering(W, n, L * M, 4)
    op = sparc.DesignOperator(W, L, M, n, o0, o1)
    B = 3
    rng = np.random.default_rng(4)
    idx = rng.integers(0, M, (B, L)).astype(np.int32)
    beta0 = np.zeros((B, L * M))
    beta0[np.arange(B)[:, None], np.arange(L) * M + idx] = 1.0
    ref = op.apply(beta0, False, _native.SG_F64)
    es = 8 if prec == _native.SG_F64 else 4
    d_i = _native.DeviceBuffer.from_array(idx)
    d_x = _native.DeviceBuffer(B * n * es)
    _native.check(_lib().sg_amp_encode_device(op.plan(prec), d_i.ptr, B, d_x.ptr, None))
    _native.synchronize()
    x = d_x.download(np.zeros((B, n), np.float64 if es == 8 else np.float32)).astype(np.float64)
    assert np.max(np.abs(x - ref)) <= tol * np.max(np.abs(ref))


def test_ldpc_trial_device_matches_host_statistically():
    c = code("802.11n", "1/2", 27)
    snr = 1.0  # Es/N0 dB: frame error rate of a few tens of percent
    host = montecarlo.LdpcTrial(c, [snr], max_it=50, precision="f32", seed=1, rng="host")
    dev = montecarlo.LdpcTrial(c, [snr], max_it=50, precision="f32", seed=1, rng="device")
    h = host(0, 0, 16, 256)
    d = dev(0, 0, 16, 256)
    assert h[0] == d[0] == 4096
    ph, pd = h[2] / h[0], d[2] / d[0]
    se = np.sqrt(max(ph * (1 - ph), 1e-4) * 2 / h[0])
    assert abs(ph - pd) < 5 * se, (ph, pd)
    assert 0.01 < pd < 0.99


def test_device_trial_is_rank_invariant():
    c = code("802.11n", "1/2", 27)
    tr = montecarlo.LdpcTrial(c, [1.2], max_it=30, precision="f32", seed=5, rng="device")
    agg = montecarlo.Aggregator()
    one = montecarlo.run_point(tr, 0, block=64, blocks_per_round=6, rank=0, world=1, agg=agg, max_units=64 * 6)
    parts = [tr(0, a, b - a, 64) for a, b in (montecarlo.shard_range(6, r, 2) for r in range(2))]
    assert np.array_equal(one, parts[0] + parts[1])


def test_sparc_trial_device_generation():
    """C2-shaped regular SPARC at reduced L: R = 1.0 decodes, R = 1.6 does not."""
    L, M = 128, 512
    W = np.array(15.0)
    res = {}
    for R in (1.0, 1.6):
        n = int(round(L * 9 / R))
        o0, o1 = sparc.generate_ordering(W, n, L * M, 0)
        op = sparc.DesignOperator(W, L, M, n, o0, o1)
        tr = montecarlo.SparcTrial(op, [1.0], t_max=25, precision="f32", seed=2)
        res[R] = tr(0, 0, 2, 16)
        assert res[R][0] == 32
    assert res[1.0][4] == 0 and res[1.0][1] == 0
    assert res[1.6][2] == 32 and res[1.6][4] > 0
