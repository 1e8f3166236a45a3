"""GPU tests of the Monte-Carlo campaign layer: the RCCL communicator (one
rank), sharding invariance with real GPU decodes, and a statistical pin of
the batched BP decoder against the reference's own 2018 campaign
(ldpc_jossy/data/results.txt, sumprod2, 200 iterations)."""
import numpy as np
import pytest

from ldpc_sparc_amd import _native
from ldpc_sparc_amd import montecarlo as mc
from ldpc_sparc_amd.ldpc import code

pytestmark = pytest.mark.gpu


def test_rccl_single_rank_allreduce():
    uid = _native.Comm.unique_id()
    comm = _native.Comm(1, 0, uid)
    agg = mc.Aggregator("rccl", comm)
    v = np.array([1, 2, 3, 4, 5], dtype=np.int64)
    assert agg.allreduce(v).tolist() == [1, 2, 3, 4, 5]
    comm.destroy()


def test_sharding_invariance_with_gpu_decodes():
    c = code("802.11n", "1/2", 27)
    trial = mc.LdpcTrial(c, [1.0], dectype="minsum", max_it=50, precision="f32", seed=3)
    whole = trial(0, 0, 6, 64)
    parts = sum(trial(0, a, b - a, 64) for a, b in (mc.shard_range(6, r, 3) for r in range(3)))
    assert whole.tolist() == parts.tolist()


def test_bp_statistics_match_reference_campaign():
    """802.11n r1/2 z=81 at Es/N0 1.1672803368313591 dB: the reference measured
    1653 blocks / 100 block errors / 16568 bit errors / 59425 iterations
    (results.txt row).  Our f32 sumprod2 FER and mean iteration count must
    agree within 3 combined binomial standard deviations."""
    c = code("802.11n", "1/2", 81)
    snr = 1.1672803368313591
    trial = mc.LdpcTrial(c, [snr], dectype="sumprod2", max_it=200, precision="f32", seed=11)
    tot = mc.run_point(trial, 0, block=1024, blocks_per_round=16, rank=0, world=1, agg=mc.Aggregator(),
                       max_units=16384)
    n, fe, be = int(tot[0]), int(tot[2]), int(tot[1])
    p_ref, n_ref = 100 / 1653, 1653
    p = fe / n
    sd = np.sqrt(p_ref * (1 - p_ref) / n_ref + p_ref * (1 - p_ref) / n)
    assert abs(p - p_ref) < 3 * sd, (p, p_ref)
    assert abs(tot[3] / n - 59425 / 1653) < 3.0  # mean reported iteration index
    ber_ref = 16568 / (1653 * c.N)
    assert abs(be / (n * c.N) - ber_ref) < 0.35 * ber_ref


@pytest.mark.parametrize("rng", ["device", "host"])
def test_concat_sweep_rank_invariant(rng):
    """C5 sweep on a small concatenated code (L=80, M=512 -> 1 x LDPC z=27 in 72
    protected sections): the per-point counters do not depend on how the
    blocks were dealt (two simulated ranks vs one), and BER falls with Eb/N0
    -- with the batches generated on the GPU (Philox, device LDPC encoder) or
    on the host (numpy)."""
    from ldpc_sparc_amd import montecarlo
    kw = dict(codewords=96, block=32, design_seed=3, seed=4, t_max=10, bp_its=50, ldpc=("802.11n", "1/2", 27),
              rng=rng)
    one = montecarlo.concat_ber_sweep(80, 512, 600, 15.0, 8, 1, [1.0, 6.0], **kw)
    # the same blocks in two shards, summed by hand
    from ldpc_sparc_amd.pipeline import ConcatPipeline
    pipe = ConcatPipeline(80, 512, 600, 15.0, 8, 1, ldpc=("802.11n", "1/2", 27), design_seed=3, t_max=10, bp_its=50)
    ub = 8 * 9 + pipe.c.K
    for p, e in enumerate([1.0, 6.0]):
        var = 15.0 / (2 * (ub / 600) * 10 ** (e / 10))
        tr = montecarlo.ConcatTrial(pipe, [var] * 2, seed=4, rng=rng)
        a = tr(p, 0, 1, 32) + tr(p, 1, 2, 32)
        assert int(a[0]) == one[p]["codewords"] == 96
        assert abs(float(a[1]) / (96 * ub) - one[p]["ber"]) < 1e-12
    assert one[1]["ber"] <= one[0]["ber"]
