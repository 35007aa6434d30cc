"""C2 (BASELINE.json configs[1]) at full size through the exact bench signature: fused
`f < 96` filter + GROUP BY Int64 key: sum(Float64) + count(*), 100M rows, 1M groups — the
tile-sorted partition + pipelined bucket kernel whose chunk walk (1024 tiles per chunk) only
iterates past ~8M rows.  Compared row for row with the oracle (Aggregator restatement,
oracle/oracle.c orc_agg_*).  Values are dyadic (m * 2^-8, m < 2^20), so every summation order
is exact and the comparison is bit-exact.  The rows arrive as two blocks (60M + 40M), so the
second consume also seeds every bucket with the first block's groups (executeOnBlock on a
non-empty AggregatedDataVariants)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, G = 100_000_000, 1_000_000


def _sorted_gpu(res):
    keys = res["keys"]
    order = torch.argsort(keys)
    return (keys[order].cpu().numpy(), res["states"][0][order].cpu().numpy(),
            res["states"][1][order].cpu().numpy().view(np.uint64))


def test_c2_full_scale_matches_oracle(tfa, ctx, dev, orc):
    rng = np.random.default_rng(1)
    f = rng.integers(0, 100, N, dtype=np.int64)
    k = rng.integers(0, G, N, dtype=np.int64)
    v = rng.integers(0, 1 << 20, N).astype(np.float64) / 256.0
    aggs = [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.Aggregator(ctx, tfa.INT64, aggs, expected_groups=G)
    cut = 60_000_000
    for lo, hi in ((0, cut), (cut, N)):
        fd, kd, vd = (torch.from_numpy(x[lo:hi]).to(dev) for x in (f, k, v))
        agg.consume_filtered(fd, tfa.LT, 96, kd, [vd, None])
        del fd, kd, vd
    gk, gs, gc = _sorted_gpu(agg.result())
    agg.close()
    ref = orc.Agg(orc.INT64, [(0, orc.FLOAT64), (2, 0)])
    ref.consume(k, [v, None], mask=(f < 96).astype(np.uint8))
    r = ref.result()
    o = np.argsort(r["keys"].view(np.int64))
    assert len(gk) == len(o) == G
    np.testing.assert_array_equal(gk, r["keys"].view(np.int64)[o])
    np.testing.assert_array_equal(gc, r["states"][1][o])
    assert np.array_equal(gs.view(np.uint64), r["states"][0][o].view(np.uint64)), "sums differ (bit-exact expected)"
    assert int(gc.sum()) == int((f < 96).sum())


def test_c2_full_scale_int64_values_exact(tfa, ctx, dev):
    """The §8(d) Int64-value variant at full size: per-group sums checked against an index_add
    of the kept rows (exact integer arithmetic)."""
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    f = torch.randint(0, 100, (N,), device=dev, generator=g)
    k = torch.randint(0, G, (N,), device=dev, generator=g)
    v = torch.randint(-(1 << 40), 1 << 40, (N,), device=dev, generator=g)
    agg = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)], expected_groups=G)
    agg.consume_filtered(f, tfa.LT, 96, k, [v, None])
    res = agg.result()
    m = f < 96
    exp_sum = torch.zeros(G, dtype=torch.int64, device=dev).index_add_(0, k[m], v[m])
    exp_cnt = torch.bincount(k[m], minlength=G)
    keys = res["keys"]
    assert keys.shape[0] == int((exp_cnt > 0).sum().item())
    assert torch.equal(res["states"][0], exp_sum[keys]) and torch.equal(res["states"][1], exp_cnt[keys])
    agg.close()
