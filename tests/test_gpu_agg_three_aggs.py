"""Three aggregates on the general (non-tiled) path with a fused predicate: sum(Float64),
count(*), sum(Int64) GROUP BY Int64 — a signature no FastOps specialisation covers (op code 312),
so the histogram + scatter partition and GenericOps<3> bucket kernels run.  Exact (dyadic floats,
integers) against numpy.  Reference: Aggregator::executeOnBlock (Aggregator.cpp:1127-1246)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [150_000, 3_000_000])
def test_sum_f64_count_sum_i64_filtered(tfa, ctx, dev, n):
    rng = np.random.default_rng(n)
    f = rng.integers(0, 100, n).astype(np.int64)
    k = rng.integers(-5000, 15000, n).astype(np.int64)
    d = rng.integers(0, 1 << 20, n).astype(np.float64) / 256.0
    m = (100 - f).astype(np.int64)
    aggs = [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0), (tfa.AGG_SUM, tfa.INT64)]
    agg = tfa.Aggregator(ctx, tfa.INT64, aggs)
    t = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    agg.consume_filtered(t(f), tfa.LT, 40, t(k), [t(d), None, t(m)])
    res = agg.result()
    agg.close()
    keep = f < 40
    kk = k[keep] + 5000
    exp_d = np.bincount(kk, weights=d[keep], minlength=20000)
    exp_c = np.bincount(kk, minlength=20000)
    exp_m = np.bincount(kk, weights=m[keep], minlength=20000).astype(np.int64)
    keys = res["keys"].cpu().numpy() + 5000
    assert len(keys) == int((exp_c > 0).sum())
    np.testing.assert_array_equal(res["states"][1].cpu().numpy().view(np.int64), exp_c[keys])
    np.testing.assert_array_equal(res["states"][0].cpu().numpy(), exp_d[keys])
    np.testing.assert_array_equal(res["states"][2].cpu().numpy(), exp_m[keys])


@pytest.mark.parametrize("order", ["count_sum", "sum_count_sum_u"])
def test_aggregate_orders_without_specialisation(tfa, ctx, dev, order):
    """count(*) before sum(Float64) (op code 130) and sum, count, sum(UInt64)-like orders: the
    signatures stage columnar rows for the generic kernels, whatever the FastOps list holds."""
    n = 2_000_000
    rng = np.random.default_rng(7 if order == "count_sum" else 8)
    k = rng.integers(0, 50_000, n).astype(np.int64)
    d = rng.integers(0, 1 << 20, n).astype(np.float64) / 256.0
    t = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    if order == "count_sum":
        aggs, args = [(tfa.AGG_COUNT_ALL, 0), (tfa.AGG_SUM, tfa.FLOAT64)], [None, t(d)]
    else:
        aggs, args = [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0), (tfa.AGG_SUM, tfa.FLOAT64)], [t(d), None, t(d)]
    agg = tfa.Aggregator(ctx, tfa.INT64, aggs)
    agg.consume(t(k), args)
    res = agg.result()
    agg.close()
    keys = res["keys"].cpu().numpy()
    exp_c = np.bincount(k, minlength=50_000)
    exp_d = np.bincount(k, weights=d, minlength=50_000)
    assert len(keys) == int((exp_c > 0).sum())
    ci = 0 if order == "count_sum" else 1
    np.testing.assert_array_equal(res["states"][ci].cpu().numpy().view(np.int64), exp_c[keys])
    np.testing.assert_array_equal(res["states"][1 - ci if order == "count_sum" else 0].cpu().numpy(), exp_d[keys])
