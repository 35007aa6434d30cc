"""GROUP BY key with count() as the only aggregate (`SELECT k, count(*) ... GROUP BY k`, the shape
a GROUP BY over a join's output takes): staged records are the keys alone (one word), on the
tile-sorted path and on the histogram + scatter path, with and without a fused predicate.
Checked against a bincount of the kept rows (exact).  Reference: Aggregator::executeOnBlock with
AggregateFunctionCount (Interpreters/Aggregator.cpp:1127-1246, AggregateFunctionCount.h:46)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,groups,filtered", [(3_000_000, 100_000, False), (3_000_000, 100_000, True),
                                               (50_000, 3_000, True), (2_000_000, 2_000_000, False)])
def test_count_only_group_by(tfa, ctx, dev, n, groups, filtered):
    g = torch.Generator(device=dev)
    g.manual_seed(n + groups)
    k = torch.randint(-groups // 2, groups - groups // 2, (n,), device=dev, generator=g)
    f = torch.randint(0, 100, (n,), device=dev, generator=g)
    agg = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_COUNT_ALL, 0)], expected_groups=groups)
    if filtered:
        agg.consume_filtered(f, tfa.LT, 60, k, [None])
        kept = k[f < 60]
    else:
        agg.consume(k, [None])
        kept = k
    res = agg.result()
    agg.close()
    exp = torch.bincount(kept - (-groups // 2), minlength=groups)
    keys = res["keys"]
    assert keys.shape[0] == int((exp > 0).sum().item())
    assert torch.equal(res["states"][0].view(torch.int64), exp[keys - (-groups // 2)])
