"""A tiled consume whose last segment is short (fewer tiles than the others) after a larger
consume on the same context: the unvisited tile slots of that segment must read as empty, not as
the previous consume's runs left in the scratch arena (partition.h, part_scatter_staged_kernel's
tail).  Sizes: 768 segments of 16384 rows (2 tiles) on a 256-CU device; the second batch ends 500
rows into its last segment.  Reference: Aggregator.cpp:852-1024 (every kept row counted once)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_short_last_segment_after_larger_consume(tfa, ctx, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(23)
    n1 = 768 * 16384
    n2 = 767 * 16384 + 500
    agg = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)])
    for n in (n1, n2, n1, n2 + 3000):
        k = torch.randint(0, 200_000, (n,), device=dev, generator=g)
        f = torch.randint(0, 100, (n,), device=dev, generator=g)
        v = torch.randint(0, 1 << 16, (n,), device=dev, generator=g).double() / 4.0
        agg.reset()
        agg.consume_filtered(f, tfa.LT, 90, k, [v, None])
        res = agg.result()
        keep = f < 90
        cnt = res["states"][1].view(torch.int64)
        assert int(cnt.sum().item()) == int(keep.sum().item()), n
        ref_s = torch.zeros(200_000, dtype=torch.float64, device=dev).index_add_(0, k[keep], v[keep])
        ref_c = torch.zeros(200_000, dtype=torch.int64, device=dev).index_add_(0, k[keep], torch.ones_like(k[keep]))
        keys = res["keys"]
        assert torch.equal(ref_c[keys], cnt)
        assert torch.equal(ref_s[keys], res["states"][0])
        assert int((ref_c > 0).sum().item()) == keys.shape[0]
    agg.close()
