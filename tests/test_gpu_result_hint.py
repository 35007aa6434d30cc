"""tfg_agg_result with a capacity hint: the groups of a tiled consume are written before their count
is read (no host round trip between consume and result).  A hint at or above the count gives the
exact result of the plain call; a hint below it reports TFG_ERR_CAPACITY and the Python front end
falls back to the exact call; first_row aggregates (value stores) never take the early path.
Reference: Aggregator::convertToBlockImplFinal (Interpreters/Aggregator.cpp:1651-1780)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _by_key(res):
    keys = res["keys"].cpu().numpy()
    s = res["states"][0].cpu().numpy()
    c = res["states"][1].view(torch.int64).cpu().numpy()
    return {int(k): (float(a), int(b)) for k, a, b in zip(keys, s, c)}


@pytest.mark.parametrize("hint_scale", [0.5, 1.0, 3.0])
def test_result_capacity_hint(tfa, ctx, dev, hint_scale):
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    n, groups = 4_000_000, 200_000
    k = torch.randint(0, groups, (n,), device=dev, generator=g)
    f = torch.rand(n, device=dev, generator=g, dtype=torch.float64) * 100
    v = torch.randint(0, 1 << 20, (n,), device=dev, generator=g).double() / 256.0
    aggs = [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)]
    a = tfa.Aggregator(ctx, tfa.INT64, aggs, expected_groups=groups)
    a.consume_filtered(f, tfa.LT, 70, k, [v, None])
    exact = _by_key(a.result())
    a.reset()
    a.consume_filtered(f, tfa.LT, 70, k, [v, None])
    hinted = a.result(capacity_hint=max(1, int(len(exact) * hint_scale)))
    a.close()
    assert hinted["keys"].shape[0] == len(exact)
    assert _by_key(hinted) == exact
    kept = k[f < 70]
    assert sum(c for _, c in exact.values()) == kept.numel()


def test_result_capacity_hint_first_row(tfa, ctx, dev):
    """a first_row aggregate keeps the exact path (its value store sizes the result)"""
    g = torch.Generator(device=dev)
    g.manual_seed(6)
    n, groups = 1_000_000, 50_000
    k = torch.randint(0, groups, (n,), device=dev, generator=g)
    y = (k % 1000).to(torch.int16)
    a = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_FIRST_ROW, tfa.INT16), (tfa.AGG_COUNT_ALL, 0)])
    a.consume(k, [y, None])
    r = a.result(capacity_hint=groups * 2)
    a.close()
    keys = r["keys"].cpu().numpy()
    fr = r["states"][0].cpu().numpy()
    assert keys.shape[0] == np.unique(k.cpu().numpy()).shape[0]
    assert np.array_equal(fr, (keys % 1000).astype(np.int16))
    assert not r["state_null"][0].cpu().numpy().any()


@pytest.mark.parametrize("hint_scale", [0.5, 1.0, 2.0])
def test_keys_result_capacity_hint_string(tfa, ctx, dev, hint_scale):
    """the packed String-key result with a capacity hint (key lengths, scan and unpack over the
    hinted slots, count read on the device) = the exact call; a hint below the count falls back"""
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    n, groups = 2_000_000, 150_000
    ids = torch.randint(0, groups, (n,), device=dev, generator=g)
    width = 1 + (ids % 7)  # keys of 2-8 bytes + '\0'
    lens = (width + 2).to(torch.int64)
    offs = torch.cumsum(lens, 0)
    chars = torch.zeros(int(offs[-1].item()), dtype=torch.uint8, device=dev)
    starts = offs - lens
    x = ids.clone()
    for j in range(8):
        sel = width > j
        chars[(starts + 1 + j)[sel]] = (48 + x % 10)[sel].to(torch.uint8)
        x = x // 10
    chars[starts] = ord("k")
    v = torch.randint(0, 1 << 30, (n,), device=dev, generator=g)
    aggs = [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)]
    a = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, expected_groups=groups)

    def table(res):
        ch, of = res["keys"][0]
        ch, of = ch.cpu().numpy(), of.cpu().numpy()
        s = res["states"][0].view(torch.int64).cpu().numpy()
        c = res["states"][1].view(torch.int64).cpu().numpy()
        out = {}
        for i in range(len(of)):
            out[bytes(ch[(of[i - 1] if i else 0):of[i]])] = (int(s[i]), int(c[i]))
        return out

    a.consume([(chars, offs)], [v, None])
    exact = table(a.result())
    a.reset()
    a.consume([(chars, offs)], [v, None])
    hinted = table(a.result(capacity_hint=max(1, int(len(exact) * hint_scale))))
    a.close()
    assert hinted == exact
    assert sum(c for _, c in exact.values()) == n
