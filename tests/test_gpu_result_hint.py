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


def _str_col(dev, words):
    """a ColumnString (chars with '\\0' per row, UInt64 end offsets) of python bytes rows"""
    buf = b"".join(w + b"\0" for w in words)
    chars = torch.tensor(list(buf), dtype=torch.uint8, device=dev)
    offs = torch.tensor(np.cumsum([len(w) + 1 for w in words]), dtype=torch.int64, device=dev)
    return chars, offs


def _rows(res, nstr):
    cols = []
    for j in range(nstr):
        ch, of = res["keys"][j]
        ch, of = ch.cpu().numpy(), of.cpu().numpy()
        assert len(ch) == (of[-1] if len(of) else 0)  # each column ends at its own last offset
        cols.append([bytes(ch[(of[i - 1] if i else 0):of[i] - 1]) for i in range(len(of))])
    c = res["states"][0].view(torch.int64).cpu().numpy()
    return sorted(zip(*cols, c.tolist()))


@pytest.mark.parametrize("hint", [10, 5000])
def test_keys_result_capacity_hint_serialized(tfa, ctx, dev, hint):
    """hinted results of the serialized method: String keys longer than 15 bytes need more than
    16 chars bytes a group, so the hinted call reports TFG_ERR_CAPACITY with cnt <= hint and the
    front end retries with the reported chars; two String key columns come back
    each sliced at its own last offset"""
    rng = np.random.default_rng(11)
    n, groups = 20_000, 400
    ids = rng.integers(0, groups, n)
    long_w = [b"a-rather-long-string-key-%05d" % i for i in ids]   # 29 bytes: the serialized method
    short_w = [b"s%d" % (i % 7) for i in ids]
    a = tfa.KeysAggregator(ctx, [tfa.STRING, tfa.STRING], [(tfa.AGG_COUNT_ALL, 0)], expected_groups=groups)
    c1, o1 = _str_col(dev, long_w)
    c2, o2 = _str_col(dev, short_w)
    a.consume([(c1, o1), (c2, o2)], [None])
    exact = _rows(a.result(), 2)
    got = _rows(a.result(capacity_hint=hint), 2)
    a.close()
    want = {}
    for x, y in zip(long_w, short_w):
        want[(x, y)] = want.get((x, y), 0) + 1
    assert exact == sorted((x, y, c) for (x, y), c in want.items())
    assert got == exact
