"""Decimal256 sums raise TFG_ERR_OVERFLOW when the exact sum leaves Int256, as the reference's
boost checked_int256_t throws (libs/libcommon/include/common/types.h:35; DECIMAL_OVERFLOW).

Sums are kept with a fifth limb in the LDS tables and no-key partials (lds_add_i256 /
add_i320), so the check is on the exact sum, whatever the order of the adds.  Decimal(65) values
stay below 2^216, so a real overflow needs ~2^39 maximal rows; the tests feed Int256 values near
2^254 directly (the ABI carries raw limbs) to reach the bound with a few rows."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


def _limbs(values):
    out = np.zeros((len(values), 4), dtype=np.uint64)
    for i, v in enumerate(values):
        v &= (1 << 256) - 1
        for k in range(4):
            out[i, k] = (v >> (64 * k)) & M64
    return out.view(np.int64)


def _ints(a):
    from oracle.oracle import limbs_to_int
    return [limbs_to_int(r) for r in a.cpu().numpy()]


def _agg(tfa, ctx, key_type):
    return tfa.Aggregator(ctx, key_type, [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL256, 65)), (tfa.AGG_COUNT_ALL, 0)])


@pytest.mark.parametrize("keyed", [True, False])
def test_decimal256_sum_overflow_raises(tfa, ctx, dev, keyed):
    big = 1 << 254
    cases = [
        ([big, big], True),                      # 2^255: one past Int256
        ([-big, -big, -1], True),                # -2^255 - 1
        ([big, big - 1], False),                 # 2^255 - 1: the largest Int256
        ([-big, -big], False),                   # -2^255: the smallest Int256
        ([big, big, -big], False),               # leaves and re-enters the range: the exact sum fits
    ]
    for vals, overflow in cases:
        g = _agg(tfa, ctx, tfa.INT64 if keyed else 0)
        k = torch.full((len(vals),), 7, dtype=torch.int64, device=dev)
        v = torch.from_numpy(_limbs(vals)).to(dev)
        if overflow:
            with pytest.raises(tfa.TfgError) as e:
                g.consume(k if keyed else None, [v, None], n=len(vals))
            assert e.value.code == -11, vals
        else:
            g.consume(k if keyed else None, [v, None], n=len(vals))
            r = g.result()
            assert _ints(r["states"][0]) == [sum(vals)], vals
        g.close()


def test_decimal256_merge_overflow_raises(tfa, ctx, dev):
    """mergeDataImpl of two aggregators whose group sums are 2^254 each -> 2^255: overflow."""
    big = 1 << 254
    parts = []
    for _ in range(2):
        g = _agg(tfa, ctx, tfa.INT64)
        g.consume(torch.tensor([3], dtype=torch.int64, device=dev), [torch.from_numpy(_limbs([big])).to(dev), None], n=1)
        parts.append(g)
    with pytest.raises(tfa.TfgError) as e:
        parts[0].merge(parts[1])
    assert e.value.code == -11
    for g in parts:
        g.close()


def test_decimal256_sums_many_groups_no_false_overflow(tfa, ctx, dev):
    """Realistic Decimal(65) values (< 10^65) over many groups: exact, never flagged."""
    rng = np.random.default_rng(9)
    n, groups = 200_000, 30_000
    k = rng.integers(0, groups, n).astype(np.int64)
    vals = [int(x) * 10**40 * (-1 if s else 1) for x, s in zip(rng.integers(0, 10**18, n), rng.integers(0, 2, n))]
    g = _agg(tfa, ctx, tfa.INT64)
    g.consume(torch.from_numpy(k).to(dev), [torch.from_numpy(_limbs(vals)).to(dev), None])
    r = g.result()
    want = {}
    for key, v in zip(k.tolist(), vals):
        want[key] = want.get(key, 0) + v
    got = dict(zip(r["keys"].cpu().tolist(), _ints(r["states"][0])))
    assert got == want
    g.close()
