"""GPU parity of the fused filter -> GROUP BY kernel (tiflash_amd/csrc/agg_fused.hip): one
persistent workgroup per CU owns a bucket's LDS table for the whole input while tiles stream
through an Infinity-Cache ring.  Opt-in (Aggregator(..., fused=True) / tfg_agg_params.fused),
it serves empty aggregators of the fast signatures (one 8-byte key without NULLs; sum Int64 /
UInt64 / Float64 + count) with 256 buckets and >= 4M rows; test_gpu_c2_full.py runs it at 100M
rows.  Here: the edge cases — a partial
last round, key 0 (ZeroValueStorage side slot), a hot key, every predicate form (mask, Int32 /
Float64 compares, nullable predicate column), and more distinct keys than the 256 tables hold
(rows spilled to the two-kernel path, so the result is still exact) — each against the oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _gpu_sorted(res):
    k = res["keys"]
    o = torch.argsort(k)
    return k[o].cpu().numpy(), res["states"][0][o].cpu().numpy(), res["states"][1][o].cpu().numpy()


def _ref_sorted(r):
    k = r["keys"].view(np.int64)
    o = np.argsort(k)
    return k[o], r["states"][0][o], r["states"][1][o].view(np.int64)


def _check(tfa, ctx, dev, orc, f, k, v, pred, vtype=None, groups=1_000_000, fnull=None):
    """pred: (op, scalar) compare on f, or "mask" (f is a UInt8 mask)."""
    vt = vtype or (tfa.FLOAT64 if v.dtype == np.float64 else tfa.INT64)
    agg = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_SUM, vt), (tfa.AGG_COUNT_ALL, 0)], expected_groups=groups,
                         fused=True)
    kd, vd = torch.from_numpy(k).to(dev), torch.from_numpy(v).to(dev)
    fd = torch.from_numpy(f).to(dev)
    if pred == "mask":
        agg.consume(kd, [vd, None], mask=fd)
        mask = f
    else:
        op, s = pred
        agg.consume_filtered(fd, op, s, kd, [vd, None],
                             pred_nullmap=torch.from_numpy(fnull).to(dev) if fnull is not None else None)
        mask = {tfa.LT: f < s, tfa.GE: f >= s, tfa.EQ: f == s}[op].astype(np.uint8)
        if fnull is not None:
            mask &= (fnull == 0).astype(np.uint8)
    ref = orc.Agg(orc.INT64, [(0, orc.FLOAT64 if vt == tfa.FLOAT64 else orc.INT64), (2, 0)])
    ref.consume(k, [v, None], mask=mask)
    gk, gs, gc = _gpu_sorted(agg.result())
    rk, rs, rc = _ref_sorted(ref.result())
    agg.close()
    np.testing.assert_array_equal(gk, rk)
    np.testing.assert_array_equal(gc.view(np.int64), rc)
    assert np.array_equal(gs.view(np.uint64), rs.view(np.uint64))


def test_fused_partial_round_key0_hot_key(tfa, ctx, dev, orc):
    rng = np.random.default_rng(31)
    n = (1 << 22) + 12345  # past FUSED_MIN_ROWS, last round partial
    k = rng.integers(-300_000, 300_000, n, dtype=np.int64)
    k[rng.random(n) < 0.05] = 0         # ZeroValueStorage
    k[rng.random(n) < 0.2] = 7777777     # one hot key: a fifth of the rows
    f = rng.integers(0, 100, n, dtype=np.int64)
    v = rng.integers(0, 1 << 20, n).astype(np.float64) / 256.0
    _check(tfa, ctx, dev, orc, f, k, v, (tfa.LT, 96), groups=600_000)


def test_fused_int64_sum_and_predicate_forms(tfa, ctx, dev, orc):
    rng = np.random.default_rng(32)
    n = 5_000_000
    k = rng.integers(0, 900_000, n, dtype=np.int64)
    v = rng.integers(-(1 << 40), 1 << 40, n, dtype=np.int64)
    f32 = rng.integers(-50, 50, n, dtype=np.int32)
    _check(tfa, ctx, dev, orc, f32, k, v, (tfa.GE, 0), groups=900_000)
    fd = rng.integers(0, 4, n).astype(np.float64)
    _check(tfa, ctx, dev, orc, fd, k, v, (tfa.EQ, 2.0), groups=900_000)
    m = (rng.random(n) < 0.7).astype(np.uint8)
    _check(tfa, ctx, dev, orc, m, k, v, "mask", groups=900_000)
    fi = rng.integers(0, 100, n, dtype=np.int64)
    fnull = (rng.random(n) < 0.1).astype(np.uint8)
    _check(tfa, ctx, dev, orc, fi, k, v, (tfa.LT, 50), groups=900_000, fnull=fnull)


def test_fused_overflowing_tables_spill_exactly(tfa, ctx, dev, orc):
    """3M distinct keys into 256 tables of <= 4505 groups each: most rows spill to the
    two-kernel path after the tables fill; the merged result must still be exact."""
    rng = np.random.default_rng(33)
    n = 6_000_000
    k = rng.integers(0, 3_000_000, n, dtype=np.int64)
    f = rng.integers(0, 100, n, dtype=np.int64)
    v = rng.integers(0, 1 << 20, n).astype(np.float64) / 256.0
    _check(tfa, ctx, dev, orc, f, k, v, (tfa.LT, 90), groups=1_000_000)


def test_fused_repeated_steps_are_identical(tfa, ctx, dev):
    """The bench loop: reset -> consume -> result, many times on the same aggregator and inputs
    (ring slots and run tags reused across launches) — every step bit-identical."""
    g = torch.Generator(device=dev)
    g.manual_seed(34)
    n = 20_000_000
    f = torch.randint(0, 100, (n,), device=dev, generator=g)
    k = torch.randint(0, 1_000_000, (n,), device=dev, generator=g)
    v = torch.randint(0, 1 << 20, (n,), device=dev, generator=g).double() / 256.0
    agg = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)], expected_groups=1_000_000,
                         fused=True)
    first = None
    for _ in range(6):
        agg.reset()
        agg.consume_filtered(f, tfa.LT, 96, k, [v, None])
        r = agg.result()
        o = torch.argsort(r["keys"])
        cur = (r["keys"][o], r["states"][0][o], r["states"][1][o])
        if first is None:
            first = cur
            assert int(cur[2].sum().item()) == int((f < 96).sum().item())
        else:
            assert all(torch.equal(a, b) for a, b in zip(first, cur))
    agg.close()
