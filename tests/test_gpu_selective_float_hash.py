"""GPU parity of two exchange-hash rows: Float keys (a22: ColumnVector<Float>::updateWeakHash32,
Columns/ColumnVector.cpp:520-529, hashes intHashCRC32(UInt64(x)) — the x86-64 conversion pinned
by tests/golden/float_weak_hash.json) and BlockInfo::selective (a25: Core/BlockInfo.h:47-49; weak
hash and scatter over the listed rows only, HashBaseWriterHelper.cpp:110-260).  The selective
checks are the reference's own property test (gtest_mpp_exchange_writer.cpp:1147-1230): the
selective hash equals the full hash at the same rows, and the scatter of the selective rows puts
exactly the selector's count of rows in each partition; both also against the oracle."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("kind", ["float64", "float32"])
def test_float_weak_hash_golden(tfa, ctx, dev, kind):
    g = json.load(open(os.path.join(GOLD, "float_weak_hash.json")))[kind]
    dt, ut = (np.float64, np.uint64) if kind == "float64" else (np.float32, np.uint32)
    vals = np.array([int(e["bits"], 16) for e in g], dtype=ut).view(dt)
    t = tfa.FLOAT64 if kind == "float64" else tfa.FLOAT32
    h = tfa.weak_hash(ctx, [torch.from_numpy(vals).to(dev)], types=[t])
    np.testing.assert_array_equal(_u32(h), np.array([e["hash"] for e in g], dtype=np.uint32))


@pytest.mark.parametrize("kind", ["float64", "float32"])
def test_float_keys_partition_matches_oracle(tfa, ctx, dev, orc, kind):
    rng = np.random.default_rng(61)
    n = 200_003
    dt = np.float64 if kind == "float64" else np.float32
    x = (rng.standard_normal(n) * np.exp(rng.uniform(-30, 50, n))).astype(dt)
    x[rng.random(n) < 0.01] = np.nan
    x[rng.random(n) < 0.01] = np.inf
    x[rng.random(n) < 0.01] = -0.0
    nulls = (rng.random(n) < 0.05).astype(np.uint8)
    t = tfa.FLOAT64 if kind == "float64" else tfa.FLOAT32
    ot = orc.FLOAT64 if kind == "float64" else orc.FLOAT32
    xd = torch.from_numpy(x).to(dev)
    h = tfa.weak_hash(ctx, [xd], types=[t], nullmaps=[torch.from_numpy(nulls).to(dev)])
    exp = orc.weak_hash([x], types=[ot], nullmaps=[nulls])
    np.testing.assert_array_equal(_u32(h), exp)
    # the one-call scatter routes float keys the same way
    sel = orc.fill_selector(exp, 5)
    perm, offs = orc.partition(sel, 5)
    payload = np.arange(n, dtype=np.int64)
    outs, hoffs = tfa.hash_partition(ctx, [xd, torch.from_numpy(payload).to(dev)], [0], 5,
                                     types=[t, tfa.INT64],
                                     nullmaps=[torch.from_numpy(nulls).to(dev), None])
    np.testing.assert_array_equal(np.array(hoffs, dtype=np.uint64), offs)
    np.testing.assert_array_equal(outs[1].cpu().numpy(), payload[perm])


def _selective(rng, n, m):
    return np.sort(rng.choice(n, m, replace=False)).astype(np.int64)


@pytest.mark.parametrize("tcode", [1, 2, 3, 4, 7, 8, 9, 10, 12, 13])  # ints, uints, floats, Decimal64/128
def test_selective_weak_hash_equals_full_hash(tfa, ctx, dev, orc, tcode):
    rng = np.random.default_rng(70 + tcode)
    rows, sel_rows = 4096, 1024
    if tcode == 13:
        col = rng.integers(-2**62, 2**62, (rows, 2), dtype=np.int64)
    elif tcode in (9, 10):
        col = (rng.standard_normal(rows) * 1e12).astype(np.float32 if tcode == 9 else np.float64)
    else:
        dt = {1: np.int8, 2: np.int16, 3: np.int32, 4: np.int64, 7: np.int32, 8: np.int64, 12: np.int64}[tcode]
        col = rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, rows, dtype=dt, endpoint=True)
    nulls = (rng.random(rows) < 0.1).astype(np.uint8)
    sel = _selective(rng, rows, sel_rows)
    cd, nd = torch.from_numpy(col).to(dev), torch.from_numpy(nulls).to(dev)
    full = tfa.weak_hash(ctx, [cd], types=[tcode], nullmaps=[nd])
    part = tfa.weak_hash(ctx, [cd], types=[tcode], nullmaps=[nd], selective=torch.from_numpy(sel).to(dev))
    assert part.shape[0] == sel_rows
    np.testing.assert_array_equal(_u32(part), _u32(full)[sel])
    np.testing.assert_array_equal(_u32(part), orc.weak_hash([col[sel]], types=[tcode], nullmaps=[nulls[sel]]))


@pytest.mark.parametrize("collator", [0, 1, 2])
def test_selective_string_weak_hash(tfa, ctx, dev, orc, collator):
    rng = np.random.default_rng(80 + collator)
    rows = 4096
    strs = [(b"k%d" % rng.integers(0, 700)) + b" " * int(rng.integers(0, 3)) + b"y" * int(rng.integers(0, 25))
            for _ in range(rows)]
    chars = np.frombuffer(b"".join(s + b"\0" for s in strs), dtype=np.uint8).copy()
    offsets = np.cumsum([len(s) + 1 for s in strs]).astype(np.uint64)
    nulls = (rng.random(rows) < 0.1).astype(np.uint8)
    sel = _selective(rng, rows, 1024)
    cd, od = torch.from_numpy(chars).to(dev), torch.from_numpy(offsets.view(np.int64)).to(dev)
    nd = torch.from_numpy(nulls).to(dev)
    full = torch.full((rows,), -1, dtype=torch.int32, device=dev)
    tfa.weak_hash_string(ctx, cd, od, full, nullmap=nd, collator=collator)
    part = torch.full((1024,), -1, dtype=torch.int32, device=dev)
    tfa.weak_hash_string(ctx, cd, od, part, nullmap=nd, collator=collator, selective=torch.from_numpy(sel).to(dev))
    np.testing.assert_array_equal(_u32(part), _u32(full)[sel])
    exp = orc.weak_hash_string(chars, offsets, np.full(rows, 0xFFFFFFFF, dtype=np.uint32), nulls, collator)
    np.testing.assert_array_equal(_u32(part), exp[sel])


def test_selective_scatter(tfa, ctx, dev, orc):
    """scatter of a selective block: partition p receives the selective rows whose selector is p,
    in selective order (IColumn::scatter with a BlockSelective)."""
    rng = np.random.default_rng(90)
    rows, m, parts = 4096, 1024, 4
    k = rng.integers(-2**40, 2**40, rows, dtype=np.int64)
    sel = _selective(rng, rows, m)
    seld = torch.from_numpy(sel).to(dev)
    kd = torch.from_numpy(k).to(dev)
    h = tfa.weak_hash(ctx, [kd], selective=seld)
    selector = tfa.fill_selector(ctx, h, parts)
    perm, offs = tfa.partition(ctx, selector, parts)
    rows_perm = tfa.selective_perm(ctx, seld, perm)
    got = tfa.gather(ctx, rows_perm, [kd])[0].cpu().numpy()
    exp_sel = orc.fill_selector(orc.weak_hash([k[sel]]), parts)
    assert sum(offs[p + 1] - offs[p] for p in range(parts)) == m
    for p in range(parts):
        assert offs[p + 1] - offs[p] == int((exp_sel == p).sum())
        np.testing.assert_array_equal(got[offs[p]:offs[p + 1]], k[sel][exp_sel == p])
    # perm = None maps positions straight to rows
    np.testing.assert_array_equal(tfa.selective_perm(ctx, seld).cpu().numpy(), sel.astype(np.int32))
