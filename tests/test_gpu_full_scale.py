"""C3 and C5 (BASELINE.json configs[2] and configs[4]) at full size, compared with the oracle
row for row — the sizes the bench runs, where the kernels take paths small tests never reach.

* C3: hash join 10M build x 100M probe, Int64 keys, ~50% hit (SURVEY §8(d) distributions, seed 7),
  the partitioned v1 join with materialised output (probe key, probe payload, build payload), as
  the bench's join leg calls it.  4096 build partitions, two-pass probe partition.  Checked as a
  multiset of output rows against orc.JoinRef (Join::joinBlock restated, oracle/oracle.c
  orc_join_*; reference JoinPartition.cpp:1465-1644 probeBlockImplTypeCase).
* C5: GROUP BY a String key "k%08d" over 10M ids, sum(Decimal(15,2)) -> Decimal(37,2) + count(*),
  100M rows as the bench (all but ~450 of the 10M ids present): the wide tiled path at its bench
  geometry — 16384 buckets (two-level: 256 coarse tile-sorted buckets, regrouped 64 ways), LDS
  tables at ~30 % load.  Spill passes are not reached at this load; the forced-spill cases (16
  buckets at the C5 shape) are in tests/test_gpu_keys_agg.py.  Checked group by group against
  orc.AggKeys (Aggregator with key_string / StringHashMap restated; reference
  Aggregator.cpp:566-1246).  Decimal sums are exact 128-bit integers: bit-exact.
* C5 with 1- to 11-byte keys (SURVEY §8(d)'s variable-length variant; bench.py's var_len_keys
  sub-leg): the same aggregation over digit keys of every length up to 11 bytes — every tile
  narrow (20-byte rows, partition.h WNARROW) — against the oracle, group by group."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lexsorted(*cols):
    o = np.lexsort(cols[::-1])
    return [c[o] for c in cols]


def test_c3_full_scale_join_matches_oracle(tfa, ctx, dev, orc):
    nb, npr = 10_000_000, 100_000_000
    rng = np.random.default_rng(7)
    bk = rng.permutation(nb).astype(np.int64) * 4 + 1
    bpay = rng.integers(0, 1 << 40, nb, dtype=np.int64)
    hit = rng.random(npr) < 0.5
    pk = np.where(hit, bk[rng.integers(0, nb, npr)], rng.integers(0, 1 << 40, npr) * 4 + 3).astype(np.int64)
    ppay = rng.integers(0, 1 << 40, npr, dtype=np.int64)
    del hit
    j = tfa.Join(ctx, tfa.INT64, expected_build_rows=nb)
    j.build(torch.from_numpy(bk).to(dev), payload=[torch.from_numpy(bpay).to(dev)])
    j.finalize()
    pkd, ppd = torch.from_numpy(pk).to(dev), torch.from_numpy(ppay).to(dev)
    op, ob, _ = j.probe_rows(pkd, [pkd, ppd], 1, capacity=npr)
    got = [op[0].cpu().numpy(), op[1].cpu().numpy(), ob[0].cpu().numpy()]
    del op, ob, pkd, ppd, j
    torch.cuda.empty_cache()
    ref = orc.JoinRef(orc.INT64)
    ref.build(bk)
    pi, bi = ref.probe(pk)
    want = [pk[pi], ppay[pi], bpay[bi]]
    assert len(got[0]) == len(want[0]) and 0.45 * npr < len(want[0]) < 0.55 * npr
    g = _lexsorted(got[1], got[0], got[2])
    w = _lexsorted(want[1], want[0], want[2])
    for a, b in zip(g, w):
        np.testing.assert_array_equal(a, b)


def test_c5_full_scale_string_groupby_matches_oracle(tfa, ctx, dev, orc):
    n, G = 100_000_000, 10_000_000
    rng = np.random.default_rng(11)
    ids = rng.integers(0, G, n)
    v = rng.integers(0, 10**9, n, dtype=np.int64)
    chars = np.empty((n, 10), np.uint8)
    chars[:, 0] = ord("k")
    x = ids.copy()
    for p in range(8, 0, -1):
        chars[:, p] = 48 + x % 10
        x //= 10
    chars[:, 9] = 0
    del x
    chars = chars.reshape(-1)
    offs = np.arange(1, n + 1, dtype=np.uint64) * 10
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, expected_groups=G)
    agg.consume([(torch.from_numpy(chars).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev))],
                [torch.from_numpy(v).to(dev), None])
    res = agg.result()
    gchars, goffs = (t.cpu().numpy() for t in res["keys"][0])
    gsum = res["states"][0].cpu().numpy().view(np.int64).reshape(-1, 2)
    gcnt = res["states"][1].cpu().numpy().view(np.int64)
    agg.close()
    g = len(goffs)
    # GPU keys: "k%08d\0" rows of 10 bytes -> ids
    assert np.array_equal(np.diff(np.concatenate([[0], goffs.view(np.uint64)])), np.full(g, 10, np.uint64))
    gk = gchars.reshape(g, 10)[:, 1:9].astype(np.int64) - 48
    gid = (gk * (10 ** np.arange(7, -1, -1, dtype=np.int64))).sum(axis=1)
    # oracle
    ref = orc.AggKeys([orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)])
    ref.consume([(chars, offs)], [v, None])
    kb, ko, (osum, ocnt), _ = ref.result_arrays()
    og = len(ko)
    assert og == g and g == len(np.unique(ids))
    # serialised key per group: NULL byte, u64 length (9), 9 bytes "k%08d"
    assert np.array_equal(np.diff(np.concatenate([[0], ko.astype(np.int64)])), np.full(og, 18))
    ok = kb.reshape(og, 18)[:, 10:18].astype(np.int64) - 48
    oid = (ok * (10 ** np.arange(7, -1, -1, dtype=np.int64))).sum(axis=1)
    go, oo = np.argsort(gid), np.argsort(oid)
    np.testing.assert_array_equal(gid[go], oid[oo])
    np.testing.assert_array_equal(gcnt[go], ocnt[oo])
    np.testing.assert_array_equal(gsum[go], osum[oo])
    assert int(gcnt.sum()) == n


def var_len_split(g):
    """group id -> (key length L in 1..11, its value q): every 1-byte key (94), every 2-byte key
    (94^2), every 3-byte key (94^3), then lengths 4..11 in turn; distinct ids give distinct keys"""
    c1, c2, c3 = 94, 94 + 94**2, 94 + 94**2 + 94**3
    r = g - c3
    L = np.where(g < c1, 1, np.where(g < c2, 2, np.where(g < c3, 3, 4 + r % 8)))
    q = np.where(g < c1, g, np.where(g < c2, g - c1, np.where(g < c3, g - c2, r // 8)))
    return L, q


def var_len_keys(ids):
    """The C5 variable-length key set (bench.py's string_agg var_len_keys sub-leg, the same map on
    the device): group id -> a key of 1-11 bytes from the 94 printable characters 33..126, its
    value q written in base 94, most significant digit first.  10M ids -> 10M distinct keys."""
    L, q = var_len_split(ids.astype(np.int64))
    offs = np.cumsum(L + 1).astype(np.uint64)
    starts = offs.astype(np.int64) - (L + 1)
    chars = np.zeros(int(offs[-1]), np.uint8)
    qq = q.copy()
    for k in range(11):
        sel = L > k
        chars[(starts + L - 1 - k)[sel]] = 33 + (qq[sel] % 94)
        qq //= 94
    return chars, offs


def _key_codes(chars, ends, lens):
    """rows of keys (<= 11 bytes) -> int64 codes: (L, base-94 value) packed (unique per key)"""
    starts = ends - lens
    val = np.zeros(len(ends), np.int64)
    for j in range(11):
        sel = lens > j
        val[sel] = val[sel] * 94 + (chars[starts[sel] + j].astype(np.int64) - 33)
    return lens.astype(np.int64) << 58 | val


def test_c5_full_scale_var_len_keys_matches_oracle(tfa, ctx, dev, orc):
    """SURVEY §8(d)'s C5 variant: 1- to 11-byte String keys (StringHashMap's size classes,
    Common/HashTable/StringHashTable.h:211-310) at the full 100M rows, vs the oracle's GROUP BY"""
    n, G = 100_000_000, 10_000_000
    rng = np.random.default_rng(17)
    ids = rng.integers(0, G, n)
    v = rng.integers(0, 10**9, n, dtype=np.int64)
    n_ids = len(np.unique(ids))
    chars, offs = var_len_keys(ids)
    del ids
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, expected_groups=G)
    agg.consume([(torch.from_numpy(chars).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev))],
                [torch.from_numpy(v).to(dev), None])
    res = agg.result()
    gchars, goffs = (t.cpu().numpy() for t in res["keys"][0])
    gsum = res["states"][0].cpu().numpy().view(np.int64).reshape(-1, 2)
    gcnt = res["states"][1].cpu().numpy().view(np.int64)
    agg.close()
    gends = goffs.astype(np.int64)
    glen = np.diff(np.concatenate([[0], gends])) - 1  # the '\0' excluded
    gcode = _key_codes(gchars, gends - 1, glen)
    ref = orc.AggKeys([orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)])
    ref.consume([(chars, offs)], [v, None])
    kb, ko, (osum, ocnt), _ = ref.result_arrays()
    # serialised key per group: NULL byte, u64 length, the bytes
    oends = ko.astype(np.int64)
    olen = np.diff(np.concatenate([[0], oends])) - 9
    ocode = _key_codes(kb, oends, olen)
    assert len(gcode) == len(ocode) and len(np.unique(gcode)) == len(gcode)
    assert len(gcode) == n_ids
    go, oo = np.argsort(gcode), np.argsort(ocode)
    np.testing.assert_array_equal(gcode[go], ocode[oo])
    np.testing.assert_array_equal(gcnt[go], ocnt[oo])
    np.testing.assert_array_equal(gsum[go], osum[oo])
    assert int(gcnt.sum()) == n
