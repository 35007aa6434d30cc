"""GPU parity: GROUP BY a String key (key_string) and several fixed keys (keys128 /
nullable_keys128), Aggregator.cpp:394-537 + ColumnsHashing.h:179-480, against the oracle's
serialized-key restatement (oracle/oracle.c orc_aggk_*).  Results compare unordered, as the
reference's ExecutorTest does (dbms/src/TestUtils/ExecutorTestUtils.cpp:243-253).

C5 shape (BASELINE.json configs[4]) at test size: String keys "k%08d", Decimal(15,2) values as
Int64 summed into Decimal128, count(*), two-phase partial -> packed-key exchange -> final.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

_SIGNED = {1, 2, 3, 4, 11, 12, 13}


def str_col(strs):
    chars = np.frombuffer(b"".join(s + b"\0" for s in strs), dtype=np.uint8).copy()
    offsets = np.cumsum([len(s) + 1 for s in strs]).astype(np.uint64)
    return chars, offsets


def to_dev(x, dev):
    if isinstance(x, tuple):
        return (torch.from_numpy(x[0]).to(dev), torch.from_numpy(x[1].view(np.int64)).to(dev))
    if x is None:
        return None
    a = x.view(np.int64) if x.dtype == np.uint64 else (x.view(np.int32) if x.dtype == np.uint32 else x)
    a = a.view(np.int16) if a.dtype == np.uint16 else a
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def gpu_groups(res, key_types):
    """tfg result -> [(key tuple, [states])] like oracle.AggKeys.result()."""
    g = res["states"][0].shape[0] if res["states"] else 0
    cols = []
    for t, k, kn in zip(key_types, res["keys"], res["key_null"]):
        nulls = kn.cpu().numpy()
        if t == 20:
            chars = k[0].cpu().numpy().tobytes()
            offs = k[1].cpu().numpy()
            vals, s = [], 0
            for i in range(g):
                e = int(offs[i])
                vals.append(None if nulls[i] else chars[s:e - 1])
                s = e
        elif t in (9, 10):
            a = k.cpu().numpy().view(np.float32 if t == 9 else np.float64)
            vals = [None if nulls[i] else float(a[i]) for i in range(g)]
        elif t in (13, 14):  # Decimal128 / Decimal256 keys: (G, limbs) int64
            from oracle.oracle import limbs_to_int
            a = k.cpu().numpy()
            vals = [None if nulls[i] else limbs_to_int(a[i]) for i in range(g)]
        else:
            a = k.cpu().numpy()
            w = a.dtype.itemsize
            raw = a.view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[w]).astype(object)
            vals = []
            for i in range(g):
                v = int(raw[i])
                if t in _SIGNED and v >= 1 << (8 * w - 1):
                    v -= 1 << (8 * w)
                vals.append(None if nulls[i] else v)
        cols.append(vals)
    sts = []
    for s in res["states"]:
        a = s.cpu().numpy()
        if a.ndim == 2:  # Decimal128 / Decimal256 limbs
            from oracle.oracle import limbs_to_int
            sts.append([limbs_to_int(x) for x in a])
        else:
            sts.append(a.tolist())
    return [(tuple(c[i] for c in cols), [st[i] for st in sts]) for i in range(g)]


def check_same(got, exp):
    assert len(got) == len(exp), (len(got), len(exp))
    g = sorted(got, key=repr)
    e = sorted(exp, key=repr)
    for a, b in zip(g, e):
        assert a == b, (a, b)


def rand_strings(rng, n, vocab):
    return [vocab[i] for i in rng.integers(0, len(vocab), n)]


def vocab_strings(rng, m, maxlen=15, pad=True):
    out = set()
    while len(out) < m:
        ln = int(rng.integers(0, maxlen + 1))
        s = bytes(rng.integers(33, 127, ln, dtype=np.uint8))
        out.add(s)
    v = sorted(out)
    if pad:  # trailing spaces: BIN_PADDING folds them, raw collation keeps them apart
        v += [s + b"  " for s in v[:m // 10] if len(s) <= 13]
    return v


@pytest.mark.parametrize("collator", [0, 2])
@pytest.mark.parametrize("nullable", [False, True])
def test_string_key_sum_count(tfa, ctx, dev, orc, collator, nullable):
    rng = np.random.default_rng(10 + collator + 2 * nullable)
    vocab = vocab_strings(rng, 3000)
    n = 60_000
    strs = rand_strings(rng, n, vocab)
    chars, offs = str_col(strs)
    knull = (rng.random(n) < 0.05).astype(np.uint8) if nullable else None
    d = rng.integers(-10**9, 10**9, n, dtype=np.int64)  # Decimal(15,2) payload
    iv = rng.integers(-2**40, 2**40, n, dtype=np.int64)
    ivn = (rng.random(n) < 0.1).astype(np.uint8)
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0), (tfa.AGG_SUM, tfa.INT64 | tfa.NULLABLE)]
    agg = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, collators=[collator])
    half = n // 2
    for lo, hi in ((0, half), (half, n)):  # two blocks: the second seeds the first's groups
        c2, o2 = str_col(strs[lo:hi])
        agg.consume([to_dev((c2, o2), dev)], [to_dev(d[lo:hi], dev), None, to_dev(iv[lo:hi], dev)],
                    key_nullmaps=[to_dev(knull[lo:hi], dev)] if nullable else None,
                    arg_nullmaps=[None, None, to_dev(ivn[lo:hi], dev)])
    got = gpu_groups(agg.result(), [20])
    ref = orc.AggKeys([orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0), (0, orc.INT64)], collators=[collator])
    ref.consume([(chars, offs)], [d, None, iv], key_nulls=[knull] if nullable else None, arg_nulls=[None, None, ivn])
    check_same(got, ref.result())


def test_string_key_c5_shape_spills(tfa, ctx, dev, orc):
    """k%08d keys, many groups per bucket (forced spill passes), Decimal sum + count."""
    rng = np.random.default_rng(11)
    n, groups = 300_000, 120_000
    ids = rng.integers(0, groups, n)
    strs = [b"k%08d" % i for i in ids]
    chars, offs = str_col(strs)
    d = rng.integers(0, 10**9, n, dtype=np.int64)
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, bucket_bits=4, expected_groups=4096)
    agg.consume([to_dev((chars, offs), dev)], [to_dev(d, dev), None])
    got = gpu_groups(agg.result(), [20])
    ref = orc.AggKeys([orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)])
    ref.consume([(chars, offs)], [d, None])
    check_same(got, ref.result())


@pytest.mark.parametrize("collator,nullable,groups", [(0, False, 2_000_000), (2, True, 600_000)])
def test_string_key_two_level_tiled(tfa, ctx, dev, orc, collator, nullable, groups):
    """The wide tiled path at > 256 buckets: String keys packed while the tiled partition reads
    them, a two-level tile sort (coarse buckets, then 64 fine buckets per coarse bucket), the
    wide bucket kernel; two blocks, so the second one merges into the first one's groups.
    Keys of 0-15 bytes with trailing spaces (BIN_PADDING folds them) and NULLs."""
    rng = np.random.default_rng(12 + collator)
    n = 4_000_000
    ids = rng.integers(0, groups, n)
    pad = rng.integers(0, 3, n) if collator == 2 else np.zeros(n, dtype=np.int64)
    strs = [(b"k%d" % i)[: 1 + (i % 15)] + b" " * int(p) for i, p in zip(ids, pad)]
    knull = (rng.random(n) < 0.02).astype(np.uint8) if nullable else None
    d = rng.integers(-10**12, 10**12, n, dtype=np.int64)
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, collators=[collator], expected_groups=groups)
    cut = n // 3
    for lo, hi in ((0, cut), (cut, n)):
        c2, o2 = str_col(strs[lo:hi])
        agg.consume([to_dev((c2, o2), dev)], [to_dev(d[lo:hi], dev), None],
                    key_nullmaps=[to_dev(knull[lo:hi], dev)] if nullable else None)
    got = gpu_groups(agg.result(), [20])
    chars, offs = str_col(strs)
    ref = orc.AggKeys([orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)], collators=[collator])
    ref.consume([(chars, offs)], [d, None], key_nulls=[knull] if nullable else None)
    check_same(got, ref.result())


@pytest.mark.parametrize("nullable", [False, True])
def test_wide_narrow_tiles_mixed(tfa, ctx, dev, orc, nullable):
    """Narrow wide-key tiles (WNARROW, partition.h: keys with bytes 11-14 zero travel as 20-byte
    rows — u64 lo, u32 hi of bytes 8-10 + the length / NULL byte, u64 value) next to 24-byte tiles:
    the first part of the input has keys of <= 11 bytes (every tile narrow), the rest mixes in keys
    of 12-15 bytes, so the regroup pass reads narrow and wide pass-1 tiles and writes both kinds;
    11 / 12-byte boundary keys, NULL keys (the NULL bit in byte 15) and two blocks (the second seeds
    the first one's groups)."""
    rng = np.random.default_rng(31 + nullable)
    n, groups = 3_000_000, 900_000
    ids = rng.integers(0, groups, n)
    long_from = n // 2
    strs = []
    for r, i in enumerate(ids):
        base = b"w%010d" % i  # 11 bytes: the widest narrow key
        if r < long_from:
            strs.append(base[: 1 + (i % 11)])
        else:
            strs.append(base + b"xyzw"[: i % 5])  # 11-15 bytes
    knull = (rng.random(n) < 0.01).astype(np.uint8) if nullable else None
    d = rng.integers(-10**12, 10**12, n, dtype=np.int64)
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, expected_groups=groups * 2)
    cut = n // 4
    for lo, hi in ((0, cut), (cut, n)):
        c2, o2 = str_col(strs[lo:hi])
        agg.consume([to_dev((c2, o2), dev)], [to_dev(d[lo:hi], dev), None],
                    key_nullmaps=[to_dev(knull[lo:hi], dev)] if nullable else None)
    got = gpu_groups(agg.result(), [20])
    chars, offs = str_col(strs)
    ref = orc.AggKeys([orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)])
    ref.consume([(chars, offs)], [d, None], key_nulls=[knull] if nullable else None)
    check_same(got, ref.result())


def test_fixed_keys_narrow_tiles(tfa, ctx, dev, orc):
    """keys128 of (Int32, Int32) — 8 key bytes, always narrow — and (Int64, UInt32) whose byte 11
    is set for some rows only: narrow and 24-byte tiles side by side, one level and two levels."""
    rng = np.random.default_rng(33)
    for n, groups in ((400_000, 50_000), (3_000_000, 1_200_000)):
        gid = rng.integers(0, groups, n)
        a = (gid % 5000).astype(np.int32)
        b = (gid // 5000).astype(np.int32) - 77
        v = rng.integers(-10**9, 10**9, n, dtype=np.int64)
        aggs = [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)]
        agg = tfa.KeysAggregator(ctx, [tfa.INT32, tfa.INT32], aggs, expected_groups=groups)
        agg.consume([to_dev(a, dev), to_dev(b, dev)], [to_dev(v, dev), None])
        ref = orc.AggKeys([orc.INT32, orc.INT32], [(0, orc.INT64), (2, 0)])
        ref.consume([a, b], [v, None])
        check_same(gpu_groups(agg.result(), [tfa.INT32, tfa.INT32]), ref.result())
        c = gid.astype(np.int64) * 3
        e = np.where(gid % 3 == 0, (gid % 1000) << 24, gid % 1000).astype(np.uint32)  # byte 11 of the key: e's top byte
        agg2 = tfa.KeysAggregator(ctx, [tfa.INT64, tfa.UINT32], aggs, expected_groups=groups)
        agg2.consume([to_dev(c, dev), to_dev(e, dev)], [to_dev(v, dev), None])
        ref2 = orc.AggKeys([orc.INT64, orc.UINT32], [(0, orc.INT64), (2, 0)])
        ref2.consume([c, e], [v, None])
        check_same(gpu_groups(agg2.result(), [tfa.INT64, tfa.UINT32]), ref2.result())


def test_fixed_keys_two_level_tiled(tfa, ctx, dev, orc):
    """keys128 (Int32, Int64) at 1.5M groups through the packed-key wide tiled path, Float64 sum."""
    rng = np.random.default_rng(13)
    n, groups = 3_000_000, 1_500_000
    gid = rng.integers(0, groups, n)
    k1 = (gid % 1000).astype(np.int32)
    k2 = (gid // 1000).astype(np.int64) * 7919
    v = rng.integers(0, 1 << 20, n).astype(np.float64) / 256.0
    aggs = [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.KeysAggregator(ctx, [tfa.INT32, tfa.INT64], aggs, expected_groups=groups)
    agg.consume([to_dev(k1, dev), to_dev(k2, dev)], [to_dev(v, dev), None])
    ref = orc.AggKeys([orc.INT32, orc.INT64], [(0, orc.FLOAT64), (2, 0)])
    ref.consume([k1, k2], [v, None])
    check_same(gpu_groups(agg.result(), [tfa.INT32, tfa.INT64]), ref.result())


def test_string_key_lengths_and_empty(tfa, ctx, dev, orc):
    strs = [b"", b"a", b"ab", b"a\x00b"[:1], b"abcdefgh", b"abcdefghi", b"x" * 15, b" ", b"", b"abcdefgh"] * 300
    chars, offs = str_col(strs)
    agg = tfa.KeysAggregator(ctx, [tfa.STRING], [(tfa.AGG_COUNT_ALL, 0)])
    agg.consume([to_dev((chars, offs), dev)], [None])
    ref = orc.AggKeys([orc.STRING], [(2, 0)])
    ref.consume([(chars, offs)], [None])
    check_same(gpu_groups(agg.result(), [20]), ref.result())
    # an empty block is a no-op
    e = tfa.KeysAggregator(ctx, [tfa.STRING], [(tfa.AGG_COUNT_ALL, 0)])
    ec, eo = torch.empty(0, dtype=torch.uint8, device=dev), torch.empty(0, dtype=torch.int64, device=dev)
    e.consume([(ec, eo)], [None])
    assert e.size() == 0


@pytest.mark.parametrize("collator", [0, 2])
def test_string_key_past_15_bytes_moves_to_serialized(tfa, ctx, dev, orc, collator):
    """key_string over keys of any length: the first block's keys fit the packed form; the second
    block holds keys of 16-300 bytes, so the aggregator moves to the serialized method carrying the
    first block's groups (keys of both blocks overlap), then a third block is consumed there."""
    rng = np.random.default_rng(20 + collator)
    short = vocab_strings(rng, 500)
    long_ = [b"L%05d" % i + bytes(rng.integers(33, 127, int(rng.integers(10, 300)), dtype=np.uint8)) for i in range(700)]
    long_ += [s + b"   " for s in long_[:50]]  # BIN_PADDING folds these onto their unpadded keys
    blocks = [rand_strings(rng, 20_000, short),
              rand_strings(rng, 30_000, short + long_),
              rand_strings(rng, 10_000, long_)]
    aggs = [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, collators=[collator])
    ref = orc.AggKeys([orc.STRING], [(0, orc.INT64), (2, 0)], collators=[collator])
    for strs in blocks:
        chars, offs = str_col(strs)
        v = rng.integers(-1000, 1000, len(strs), dtype=np.int64)
        agg.consume([to_dev((chars, offs), dev)], [to_dev(v, dev), None])
        ref.consume([(chars, offs)], [v, None])
    check_same(gpu_groups(agg.result(), [20]), ref.result())


@pytest.mark.parametrize("types", [(3, 5), (4, 4), (2, 7, 1), (1, 2, 3, 8)])
@pytest.mark.parametrize("nullable", [False, True])
def test_multi_fixed_keys(tfa, ctx, dev, orc, types, nullable):
    widths = {1: 1, 2: 2, 3: 4, 4: 8, 5: 1, 7: 4, 8: 8}
    # nullable tuples of 16 bytes have no spare byte in the packed key: the serialized method
    np_t = {1: np.int8, 2: np.int16, 3: np.int32, 4: np.int64, 5: np.uint8, 7: np.uint32, 8: np.uint64}
    rng = np.random.default_rng(sum(types) + nullable)
    n = 50_000
    keys, nulls = [], []
    for t in types:
        info = np.iinfo(np_t[t])
        card = 40 if widths[t] > 1 else 7
        base = rng.integers(info.min, info.max, card, dtype=np_t[t], endpoint=True)
        base[0] = 0
        keys.append(base[rng.integers(0, card, n)])
        nulls.append((rng.random(n) < 0.08).astype(np.uint8) if nullable else None)
    v = rng.integers(-1000, 1000, n, dtype=np.int64)
    agg = tfa.KeysAggregator(ctx, list(types), [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)])
    agg.consume([to_dev(k, dev) for k in keys], [to_dev(v, dev), None],
                key_nullmaps=[to_dev(x, dev) for x in nulls] if nullable else None)
    ref = orc.AggKeys(list(types), [(0, orc.INT64), (2, 0)])
    ref.consume(keys, [v, None], key_nulls=nulls if nullable else None)
    check_same(gpu_groups(agg.result(), list(types)), ref.result())


def test_two_phase_string_packed_and_unpacked(tfa, ctx, dev, orc):
    """partial aggregations -> (packed keys | key columns) -> final merge, vs one aggregation."""
    rng = np.random.default_rng(12)
    vocab = [b"k%08d" % i for i in range(20_000)]
    n = 100_000
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0)]
    fin_p = tfa.KeysAggregator(ctx, [tfa.STRING], aggs)
    fin_u = tfa.KeysAggregator(ctx, [tfa.STRING], aggs)
    ref = orc.AggKeys([orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)])
    for part in range(3):
        strs = rand_strings(rng, n, vocab)
        chars, offs = str_col(strs)
        d = rng.integers(0, 10**9, n, dtype=np.int64)
        ref.consume([(chars, offs)], [d, None])
        p = tfa.KeysAggregator(ctx, [tfa.STRING], aggs)
        p.consume([to_dev((chars, offs), dev)], [to_dev(d, dev), None])
        rp = p.result_packed()
        fin_p.consume_partial_packed(rp["keys"], rp["states"])
        ru = p.result()
        fin_u.consume_partial(ru["keys"], ru["states"])
    exp = ref.result()
    check_same(gpu_groups(fin_p.result(), [20]), exp)
    check_same(gpu_groups(fin_u.result(), [20]), exp)


def test_merge_multi_key(tfa, ctx, dev, orc):
    rng = np.random.default_rng(13)
    n = 40_000
    aggs = [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)]
    a = tfa.KeysAggregator(ctx, [tfa.INT32, tfa.INT64], aggs)
    b = tfa.KeysAggregator(ctx, [tfa.INT32, tfa.INT64], aggs)
    ref = orc.AggKeys([orc.INT32, orc.INT64], [(0, orc.FLOAT64), (2, 0)])
    for x in (a, b):
        k1 = rng.integers(-50, 50, n, dtype=np.int32)
        k2 = rng.integers(0, 300, n, dtype=np.int64)
        v = rng.integers(0, 1 << 20, n).astype(np.float64) / 256.0
        x.consume([to_dev(k1, dev), to_dev(k2, dev)], [to_dev(v, dev), None])
        ref.consume([k1, k2], [v, None])
    a.merge(b)
    check_same(gpu_groups(a.result(), [3, 4]), ref.result())


def test_groupby_keys_reference_cases(tfa, ctx, dev):
    """GroupBy string_ and two-column GROUP BYs (gtest_aggregation_executor.cpp:408-482): the
    String + fixed combinations take the serialized method, nullable 16-byte tuples move to it."""
    import json
    import os
    from test_oracle_cpu import golden_key_columns
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_cases.json")))["groupby_keys"]
    ran = 0
    for case in g["cases"]:
        types, keys, nulls, exp = golden_key_columns(case, g["columns"])
        agg = tfa.KeysAggregator(ctx, types, [(tfa.AGG_COUNT_ALL, 0)])
        agg.consume([to_dev(k, dev) for k in keys], [None], key_nullmaps=[to_dev(x, dev) for x in nulls])
        got = [k for k, _ in gpu_groups(agg.result(), types)]
        assert sorted(got, key=repr) == sorted(exp, key=repr), case["group_by"]
        ran += 1
    assert ran == len(g["cases"]) == 7


def test_reference_aggregate_values(tfa, ctx, dev, orc):
    """The aggregate VALUES the reference's tests pin (tests/golden/reference_cases.json
    "aggregates"): AggregationCount over the clerk table, gtest_aggregation_executor.cpp:562-585
    (count(x) skips NULL x), and sum(s2) = 6 (:755-757), on the device."""
    import json
    import os
    case = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_cases.json")))["aggregates"]
    clerk = case["clerk"]
    age = np.array([0 if a is None else a for a in clerk["age"]], dtype=np.int32)
    age_null = np.array([a is None for a in clerk["age"]], dtype=np.uint8)
    pr = np.array(clerk["pr"], dtype=np.uint64)
    country = str_col([s.encode() for s in clerk["country"]])
    gender = str_col([s.encode() for s in clerk["gender"]])
    for c in case["counts"]:
        kind, arg, atype, nulls = {"count(age)": (tfa.AGG_COUNT, age, tfa.INT32, age_null),
                                   "count(gender)": (tfa.AGG_COUNT_ALL, None, 0, None),
                                   "count(1)": (tfa.AGG_COUNT_ALL, None, 0, None),
                                   "count(pr)": (tfa.AGG_COUNT, pr, tfa.UINT64, None)}[c["func"]]
        word = atype | (tfa.NULLABLE if nulls is not None else 0)
        if not c["group_by"]:
            g = tfa.Aggregator(ctx, 0, [(kind, word)])
            g.consume(None, [to_dev(arg, dev) if arg is not None else None], n=len(age))
            got = [int(x) for x in g.result()["states"][0].cpu().numpy()]
        else:
            cols = {"country": country, "gender": gender}
            g = tfa.KeysAggregator(ctx, [tfa.STRING] * len(c["group_by"]), [(kind, word)])
            g.consume([to_dev(cols[k], dev) for k in c["group_by"]], [to_dev(arg, dev) if arg is not None else None],
                      arg_nullmaps=[to_dev(nulls, dev)] if nulls is not None else None)
            got = sorted(int(x) for x in g.result()["states"][0].cpu().numpy())
        assert got == sorted(c["expected"]), c
    s2 = np.array(case["test_table"]["s2"], dtype=np.int64)
    g = tfa.Aggregator(ctx, 0, [(tfa.AGG_SUM, tfa.INT64)])
    g.consume(None, [to_dev(s2, dev)], n=3)
    assert int(g.result()["states"][0].item()) == case["sums"][0]["expected"][0]


def rand_fixed(rng, t, n, card):
    np_t = {1: np.int8, 2: np.int16, 3: np.int32, 4: np.int64, 5: np.uint8, 6: np.uint16, 7: np.uint32, 8: np.uint64,
            10: np.float64}[t]
    if t == 10:
        base = rng.integers(-50, 50, card).astype(np.float64) / 4
        base[0] = -0.0  # raw bits: -0.0 and 0.0 are different keys, as serializeValueIntoArena copies bytes
        base[1] = 0.0
    else:
        info = np.iinfo(np_t)
        base = rng.integers(info.min, info.max, card, dtype=np_t, endpoint=True)
    return base[rng.integers(0, card, n)]


SERIAL_SETS = [
    [4, 20],            # bigint_, string_ (the reference's serialized case)
    [20, 20],           # country, gender
    [20, 3, 20, 1],     # String / fixed interleaved
    [4, 4, 8],          # 24 bytes: past keys128
    [4, 4, 4, 8, 3],    # five keys
    [1, 2, 3, 4, 5, 6, 7, 8],  # eight keys
    [13, 3],            # Decimal128 + Int32
    [10, 20],           # Float64 raw bits + String
]


@pytest.mark.parametrize("types", SERIAL_SETS, ids=lambda t: "-".join(map(str, t)))
@pytest.mark.parametrize("nullable", [False, True])
def test_serialized_keys(tfa, ctx, dev, orc, types, nullable):
    """The serialized method (HashMethodSerialized, ColumnsHashing.h:578-629) vs the oracle's
    serialised-bytes HashMap: two blocks (the second seeds the first's groups), a filter mask on
    the second, NULLs in every key column, String keys of 0-40 bytes under BIN_PADDING."""
    rng = np.random.default_rng(sum(types) * 7 + nullable)
    n = 40_000
    colls = [2 if t == 20 else 0 for t in types]
    vocab = vocab_strings(rng, 60, maxlen=40)
    blocks = []
    for b in range(2):
        keys, nulls = [], []
        for t in types:
            if t == 20:
                keys.append(str_col(rand_strings(rng, n, vocab)))
            elif t == 13:
                d = rng.integers(-3, 3, n).astype(object) * (1 << 100) + rng.integers(0, 5, n).astype(object)
                keys.append(np.array([[x & ((1 << 64) - 1), (x >> 64) & ((1 << 64) - 1)] for x in d],
                                     dtype=np.uint64).view(np.int64).reshape(-1))
            else:
                keys.append(rand_fixed(rng, t, n, 5 if len(types) > 3 else 13))
            nulls.append((rng.random(n) < 0.07).astype(np.uint8) if nullable else None)
        v = rng.integers(-10**6, 10**6, n, dtype=np.int64)
        mask = (rng.random(n) < 0.8).astype(np.uint8) if b == 1 else None
        blocks.append((keys, nulls, v, mask))
    aggs = [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.KeysAggregator(ctx, list(types), aggs, collators=colls)
    ref = orc.AggKeys(list(types), [(0, orc.INT64), (2, 0)], collators=colls)
    for keys, nulls, v, mask in blocks:
        dk = [to_dev(k, dev) for k in keys]
        agg.consume(dk, [to_dev(v, dev), None], key_nullmaps=[to_dev(x, dev) for x in nulls] if nullable else None,
                    mask=to_dev(mask, dev) if mask is not None else None)
        ref.consume(keys, [v, None], key_nulls=nulls if nullable else None, mask=mask)
    exp = ref.result()
    check_same(gpu_groups(agg.result(), list(types)), exp)
    # two-phase: the result's key columns merged into a fresh aggregator, and merge()
    res = agg.result()
    fin = tfa.KeysAggregator(ctx, list(types), aggs, collators=colls)
    fin.consume_partial(res["keys"], res["states"], key_nullmaps=res["key_null"])
    check_same(gpu_groups(fin.result(), list(types)), exp)
    other = tfa.KeysAggregator(ctx, list(types), aggs, collators=colls)
    other.merge(agg)
    check_same(gpu_groups(other.result(), list(types)), exp)
    agg.reset()
    assert agg.size() == 0


def test_serialized_keys_many_groups(tfa, ctx, dev, orc):
    """(Int64, String > 15 bytes) at 1.5M groups over 3M rows: the dictionary's slot table and key
    arena grow across blocks, Decimal(15,2) sums in Decimal128."""
    rng = np.random.default_rng(31)
    n, groups = 3_000_000, 1_500_000
    gid = rng.integers(0, groups, n)
    k1 = (gid % 997).astype(np.int64) - 400
    strs = [b"customer-%012d" % (g // 997) for g in gid]
    d = rng.integers(-10**12, 10**12, n, dtype=np.int64)
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.KeysAggregator(ctx, [tfa.INT64, tfa.STRING], aggs)
    cut = n // 3
    for lo, hi in ((0, cut), (cut, n)):
        c2, o2 = str_col(strs[lo:hi])
        agg.consume([to_dev(k1[lo:hi], dev), to_dev((c2, o2), dev)], [to_dev(d[lo:hi], dev), None])
    chars, offs = str_col(strs)
    ref = orc.AggKeys([orc.INT64, orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)])
    ref.consume([k1, (chars, offs)], [d, None])
    check_same(gpu_groups(agg.result(), [tfa.INT64, 20]), ref.result())


@pytest.mark.parametrize("collator", [0, 2])
def test_weak_hash_packed_string_keys(tfa, ctx, dev, orc, collator):
    """tfg_agg_weak_hash_packed (the two-phase sender's routing hash, computed from the packed
    keys) = IColumn::updateWeakHash32 of the key column (the oracle's ColumnString hash,
    ColumnString.cpp:1228-1327; NULL rows keep the seed, ColumnNullable.cpp:131-173): keys of 0-15
    bytes, trailing spaces (BIN_PADDING trims them before packing and before hashing), NULLs"""
    rng = np.random.default_rng(41 + collator)
    vocab = vocab_strings(rng, 2000)
    n = 40_000
    strs = rand_strings(rng, n, vocab)
    chars, offs = str_col(strs)
    knull = (rng.random(n) < 0.05).astype(np.uint8)
    agg = tfa.KeysAggregator(ctx, [tfa.STRING], [(tfa.AGG_COUNT_ALL, 0)], collators=[collator])
    agg.consume([to_dev((chars, offs), dev)], [None], key_nullmaps=[to_dev(knull, dev)])
    assert agg.holds_packed()
    packed = agg.result_packed()
    k16 = packed["keys"]
    g = k16.shape[0]
    h = torch.empty(g, dtype=torch.int32, device=dev)
    tfa.check(tfa.lib().tfg_weak_hash_init(ctx.h, tfa._p(h), tfa.ctypes.c_int64(g)))
    got = agg.weak_hash_packed(k16, h).cpu().numpy().view(np.uint32)
    agg.close()
    raw = k16.cpu().numpy().view(np.uint8).reshape(g, 16)
    isnull = (raw[:, 15] >> 7).astype(np.uint8)
    keys = [bytes(raw[i, :raw[i, 15] & 0x7F]) if not isnull[i] else b"" for i in range(g)]
    kc, ko = str_col(keys)
    want = orc.weak_hash_string(kc, ko, np.full(g, 0xFFFFFFFF, np.uint32), nullmap=isnull, collator=collator)
    np.testing.assert_array_equal(got, want)


def test_weak_hash_packed_fixed_keys(tfa, ctx, dev, orc):
    """the same for a keys128 tuple (Int32, nullable Int64): the values at their packed offsets,
    hashed as hash_key_row feeds them to crc32q, NULL bits in byte 15"""
    rng = np.random.default_rng(43)
    n = 50_000
    a = rng.integers(-1000, 1000, n).astype(np.int32)
    b = rng.integers(-2**40, 2**40, n).astype(np.int64) % 997
    bn = (rng.random(n) < 0.1).astype(np.uint8)
    agg = tfa.KeysAggregator(ctx, [tfa.INT32, tfa.INT64], [(tfa.AGG_COUNT_ALL, 0)])
    agg.consume([to_dev(a, dev), to_dev(b, dev)], [None], key_nullmaps=[None, to_dev(bn, dev)])
    packed = agg.result_packed()
    k16 = packed["keys"]
    g = k16.shape[0]
    h = torch.empty(g, dtype=torch.int32, device=dev)
    tfa.check(tfa.lib().tfg_weak_hash_init(ctx.h, tfa._p(h), tfa.ctypes.c_int64(g)))
    got = agg.weak_hash_packed(k16, h).cpu().numpy().view(np.uint32)
    agg.close()
    raw = k16.cpu().numpy().view(np.uint8).reshape(g, 16)
    ga = raw[:, 0:4].copy().view(np.int32).reshape(-1)
    gb = raw[:, 4:12].copy().view(np.int64).reshape(-1)
    nb = ((raw[:, 15] >> 1) & 1).astype(np.uint8)
    want = orc.weak_hash([ga, gb], types=[orc.INT32, orc.INT64], nullmaps=[None, nb])
    np.testing.assert_array_equal(got, want)
