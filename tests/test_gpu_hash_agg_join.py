"""GPU parity: weak hash / fillSelector / scatter (a22-a24), GROUP BY (a9-a17), hash join (a18-a21).

Known answers from the reference tests: keys 0..63 per block, P=4 -> 1024 rows per partition
(dbms/src/Flash/Mpp/tests/gtest_mpp_exchange_writer.cpp:663-718); aggregation / join results
are compared unordered like ExecutorTest (dbms/src/TestUtils/ExecutorTestUtils.cpp:243-253).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


# ------------------------------------------------------------------ hash / partition
@pytest.mark.parametrize("dtype,tcode", [(np.int8, 1), (np.int16, 2), (np.int32, 3), (np.int64, 4), (np.uint8, 5),
                                         (np.uint32, 7)])
def test_weak_hash_matches_hw_crc(tfa, ctx, dev, orc, dtype, tcode):
    rng = np.random.default_rng(tcode)
    n = 100_001
    info = np.iinfo(dtype)
    a = rng.integers(info.min, info.max, n, dtype=dtype, endpoint=True)
    nulls = (rng.random(n) < 0.1).astype(np.uint8)
    b = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    ta = torch.from_numpy(a.view({1: np.int8, 2: np.int16, 4: np.int32, 8: np.int64}[a.itemsize]) if dtype in (np.uint32,) else a).to(dev)
    h = tfa.weak_hash(ctx, [ta, torch.from_numpy(b).to(dev)], types=[tcode, tfa.INT64],
                      nullmaps=[torch.from_numpy(nulls).to(dev), None])
    exp = orc.weak_hash([a, b], types=[tcode, orc.INT64], nullmaps=[nulls, None])
    np.testing.assert_array_equal(_u32(h), exp)


def test_weak_hash_decimal128(tfa, ctx, dev, orc):
    rng = np.random.default_rng(9)
    n = 10_000
    d = rng.integers(-2**62, 2**62, (n, 2), dtype=np.int64)
    h = tfa.weak_hash(ctx, [torch.from_numpy(d).to(dev)], types=[tfa.DECIMAL128])
    np.testing.assert_array_equal(_u32(h), orc.weak_hash([d], types=[orc.DECIMAL128]))


@pytest.mark.parametrize("collator", [0, 1, 2])
def test_weak_hash_string(tfa, ctx, dev, orc, collator):
    strs = [b"", b"a", b"abc  ", b"12345678", b"123456789", b"k%08d" % 7, b"  ", b"x" * 31 + b" "] * 500
    chars = np.frombuffer(b"".join(s + b"\0" for s in strs), dtype=np.uint8).copy()
    offsets = np.cumsum([len(s) + 1 for s in strs]).astype(np.uint64)
    n = len(strs)
    nulls = (np.arange(n) % 11 == 0).astype(np.uint8)
    h = torch.full((n,), -1, dtype=torch.int32, device=dev)
    tfa.weak_hash_string(ctx, torch.from_numpy(chars).to(dev), torch.from_numpy(offsets.view(np.int64)).to(dev), h,
                         nullmap=torch.from_numpy(nulls).to(dev), collator=collator)
    exp = orc.weak_hash_string(chars, offsets, np.full(n, 0xFFFFFFFF, dtype=np.uint32), nulls, collator)
    np.testing.assert_array_equal(_u32(h), exp)


def test_exchange_known_answer(tfa, ctx, dev):
    """gtest_mpp_exchange_writer testHashPartitionWriter: 64 blocks x keys 0..63, P=4 -> 1024 each."""
    keys = torch.arange(64, dtype=torch.int64, device=dev).repeat(64)
    cols = [keys] + [keys.clone() for _ in range(9)]
    outs, offs = tfa.hash_partition(ctx, cols, [0], 4)
    assert [offs[i + 1] - offs[i] for i in range(4)] == [1024, 1024, 1024, 1024]
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("parts,fgs", [(1, 0), (2, 0), (4, 0), (7, 0), (8, 0), (4, 8), (64, 0), (1000, 0)])
@pytest.mark.parametrize("n", [0, 1, 1000, 300_017])
def test_stable_scatter(tfa, ctx, dev, orc, parts, fgs, n):
    rng = np.random.default_rng(parts * 31 + n)
    k = rng.integers(-2**40, 2**40, n, dtype=np.int64)
    p = rng.integers(0, 1 << 20, n, dtype=np.int64)
    h = orc.weak_hash([k])
    sel = orc.fill_selector(h, parts, fgs)
    total_parts = parts * fgs if fgs else parts
    perm, offs = orc.partition(sel, total_parts)
    # GPU pieces
    kd = torch.from_numpy(k).to(dev)
    hd = tfa.weak_hash(ctx, [kd])
    np.testing.assert_array_equal(_u32(hd), h)
    sd = tfa.fill_selector(ctx, hd, parts, fgs)
    np.testing.assert_array_equal(_u32(sd), sel)
    gperm, goffs = tfa.partition(ctx, sd, total_parts)
    np.testing.assert_array_equal(np.array(goffs, dtype=np.uint64), offs)
    np.testing.assert_array_equal(_u32(gperm), perm)  # stable: exact scatter order
    if fgs == 0:
        outs, hoffs = tfa.hash_partition(ctx, [kd, torch.from_numpy(p).to(dev)], [0], parts)
        np.testing.assert_array_equal(np.array(hoffs, dtype=np.uint64), offs)
        np.testing.assert_array_equal(outs[0].cpu().numpy(), k[perm])
        np.testing.assert_array_equal(outs[1].cpu().numpy(), p[perm])


# ------------------------------------------------------------------ aggregation
def _sorted_rows(keys, key_null, states, state_null=None):
    rows = []
    for i in range(len(keys)):
        kn = int(key_null[i]) if key_null is not None else 0
        r = [kn, 0 if kn else int(keys[i])]
        for j, s in enumerate(states):
            v = s[i]
            if s.ndim == 2:
                v = tuple(int(x) for x in v)
            elif s.dtype == np.float64:
                v = float(v)
            else:
                v = int(v)
            if state_null is not None and state_null[j] is not None and state_null[j][i]:
                v = None
            r.append(v)
        rows.append(tuple(r))
    return sorted(rows, key=repr)


def _gpu_rows(res, key_np_dtype, with_null):
    keys = res["keys"].cpu().numpy().view(key_np_dtype) if res["keys"] is not None else np.zeros(len(res["key_null"]), key_np_dtype)
    states = [s.cpu().numpy() for s in res["states"]]
    states = [s.view(np.uint64) if s.dtype == np.int64 and s.ndim == 1 else s for s in states]
    return _sorted_rows(keys.astype(np.int64) if keys.dtype != np.uint64 else keys, res["key_null"].cpu().numpy(),
                        states, [s.cpu().numpy() for s in res["state_null"]] if with_null else None)


def _ref_rows(r, key_np_dtype, with_null):
    keys = r["keys"].astype(np.uint64).view(np.uint64)
    width = np.dtype(key_np_dtype).itemsize
    keys = (keys & np.uint64((1 << (8 * width)) - 1) if width < 8 else keys).astype(np.uint64)
    keys = keys.astype({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[width]).view(key_np_dtype)
    states = [s.view(np.uint64) if s.dtype == np.int64 and s.ndim == 1 else s for s in r["states"]]
    return _sorted_rows(keys.astype(np.int64) if keys.dtype != np.uint64 else keys, r["key_null"], states,
                        r["state_null"] if with_null else None)


@pytest.mark.parametrize("groups", [1, 7, 1000, 100_000])
@pytest.mark.parametrize("n", [0, 1, 5000, 400_000])
def test_groupby_sum_count_int64_key(tfa, ctx, dev, orc, groups, n):
    rng = np.random.default_rng(groups + n)
    k = rng.integers(-groups // 2, groups - groups // 2, n, dtype=np.int64)  # includes key 0
    vi = rng.integers(-2**40, 2**40, n, dtype=np.int64)
    vf = rng.integers(0, 1 << 20, n).astype(np.float64) / 256.0  # dyadic -> exact, order-independent
    aggs = [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)]
    g = tfa.Aggregator(ctx, tfa.INT64, aggs)
    g.consume(torch.from_numpy(k).to(dev), [torch.from_numpy(vi).to(dev), torch.from_numpy(vf).to(dev), None], n=n)
    ref = orc.Agg(orc.INT64, [(0, orc.INT64), (0, orc.FLOAT64), (2, 0)])
    ref.consume(k, [vi, vf, None], n=n)
    assert g.size() == ref.size()
    assert _gpu_rows(g.result(), np.int64, False) == _ref_rows(ref.result(), np.int64, False)


@pytest.mark.parametrize("key_dtype,kt", [(np.int8, 1), (np.int16, 2), (np.int32, 3), (np.uint8, 5), (np.uint64, 8)])
def test_groupby_nullable_keys_and_args(tfa, ctx, dev, orc, key_dtype, kt):
    rng = np.random.default_rng(kt)
    n = 200_000
    info = np.iinfo(key_dtype)
    k = rng.integers(max(info.min, -3000), min(info.max, 3000), n, dtype=key_dtype, endpoint=True)
    kn = (rng.random(n) < 0.05).astype(np.uint8)
    v = rng.integers(-1000, 1000, n, dtype=np.int32)
    vn = (rng.random(n) < 0.3).astype(np.uint8)
    aggs = [(tfa.AGG_SUM, tfa.INT32 | tfa.NULLABLE), (tfa.AGG_COUNT, tfa.INT32 | tfa.NULLABLE), (tfa.AGG_COUNT_ALL, 0)]
    g = tfa.Aggregator(ctx, kt, aggs, bucket_bits=5)
    vd, vnd = torch.from_numpy(v).to(dev), torch.from_numpy(vn).to(dev)
    kd = torch.from_numpy(k.view({1: np.int8, 2: np.int16, 4: np.int32, 8: np.int64}[k.itemsize]) if key_dtype == np.uint64 else k).to(dev)
    g.consume(kd, [vd, vd, None], key_nullmap=torch.from_numpy(kn).to(dev), arg_nullmaps=[vnd, vnd, None])
    ref = orc.Agg(kt, [(0, orc.INT32), (1, orc.INT32), (2, 0)])
    ref.consume(k, [v, v, None], key_null=kn, arg_nulls=[vn, vn, None])
    assert _gpu_rows(g.result(), key_dtype, True) == _ref_rows(ref.result(), key_dtype, True)


def _limbs_to_ints(a):
    """(n, L) int64 limbs (little-endian two's complement) -> Python ints."""
    from oracle.oracle import limbs_to_int
    return [limbs_to_int(r) for r in a]


def _exact_group_sums(k, vals):
    """Python big-int sums per key: the exact value boost checked_int256_t holds (no overflow)."""
    out = {}
    for key, v in zip(k.tolist(), vals):
        out[key] = out.get(key, 0) + v
    return out


def test_groupby_decimal_sum_result_types(tfa, ctx):
    """SumDecimalInferer (Common/Decimal.h:156-163) -> Decimal(min(p+22,65)): Decimal128 up to 38
    digits, Decimal256 above (AggregateFunctionSum.cpp:57-85); integer sums per
    gtest_sum_int_agg_func.cpp ReturnTypeForIntegerInputs."""
    import ctypes
    cases = [(tfa.prec(tfa.DECIMAL32, 9), tfa.DECIMAL128, 16), (tfa.prec(tfa.DECIMAL64, 15), tfa.DECIMAL128, 16),
             (tfa.prec(tfa.DECIMAL64, 16), tfa.DECIMAL128, 16), (tfa.prec(tfa.DECIMAL64, 17), tfa.DECIMAL256, 32),
             (tfa.DECIMAL64, tfa.DECIMAL256, 32), (tfa.prec(tfa.DECIMAL128, 19), tfa.DECIMAL256, 32),
             (tfa.DECIMAL128, tfa.DECIMAL256, 32), (tfa.prec(tfa.DECIMAL256, 65), tfa.DECIMAL256, 32),
             (tfa.INT8, tfa.INT64, 8), (tfa.INT32, tfa.INT64, 8), (tfa.UINT16, tfa.UINT64, 8),
             (tfa.UINT64, tfa.UINT64, 8), (tfa.FLOAT32, tfa.FLOAT64, 8)]
    for arg, want_t, want_w in cases:
        g = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_SUM, arg)])
        t, w = ctypes.c_int(), ctypes.c_int()
        tfa.check(tfa.lib().tfg_agg_result_type(g.h, 0, ctypes.byref(t), ctypes.byref(w)))
        assert (t.value, w.value) == (want_t, want_w), (hex(arg), t.value, w.value)
        g.close()


def test_groupby_decimal_sum_exact(tfa, ctx, dev, orc):
    """sum(Decimal(15,2)) -> Decimal(37,2) (Int128); sum(Decimal(18,s)) and sum(Decimal128) ->
    Decimal256, exact where Int128 would overflow: Decimal128 values near 2^126, ~60 per group,
    sum past 2^127.  Checked against Python big-int sums and the oracle."""
    rng = np.random.default_rng(12)
    n = 300_000
    k = rng.integers(0, 5000, n, dtype=np.int64)
    d15 = rng.integers(-10**15 + 1, 10**15 - 1, n, dtype=np.int64)
    d18 = rng.integers(-10**18 + 1, 10**18 - 1, n, dtype=np.int64)
    hi = rng.integers(2**61, 2**62, n, dtype=np.int64) * np.where(rng.random(n) < 0.8, 1, -1)
    d128 = np.stack([rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64), hi], axis=1)
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 18)),
            (tfa.AGG_SUM, tfa.DECIMAL128), (tfa.AGG_COUNT_ALL, 0)]
    g = tfa.Aggregator(ctx, tfa.INT64, aggs)
    g.consume(torch.from_numpy(k).to(dev), [torch.from_numpy(x).to(dev) for x in (d15, d18, d128)] + [None])
    r = g.result()
    assert r["states"][0].shape[1] == 2 and r["states"][1].shape[1] == 4 and r["states"][2].shape[1] == 4
    keys = r["keys"].cpu().numpy().tolist()
    got = [dict(zip(keys, _limbs_to_ints(r["states"][i].cpu().numpy()))) for i in range(3)]
    v128 = [(int(b) << 64) | (int(a) & (2**64 - 1)) for a, b in d128]
    exp = [_exact_group_sums(k, d15.tolist()), _exact_group_sums(k, d18.tolist()), _exact_group_sums(k, v128)]
    assert got == exp
    assert max(abs(v) for v in exp[2].values()) >= 2**127, "the Decimal128 sums must leave Int128"
    ref = orc.Agg(orc.INT64, [(0, orc.prec(orc.DECIMAL64, 15)), (0, orc.prec(orc.DECIMAL64, 18)), (0, orc.DECIMAL128)])
    ref.consume(k, [d15, d18, d128])
    rr = ref.result()
    for i in range(3):
        assert dict(zip(rr["keys"].view(np.int64).tolist(), _limbs_to_ints(rr["states"][i]))) == exp[i]


def test_groupby_decimal256_args_and_two_phase(tfa, ctx, dev, orc):
    """sum(Decimal(65,s)) over Decimal256 arguments (|x| < 10^65) with a nullable argument;
    partial (32-byte states) -> hash repartition -> final (sumOnPartialResult keeps the type)."""
    rng = np.random.default_rng(13)
    n = 80_000
    k = rng.integers(0, 3000, n, dtype=np.int64)
    vals = [int(x) * 10**48 + int(y) for x, y in zip(rng.integers(-10**16, 10**16, n), rng.integers(0, 10**15, n))]
    from oracle.oracle import int_to_limbs
    d256 = np.stack([int_to_limbs(v, 4) for v in vals])
    vn = (rng.random(n) < 0.1).astype(np.uint8)
    word = tfa.prec(tfa.DECIMAL256, 65) | tfa.NULLABLE
    aggs = [(tfa.AGG_SUM, word), (tfa.AGG_COUNT_ALL, 0)]
    exp = {}
    for key, v, isnull in zip(k.tolist(), vals, vn.tolist()):
        s = exp.setdefault(key, [0, 0])
        if not isnull:
            s[0] += v
        s[1] += 1
    halves = []
    for lo, hi in ((0, n // 2), (n // 2, n)):
        p = tfa.Aggregator(ctx, tfa.INT64, aggs, bucket_bits=5)
        p.consume(torch.from_numpy(k[lo:hi]).to(dev), [torch.from_numpy(d256[lo:hi]).to(dev), None],
                  arg_nullmaps=[torch.from_numpy(vn[lo:hi]).to(dev), None])
        halves.append(p.result())
    fin = tfa.Aggregator(ctx, tfa.INT64, aggs, bucket_bits=4)
    for r in halves:
        cols, offs = tfa.hash_partition(ctx, [r["keys"], r["states"][0], r["states"][1], r["state_null"][0]], [0], 2,
                                        types=[tfa.INT64, tfa.DECIMAL256, tfa.INT64, tfa.UINT8])
        fin.consume_partial(cols[0], [cols[1], cols[2]], state_nullmaps=[cols[3], None])
    fr = fin.result()
    got = dict(zip(fr["keys"].cpu().numpy().tolist(),
                   [[a, int(c)] for a, c in zip(_limbs_to_ints(fr["states"][0].cpu().numpy()), fr["states"][1].cpu().numpy())]))
    assert got == exp
    ref = orc.Agg(orc.INT64, [(0, orc.prec(orc.DECIMAL256, 65)), (2, 0)])
    ref.consume(k, [d256, None], arg_nulls=[vn, None])
    rr = ref.result()
    assert dict(zip(rr["keys"].view(np.int64).tolist(), _limbs_to_ints(rr["states"][0]))) == {a: b[0] for a, b in exp.items()}


def test_groupby_multi_block_and_overflowing_buckets(tfa, ctx, dev, orc):
    """Many blocks (executeOnBlock repeatedly) + far more groups than the LDS tables hold in few
    buckets (forces the spill iterations, like force_agg_two_level / partial-block failpoints)."""
    rng = np.random.default_rng(21)
    aggs = [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)]
    g = tfa.Aggregator(ctx, tfa.INT64, aggs, bucket_bits=4)  # 16 buckets for ~200K groups
    ref = orc.Agg(orc.INT64, [(0, orc.INT64), (2, 0)])
    for blk in range(6):
        n = [1, 65536, 0, 100_000, 7, 250_000][blk]
        k = rng.integers(0, 200_000, n, dtype=np.int64)
        v = rng.integers(-100, 100, n, dtype=np.int64)
        g.consume(torch.from_numpy(k).to(dev), [torch.from_numpy(v).to(dev), None], n=n)
        ref.consume(k, [v, None], n=n)
    assert g.size() == ref.size()
    assert _gpu_rows(g.result(), np.int64, False) == _ref_rows(ref.result(), np.int64, False)


def test_groupby_merge_and_partial(tfa, ctx, dev, orc):
    """Per-thread tables merged (mergeDataImpl) and two-phase partial -> final (gtest_compute_server)."""
    rng = np.random.default_rng(5)
    aggs = [(tfa.AGG_SUM, tfa.INT64 | tfa.NULLABLE), (tfa.AGG_COUNT_ALL, 0)]
    parts, ref = [], orc.Agg(orc.INT64, [(0, orc.INT64), (2, 0)])
    for t in range(4):
        n = 100_000
        k = rng.integers(0, 30_000, n, dtype=np.int64)
        v = rng.integers(-100, 100, n, dtype=np.int64)
        vn = (rng.random(n) < 0.5).astype(np.uint8)
        a = tfa.Aggregator(ctx, tfa.INT64, aggs, bucket_bits=6)
        a.consume(torch.from_numpy(k).to(dev), [torch.from_numpy(v).to(dev), None],
                  arg_nullmaps=[torch.from_numpy(vn).to(dev), None])
        parts.append(a)
        ref.consume(k, [v, None], arg_nulls=[vn, None])
    merged = tfa.Aggregator(ctx, tfa.INT64, aggs, bucket_bits=6)
    for a in parts:
        merged.merge(a)
    exp = _ref_rows(ref.result(), np.int64, True)
    assert _gpu_rows(merged.result(), np.int64, True) == exp
    final = tfa.Aggregator(ctx, tfa.INT64, aggs, bucket_bits=3)
    for a in parts:
        r = a.result()
        final.consume_partial(r["keys"], r["states"], state_nullmaps=r["state_null"])
    assert _gpu_rows(final.result(), np.int64, True) == exp


def test_groupby_without_key(tfa, ctx, dev, orc):
    rng = np.random.default_rng(8)
    n = 1_000_000
    a = rng.integers(0, 2**31, n, dtype=np.int64)
    aggs = [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0), (tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 12)),
            (tfa.AGG_SUM, tfa.DECIMAL64)]
    g = tfa.Aggregator(ctx, 0, aggs)
    ad = torch.from_numpy(a).to(dev)
    g.consume_filtered(ad, tfa.LT, 2**30, None, [ad, None, ad, ad])
    r = g.result()
    m = a < 2**30
    assert g.size() == 1
    assert int(r["states"][0].item()) == int(a[m].sum())
    assert int(r["states"][1].item()) == int(m.sum())
    assert r["states"][2].shape[1] == 2 and r["states"][3].shape[1] == 4  # Decimal(34,s) / Decimal(40,s)
    assert _limbs_to_ints(r["states"][2].cpu().numpy()) == [int(a[m].sum())]
    assert _limbs_to_ints(r["states"][3].cpu().numpy()) == [int(a[m].sum())]


def test_groupby_reference_gtest_groups(tfa, ctx, dev):
    """GroupBy expected key sets from dbms/src/Flash/tests/gtest_aggregation_executor.cpp:313-420."""
    import json, os
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_cases.json")))["groupby"]
    for case in cases:
        vals = case["column"]
        n = len(vals)
        kn = np.array([v is None for v in vals], dtype=np.uint8)
        k = np.array([0 if v is None else v for v in vals], dtype=case["dtype"])
        g = tfa.Aggregator(ctx, case["type"], [(tfa.AGG_COUNT_ALL, 0)], bucket_bits=4)
        g.consume(torch.from_numpy(k).to(dev), [None], key_nullmap=torch.from_numpy(kn).to(dev), n=n)
        r = g.result()
        keys = r["keys"].cpu().numpy().view(case["dtype"])
        got = sorted([None if r["key_null"][i] else int(keys[i]) for i in range(g.size())], key=repr)
        assert got == sorted(case["expected"], key=repr), case["name"]


# ------------------------------------------------------------------ join
def _pairs(pi, bi):
    return sorted(zip(pi.tolist(), bi.tolist()))


JOIN_VERSIONS = [dict(), dict(v2=True, tagged=False), dict(v2=True, tagged=True)]  # v1; JoinV2 pointer table
JOIN_IDS = ["v1", "v2", "v2tagged"]


@pytest.mark.parametrize("ver", JOIN_VERSIONS, ids=JOIN_IDS)
@pytest.mark.parametrize("kind", [0, 1, 2, 3])
@pytest.mark.parametrize("nb,np_,dup", [(0, 100, 1), (1, 1, 1), (1000, 5000, 1), (50_000, 400_000, 1),
                                        (20_000, 100_000, 3), (3000, 20_000, 2500)])
def test_join_kinds(tfa, ctx, dev, orc, kind, nb, np_, dup, ver):
    rng = np.random.default_rng(nb + np_ + kind)
    distinct = max(1, nb // dup)
    bk = rng.integers(-distinct, distinct, nb, dtype=np.int64) if dup > 1 else rng.permutation(nb).astype(np.int64) * 4 + 1
    bnull = (rng.random(nb) < 0.02).astype(np.uint8)
    pk = np.where(rng.random(np_) < 0.5, bk[rng.integers(0, max(nb, 1), np_)] if nb else 3,
                  rng.integers(-2**40, 2**40, np_) * 4 + 3)
    pk[: min(np_, 3)] = [0, -1, 1][: min(np_, 3)]
    pnull = (rng.random(np_) < 0.02).astype(np.uint8)
    j = tfa.Join(ctx, tfa.INT64, **ver)
    if nb:
        j.build(torch.from_numpy(bk).to(dev), key_nullmap=torch.from_numpy(bnull).to(dev))
    pi, bi = j.probe(torch.from_numpy(pk).to(dev), kind=kind, key_nullmap=torch.from_numpy(pnull).to(dev))
    ref = orc.JoinRef(orc.INT64)
    ref.build(bk, bnull if nb else None)
    epi, ebi = ref.probe(pk, kind=kind, key_null=pnull)
    got_b = bi.cpu().numpy().view(np.uint32)
    if kind in (2, 3):  # SEMI / ANTI: probe rows only
        assert sorted(pi.cpu().numpy().view(np.uint32).tolist()) == sorted(epi.tolist())
    else:
        assert _pairs(pi.cpu().numpy().view(np.uint32), got_b) == _pairs(epi, ebi)


@pytest.mark.parametrize("ver", JOIN_VERSIONS, ids=JOIN_IDS)
def test_join_multi_block_build_and_small_keys(tfa, ctx, dev, orc, ver):
    rng = np.random.default_rng(4)
    j = tfa.Join(ctx, tfa.INT32, **ver)
    ref = orc.JoinRef(orc.INT32)
    for n in (10, 0, 5000, 20_000):
        bk = rng.integers(-3000, 3000, n).astype(np.int32)
        if n:
            j.build(torch.from_numpy(bk).to(dev))
        ref.build(bk)
    pk = rng.integers(-4000, 4000, 100_000).astype(np.int32)
    pi, bi = j.probe(torch.from_numpy(pk).to(dev), kind=tfa.JOIN_INNER)
    epi, ebi = ref.probe(pk)
    assert _pairs(pi.cpu().numpy().view(np.uint32), bi.cpu().numpy().view(np.uint32)) == _pairs(epi, ebi)


def test_join_capacity_retry(tfa, ctx, dev):
    keys = torch.zeros(1000, dtype=torch.int64, device=dev)
    j = tfa.Join(ctx, tfa.INT64)
    j.build(keys)
    with pytest.raises(tfa.TfgError) as e:
        j.probe(keys[:10], capacity=5, out_probe=torch.empty(5, dtype=torch.int32, device=dev),
                out_build=torch.empty(5, dtype=torch.int32, device=dev))
    assert e.value.code == tfa.TFG_ERR_CAPACITY
    pi, bi = j.probe(keys[:10])
    assert pi.shape[0] == 10_000


@pytest.mark.gpu
@pytest.mark.parametrize("ver", JOIN_VERSIONS, ids=JOIN_IDS)
@pytest.mark.parametrize("kind", [0, 1, 2, 3])
@pytest.mark.parametrize("key_as_payload", [True, False])
@pytest.mark.parametrize("nb,np_,dup", [(0, 1000, 1), (3000, 50_000, 1), (20_000, 60_000, 30), (200_000, 300_000, 1),
                                        (9000, 2000, 9000)])
def test_join_probe_rows_materialised(tfa, ctx, dev, orc, kind, key_as_payload, nb, np_, dup, ver):
    """Materialising probe (tfg_join_probe_rows): every output row carries the probe payloads and
    the matched build payload; compared as a multiset with the restatement's pairs."""
    rng = np.random.default_rng(nb + np_ + kind + 17 * key_as_payload)
    distinct = max(1, nb // dup)
    bk = rng.integers(-distinct, distinct, nb, dtype=np.int64) if dup > 1 else rng.permutation(nb).astype(np.int64) * 4 + 1
    bnull = (rng.random(nb) < 0.02).astype(np.uint8)
    bpay = rng.integers(-2**62, 2**62, nb, dtype=np.int64)
    pk = np.where(rng.random(np_) < 0.5, bk[rng.integers(0, max(nb, 1), np_)] if nb else 3,
                  rng.integers(-2**40, 2**40, np_) * 4 + 3)
    pk[:3] = [0, -1, 1]
    pnull = (rng.random(np_) < 0.02).astype(np.uint8)
    ppay = rng.integers(-2**62, 2**62, np_, dtype=np.int64)
    j = tfa.Join(ctx, tfa.INT64, expected_build_rows=nb, **ver)
    half = nb // 2
    for lo, hi in ((0, half), (half, nb)):  # two build blocks
        if hi > lo:
            j.build(torch.from_numpy(bk[lo:hi]).to(dev), key_nullmap=torch.from_numpy(bnull[lo:hi]).to(dev),
                    payload=[torch.from_numpy(bpay[lo:hi]).to(dev)])
    if nb == 0:
        j.build(torch.empty(0, dtype=torch.int64, device=dev), payload=[torch.empty(0, dtype=torch.int64, device=dev)])
    pkd = torch.from_numpy(pk).to(dev)
    pay = [pkd, torch.from_numpy(ppay).to(dev)] if key_as_payload else [torch.from_numpy(ppay).to(dev)]
    op, ob, bnl = j.probe_rows(pkd, pay, 1, kind=kind, key_nullmap=torch.from_numpy(pnull).to(dev))
    ref = orc.JoinRef(orc.INT64)
    ref.build(bk, bnull if nb else None)
    epi, ebi = ref.probe(pk, kind=kind, key_null=pnull)
    want_p = ppay[epi]
    got_p = op[-1].cpu().numpy()
    if kind in (2, 3):
        assert len(ob) == 0
        assert sorted(got_p.tolist()) == sorted(want_p.tolist())
        if key_as_payload:
            assert sorted(op[0].cpu().numpy().tolist()) == sorted(pk[epi].tolist())
        return
    unmatched = ebi == 0xFFFFFFFF
    bp = np.append(bpay, 0)
    want_b = bp[np.where(unmatched, len(bpay), ebi)]
    got_b = ob[0].cpu().numpy()
    want = sorted(zip(want_p.tolist(), want_b.tolist(), unmatched.astype(int).tolist()))
    gotn = bnl.cpu().numpy().astype(int) if kind == 1 else np.zeros(len(got_p), dtype=int)
    got = sorted(zip(got_p.tolist(), got_b.tolist(), gotn.tolist()))
    assert got == want
    if key_as_payload:
        assert sorted(op[0].cpu().numpy().tolist()) == sorted(pk[epi].tolist())


@pytest.mark.parametrize("with_payload", [True, False])
def test_join_two_pass_partitions(tfa, ctx, dev, orc, with_payload):
    """Build sides above 1024 x 2560 rows partition in two radix passes (P = 4096): pairs and
    payloads must match the restatement."""
    rng = np.random.default_rng(55)
    nb, np_ = 5_500_000, 400_000
    bk = rng.permutation(nb).astype(np.int64) * 4 + 1
    pk = np.where(rng.random(np_) < 0.5, bk[rng.integers(0, nb, np_)], rng.integers(0, 2**40, np_) * 4 + 3)
    j = tfa.Join(ctx, tfa.INT64, expected_build_rows=nb)
    bkd, pkd = torch.from_numpy(bk).to(dev), torch.from_numpy(pk).to(dev)
    ref = orc.JoinRef(orc.INT64)
    ref.build(bk)
    epi, ebi = ref.probe(pk)
    if with_payload:
        j.build(bkd, payload=[bkd * 7])
        op, ob, _ = j.probe_rows(pkd, [pkd], 1)
        assert j.stats()[1] == 4096
        got = sorted(zip(op[0].cpu().tolist(), ob[0].cpu().tolist()))
        assert got == sorted(zip(pk[epi].tolist(), (bk[ebi] * 7).tolist()))
    else:
        j.build(bkd)
        pi, bi = j.probe(pkd)
        assert _pairs(pi.cpu().numpy().view(np.uint32), bi.cpu().numpy().view(np.uint32)) == _pairs(epi, ebi)


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
@pytest.mark.parametrize("pays", ["key", "key+pay", "pay2"])
def test_join_two_level_probe_partition(tfa, ctx, dev, orc, kind, pays):
    """Probe sides of a build above 1024 x 2560 rows (P = 2048 here) take the two-level tiled
    partition (join.part.tiled + join.part.regroup) for 1-3 word probe records; NULL keys,
    duplicate build keys and a skewed probe block (a third of the rows on one key) included."""
    rng = np.random.default_rng(61 + kind)
    nb, np_ = 3_000_000, 900_000
    bk = rng.permutation(nb).astype(np.int64) * 4 + 1
    bk[: nb // 10] = bk[nb // 10: nb // 5]  # 10% of the keys appear twice
    bnull = (rng.random(nb) < 0.01).astype(np.uint8)
    bpay = rng.integers(-2**62, 2**62, nb, dtype=np.int64)
    pk = np.where(rng.random(np_) < 0.5, bk[rng.integers(0, nb, np_)], rng.integers(0, 2**40, np_) * 4 + 3)
    pk[: np_ // 3] = bk[nb // 2]
    pnull = (rng.random(np_) < 0.01).astype(np.uint8)
    pp1 = rng.integers(-2**62, 2**62, np_, dtype=np.int64)
    pp2 = rng.integers(-2**62, 2**62, np_, dtype=np.int64)
    j = tfa.Join(ctx, tfa.INT64, expected_build_rows=nb)
    j.build(torch.from_numpy(bk).to(dev), key_nullmap=torch.from_numpy(bnull).to(dev),
            payload=[torch.from_numpy(bpay).to(dev)])
    pkd = torch.from_numpy(pk).to(dev)
    cols = {"key": [pk], "key+pay": [pk, pp1], "pay2": [pp1, pp2]}[pays]
    pay = [pkd if c is pk else torch.from_numpy(c).to(dev) for c in cols]
    op, ob, bnl = j.probe_rows(pkd, pay, 1, kind=kind, key_nullmap=torch.from_numpy(pnull).to(dev),
                               capacity=2 * np_)
    assert j.stats()[1] == 2048
    ref = orc.JoinRef(orc.INT64)
    ref.build(bk, bnull)
    epi, ebi = ref.probe(pk, kind=kind, key_null=pnull)
    want_p = np.stack([c[epi] for c in cols], 1)
    got_p = np.stack([o.cpu().numpy() for o in op], 1)
    if kind in (2, 3):
        assert len(ob) == 0
        assert sorted(map(tuple, got_p.tolist())) == sorted(map(tuple, want_p.tolist()))
        return
    unmatched = ebi == 0xFFFFFFFF
    want_b = np.append(bpay, 0)[np.where(unmatched, nb, ebi)]
    gotn = bnl.cpu().numpy().astype(np.int64) if kind == 1 else np.zeros(len(got_p), dtype=np.int64)
    got = np.concatenate([got_p, ob[0].cpu().numpy()[:, None], gotn[:, None]], 1)
    want = np.concatenate([want_p, want_b[:, None], unmatched.astype(np.int64)[:, None]], 1)
    assert got.shape == want.shape
    assert np.array_equal(got[np.lexsort(got.T[::-1])], want[np.lexsort(want.T[::-1])])


@pytest.mark.parametrize("tagged", [False, True])
def test_join_v2_c3_shape(tfa, ctx, dev, orc, tagged):
    """JoinV2 pointer table at C3's shape, scaled (2M build rows with unique keys k*4+1, 20M probe
    rows half hits / half k*4+3 misses, Int64 payloads materialised): the multiset of (probe
    payload, build payload) rows equals the v1 restatement's."""
    rng = np.random.default_rng(57)
    nb, np_ = 2_000_000, 20_000_000
    bk = rng.permutation(nb).astype(np.int64) * 4 + 1
    pk = np.where(rng.random(np_) < 0.5, bk[rng.integers(0, nb, np_)], rng.integers(0, 2**40, np_) * 4 + 3)
    bkd, pkd = torch.from_numpy(bk).to(dev), torch.from_numpy(pk).to(dev)
    j = tfa.Join(ctx, tfa.INT64, expected_build_rows=nb, v2=True, tagged=tagged)
    j.build(bkd, payload=[bkd * 7 + 1])
    op, ob, _ = j.probe_rows(pkd, [pkd], 1)
    ref = orc.JoinRef(orc.INT64)
    ref.build(bk)
    epi, ebi = ref.probe(pk)
    got = np.stack([op[0].cpu().numpy(), ob[0].cpu().numpy()], 1)
    want = np.stack([pk[epi], bk[ebi] * 7 + 1], 1)
    assert got.shape == want.shape
    np.testing.assert_array_equal(got[np.lexsort(got.T[::-1])], want[np.lexsort(want.T[::-1])])


def test_groupby_two_pass_buckets(tfa, ctx, dev, orc):
    """4096 aggregation buckets (two-pass radix partition) vs the restatement."""
    rng = np.random.default_rng(56)
    n = 3_000_000
    k = rng.integers(0, 8_000_000, n, dtype=np.int64)
    v = rng.integers(-1000, 1000, n, dtype=np.int64)
    g = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)], expected_groups=8_000_000)
    g.consume(torch.from_numpy(k).to(dev), [torch.from_numpy(v).to(dev), None])
    r = g.result()
    ref = orc.Agg(orc.INT64, [(0, orc.INT64), (2, 0)])
    ref.consume(k, [v, None])
    rr = ref.result()
    got = sorted(zip(r["keys"].cpu().numpy().view(np.int64).tolist(), r["states"][0].cpu().tolist(),
                     r["states"][1].cpu().tolist()))
    want = sorted(zip(rr["keys"].view(np.int64).tolist(), rr["states"][0].tolist(), rr["states"][1].tolist()))
    assert got == want


@pytest.mark.parametrize("filtered", [False, True])
def test_groupby_tiled_narrow_and_wide_tiles(tfa, ctx, dev, orc, filtered):
    """The tiled partition writes a tile whose kept keys all fit 32 bits as u32 keys + values
    (12 B a row) and any other tile as {key, value} records: one consume whose tiles mix both
    (runs of keys below 2^32, runs of full-range Int64 keys incl. negatives, the 2^32 - 1 / 2^32
    boundary), through the C2 fast signature (sum Float64 + count) and the filtered consume."""
    rng = np.random.default_rng(77)
    n = 3_000_000
    small = rng.integers(0, 1 << 20, n, dtype=np.int64)
    big = rng.integers(-2**63, 2**63 - 1, 50_000, dtype=np.int64)[rng.integers(0, 50_000, n)]
    edge = np.array([2**32 - 1, 2**32, 0, -1], dtype=np.int64)[rng.integers(0, 4, n)]
    seg = (np.arange(n) // 40_000) % 5  # 40K-row segments: a tile of 8192 rows is all one kind or mixed
    k = np.where(seg < 3, small, np.where(seg == 3, big, edge))
    v = rng.integers(0, 1 << 20, n).astype(np.float64) / 256.0
    f = rng.integers(0, 100, n, dtype=np.int64)
    aggs = [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)]
    g = tfa.Aggregator(ctx, tfa.INT64, aggs)
    kd, vd, fd = (torch.from_numpy(x).to(dev) for x in (k, v, f))
    ref = orc.Agg(orc.INT64, [(0, orc.FLOAT64), (2, 0)])
    if filtered:
        g.consume_filtered(fd, tfa.LT, 60, kd, [vd, None])
        ref.consume(k, [v, None], mask=(f < 60).astype(np.uint8))
    else:
        g.consume(kd, [vd, None], n=n)
        ref.consume(k, [v, None], n=n)
    assert g.size() == ref.size()
    assert _gpu_rows(g.result(), np.int64, False) == _ref_rows(ref.result(), np.int64, False)
