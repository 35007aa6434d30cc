"""CPU tests: pin the oracle (CPU restatement) against the reference's own known answers and the
hardware CRC32-C instruction.  No GPU needed."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_crc_sw_matches_hw_instruction(orc):
    assert orc.lib().orc_has_hw_crc() == 1, "oracle must be built with SSE4.2 (the reference's crc32q)"
    rng = np.random.default_rng(0)
    for _ in range(20000):
        s, x = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**63)) * 2 + int(rng.integers(0, 2))
        assert orc.crc32c_u64(s, x) == orc.crc32c_u64_sw(s, x)


def test_crc_golden_vectors(orc):
    g = _load("crc_vectors.json")
    for v in g["crc32c_u64"]:
        assert orc.crc32c_u64(v["crc"], v["x"]) == v["out"]
        assert orc.crc32c_u64_sw(v["crc"], v["x"]) == v["out"]
    for v in g["weak_hash_bytes"]:
        s = v["s"].encode()
        assert orc.lib().orc_update_weak_hash32_bytes(s, len(s), 0xFFFFFFFF) == v["h"]


def test_exchange_known_answer(orc):
    """gtest_mpp_exchange_writer.cpp:663-718: 64 blocks x keys 0..63, 4 partitions -> 1024 rows each."""
    case = _load("reference_cases.json")["exchange"]
    keys = np.tile(np.arange(case["block_rows"], dtype=np.int64), case["blocks"])
    sel = orc.fill_selector(orc.weak_hash([keys]), case["parts"])
    counts = np.bincount(sel, minlength=case["parts"])
    assert counts.tolist() == [case["rows_per_part"]] * case["parts"]
    perm, offs = orc.partition(sel, case["parts"])
    assert np.all(np.diff(perm[offs[0]:offs[1]].astype(np.int64)) > 0)  # stable within a partition


def test_fine_grained_selector(orc):
    h = np.array([0, 1, 0xFFFFFFFF, 0x80000000, 12345], dtype=np.uint32)
    sel = orc.fill_selector(h, 4, 8)
    exp = [((int(x) * 4) >> 32) * 8 + int(x) % 8 for x in h]
    assert sel.tolist() == exp


def test_accurate_comparison_semantics(orc):
    # Int8(-1) != UInt8(255) (Core/AccurateComparison.h:27-29)
    a = np.array([-1], dtype=np.int8)
    b = np.array([255], dtype=np.uint8)
    assert orc.cmp(a, 0, b)[0] == 0 and orc.cmp(a, 2, b)[0] == 1
    # Int64 vs Float64 exactly (DecomposedFloat): 2^53+1 > 2^53
    x = np.array([2**53 + 1], dtype=np.int64)
    y = np.array([float(2**53)])
    assert orc.cmp(x, 4, y)[0] == 1 and orc.cmp(x, 0, y)[0] == 0
    # NaN: only != is true
    nan = np.array([np.nan])
    one = np.array([1], dtype=np.int64)
    assert [orc.cmp(nan, op, one)[0] for op in range(6)] == [0, 1, 0, 0, 0, 0]
    # UInt64 max vs Int64 -1
    u = np.array([2**64 - 1], dtype=np.uint64)
    assert orc.cmp(u, 4, np.array([-1], dtype=np.int64))[0] == 1


def test_filter_stable_and_count(orc):
    rng = np.random.default_rng(1)
    for n in (0, 1, 63, 64, 65, 1000):
        col = rng.integers(0, 1000, n, dtype=np.int64)
        f = rng.integers(0, 3, n).astype(np.uint8)
        out = orc.filter(col, f)
        np.testing.assert_array_equal(out, col[f != 0])
        assert orc.count_bytes_in_filter(f) == int((f != 0).sum())


def test_groupby_reference_cases(orc):
    for case in _load("reference_cases.json")["groupby"]:
        vals = case["column"]
        kn = np.array([v is None for v in vals], dtype=np.uint8)
        k = np.array([0 if v is None else v for v in vals], dtype=case["dtype"])
        a = orc.Agg(case["type"], [(2, 0)])
        a.consume(k, [None], key_null=kn)
        r = a.result()
        width = k.itemsize
        raw = r["keys"].astype({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[width]).view(case["dtype"])
        got = [None if r["key_null"][i] else int(raw[i]) for i in range(a.size())]
        assert sorted(got, key=repr) == sorted(case["expected"], key=repr), case["name"]


def golden_key_columns(case, cols):
    """numpy key columns (String: (chars, offsets)) + null maps of one groupby_keys case."""
    np_t = {1: np.int8, 2: np.int16, 3: np.int32, 4: np.int64, 8: np.uint64, 9: np.float32, 10: np.float64}
    keys, nulls, types = [], [], []
    for name in case["group_by"]:
        t, vals = cols[name]["type"], cols[name]["values"]
        nulls.append(np.array([v is None for v in vals], dtype=np.uint8))
        if t == 20:
            strs = [b"" if v is None else v.encode() for v in vals]
            keys.append((np.frombuffer(b"".join(x + b"\0" for x in strs), np.uint8).copy(),
                         np.cumsum([len(x) + 1 for x in strs]).astype(np.uint64)))
        else:
            keys.append(np.array([0 if v is None else v for v in vals], dtype=np_t[t]))
        types.append(t)
    exp = []
    for row in zip(*case["expected"]):
        k = []
        for t, v in zip(types, row):
            if v is None:
                k.append(None)
            elif t == 20:
                k.append(v.encode())
            elif t in (9, 10):
                k.append(float((np.float32 if t == 9 else np.float64)(v)))
            else:
                k.append(int(v))
        exp.append(tuple(k))
    return types, keys, nulls, exp


def test_groupby_keys_reference_cases(orc):
    """GroupBy string_ and two-column GROUP BYs (gtest_aggregation_executor.cpp:408-482)."""
    g = _load("reference_cases.json")["groupby_keys"]
    for case in g["cases"]:
        types, keys, nulls, exp = golden_key_columns(case, g["columns"])
        a = orc.AggKeys(types, [(2, 0)])
        a.consume(keys, [None], key_nulls=nulls)
        got = [k for k, _ in a.result()]
        assert sorted(got, key=repr) == sorted(exp, key=repr), case["group_by"]


def _join_rows(case, pi, bi):
    p, b = case["probe"], case["build"]
    rows = []
    for i, j in zip(pi.tolist(), bi.tolist()):
        row = [p["a"][i], p["b"][i]]
        if case["kind"] in ("inner", "left"):
            row += [None, None] if j == 0xFFFFFFFF else [b["a"][j], b["b"][j]]
        rows.append(tuple(row))
    return sorted(rows, key=repr)


def test_join_reference_cases(orc):
    kinds = {"inner": 0, "left": 1, "semi": 2, "anti": 3}
    for case in _load("reference_cases.json")["join"]:
        key = case["key"]
        bcol, pcol = case["build"][key], case["probe"][key]
        j = orc.JoinRef(orc.INT64)
        j.build(np.array([0 if v is None else v for v in bcol], dtype=np.int64),
                np.array([v is None for v in bcol], dtype=np.uint8))
        pi, bi = j.probe(np.array([0 if v is None else v for v in pcol], dtype=np.int64), kinds[case["kind"]],
                         np.array([v is None for v in pcol], dtype=np.uint8))
        exp = sorted(zip(*case["expected_columns"]), key=repr)
        assert _join_rows(case, pi, bi) == exp, case["name"]


def test_join_rowreflist_order(orc):
    """insertRowToList (JoinPartition.cpp:39-60): head first, then newest -> oldest."""
    j = orc.JoinRef(orc.INT64)
    j.build(np.array([7, 7, 7, 7], dtype=np.int64))
    pi, bi = j.probe(np.array([7], dtype=np.int64))
    assert bi.tolist() == [0, 3, 2, 1]


def test_decimal_arith(orc):
    # Decimal(10,2) 1.25 + Decimal(10,3) 0.125 -> scale 3: 1375 ; multiply -> scale 5
    a = np.array([125, -1], dtype=np.int64)
    b = np.array([125, 1000], dtype=np.int64)
    out = orc.arith(0, a, b, orc.DECIMAL64, a_type=orc.DECIMAL64, b_type=orc.DECIMAL64, a_scale=2, b_scale=3,
                    res_scale=3).view(np.int64)
    assert out.tolist() == [1375, 990]
    out = orc.arith(2, a, b, orc.DECIMAL128, a_type=orc.DECIMAL64, b_type=orc.DECIMAL64, a_scale=2, b_scale=3,
                    res_scale=5).view(np.int64).reshape(-1, 2)
    assert out[:, 0].tolist() == [15625, -1000] and out[:, 1].tolist() == [0, -1]


def test_bench_legs_run(orc):
    rng = np.random.default_rng(3)
    n = 100_000
    f = rng.integers(0, 100, n, dtype=np.int64)
    k = rng.integers(0, 1000, n, dtype=np.int64)
    v = rng.integers(0, 1 << 20, n).astype(np.float64) / 256
    g, cs = orc.bench_filter_agg(f, 96, k, v, 2, 4096)
    ref = orc.Agg(orc.INT64, [(0, orc.FLOAT64), (2, 0)])
    ref.consume(k, [v, None], mask=(f < 96).astype(np.uint8))
    r = ref.result()
    assert g == ref.size()
    assert cs == pytest.approx(float(r["states"][0].sum() + r["states"][1].sum()))
    m, _ = orc.bench_join(np.arange(1000, dtype=np.int64), rng.integers(0, 2000, 5000, dtype=np.int64), 2)
    assert 0 < m < 5000


@pytest.mark.parametrize("groups", [1000, 300_000])
def test_bench_ref_leg_matches_oracle(orc, groups):
    """cpu_baseline.c (the timed CPU leg) computes the same groups and sums as the restatement,
    below and above the two-level threshold (100k keys), including key 0."""
    rng = np.random.default_rng(4)
    n = 600_000
    f = rng.integers(0, 100, n, dtype=np.int64)
    k = rng.integers(0, groups, n, dtype=np.int64)
    v = rng.integers(0, 1 << 20, n).astype(np.float64) / 256
    ref = orc.Agg(orc.INT64, [(0, orc.FLOAT64), (2, 0)])
    ref.consume(k, [v, None], mask=(f < 96).astype(np.uint8))
    r = ref.result()
    for threads in (1, 3):
        g, cs = orc.bench_filter_agg_ref(f, 96, k, v, threads, 4096)
        assert g == ref.size()
        assert cs == pytest.approx(float(r["states"][0].sum() + r["states"][1].sum()), rel=1e-12)


def test_bench_join_ref_leg_matches_oracle(orc):
    """cpu_baseline.c's join leg finds the same matches as the restatement (duplicates, key 0)."""
    rng = np.random.default_rng(9)
    bk = rng.integers(0, 5000, 20_000, dtype=np.int64)
    bk[:5] = 0
    pk = rng.integers(0, 8000, 50_000, dtype=np.int64)
    jb = orc.JoinBench(bk, bk * 3, 3)
    m, _ = jb.probe(pk, pk)
    ref = orc.JoinRef(orc.INT64)
    ref.build(bk)
    pi, _ = ref.probe(pk)
    assert m == len(pi)


def _str_col(strs):
    chars = np.frombuffer(b"".join(s.encode() + b"\0" for s in strs), dtype=np.uint8).copy()
    return chars, np.cumsum([len(s) + 1 for s in strs]).astype(np.uint64)


def test_aggregate_value_reference_cases(orc):
    """Aggregate VALUES pinned by the reference's tests: AggregationCount over the clerk table
    (gtest_aggregation_executor.cpp:562-585; count(x) skips NULL x) and sum(s2) = 6 (:755-757)."""
    case = _load("reference_cases.json")["aggregates"]
    clerk = case["clerk"]
    n = len(clerk["age"])
    age = np.array([0 if a is None else a for a in clerk["age"]], dtype=np.int32)
    age_null = np.array([a is None for a in clerk["age"]], dtype=np.uint8)
    pr = np.array(clerk["pr"], dtype=np.uint64)
    country = _str_col(clerk["country"])
    for c in case["counts"]:
        if len(c["group_by"]) > 1:
            continue  # (country, gender): two String keys, the serialized method (GPU tests)
        kind, arg, nulls = {"count(age)": (1, age, age_null), "count(1)": (2, None, None),
                            "count(pr)": (1, pr, None)}[c["func"]]
        if c["group_by"]:
            a = orc.AggKeys([orc.STRING], [(kind, orc.type_of(arg) if arg is not None else 0)])
            a.consume([country], [arg], arg_nulls=[nulls] if nulls is not None else None)
            got = sorted(v[0] for _, v in a.result())
        else:
            a = orc.Agg(0, [(kind, 0)])
            a.consume(None, [arg], n=n)
            got = [int(x) for x in a.result()["states"][0]]
        assert got == sorted(c["expected"]), c
    s2 = np.array(case["test_table"]["s2"], dtype=np.int64)
    a = orc.Agg(0, [(0, orc.INT64)])
    a.consume(None, [s2], n=len(s2))
    assert int(a.result()["states"][0][0]) == case["sums"][0]["expected"][0]


def test_sum_result_types(orc):
    """SumDecimalInferer: Decimal(min(p+22, 65), s) (Common/Decimal.h:156-163); Decimal256 above 38."""
    case = _load("reference_cases.json")["sum_types"]
    for d in case["decimal"]:
        p = d["arg_prec"]
        t = orc.DECIMAL32 if p <= 9 else orc.DECIMAL64 if p <= 18 else orc.DECIMAL128 if p <= 38 else orc.DECIMAL256
        assert orc.sum_result_prec(orc.prec(t, p)) == d["result_prec"]
        assert orc.sum_limbs(0, orc.prec(t, p)) == (4 if d["result_prec"] > 38 else 2)
    assert orc.sum_result_prec(orc.DECIMAL64) == 40  # precision unknown: the type's maximum (18)
    assert case["decimal256_max_digits"] == 65 and 10**65 - 1 < 2**216  # |x| < 2^216: sums exact in 256 bits


def test_decimal256_sums_exact(orc):
    """Decimal256 accumulation (boost checked_int256_t) restated with 4 limbs = Python big ints."""
    rng = np.random.default_rng(3)
    n = 20000
    k = rng.integers(0, 50, n, dtype=np.int64)
    hi = rng.integers(2**61, 2**62, n, dtype=np.int64) * np.where(rng.random(n) < 0.7, 1, -1)
    d128 = np.stack([rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64), hi], axis=1)
    vals = [orc.limbs_to_int(r) for r in d128]
    big = [int(x) * 10**46 for x in rng.integers(-10**18, 10**18, n)]
    d256 = np.stack([orc.int_to_limbs(v, 4) for v in big])
    a = orc.Agg(orc.INT64, [(0, orc.DECIMAL128), (0, orc.prec(orc.DECIMAL256, 65)), (0, orc.prec(orc.DECIMAL64, 15))])
    d15 = rng.integers(-10**15 + 1, 10**15, n, dtype=np.int64)
    a.consume(k, [d128, d256, d15])
    r = a.result()
    exp = [{}, {}, {}]
    for i, key in enumerate(k.tolist()):
        for j, v in enumerate((vals[i], big[i], int(d15[i]))):
            exp[j][key] = exp[j].get(key, 0) + v
    keys = r["keys"].view(np.int64).tolist()
    assert r["states"][0].shape[1] == 4 and r["states"][1].shape[1] == 4 and r["states"][2].shape[1] == 2
    for j in range(3):
        assert dict(zip(keys, [orc.limbs_to_int(x) for x in r["states"][j]])) == exp[j]
    assert max(abs(v) for v in exp[0].values()) >= 2**127


def _float_golden(kind):
    g = _load("float_weak_hash.json")[kind]
    dt, ut = (np.float64, np.uint64) if kind == "float64" else (np.float32, np.uint32)
    vals = np.array([int(e["bits"], 16) for e in g], dtype=ut).view(dt)
    conv = np.array([int(e["u64"], 16) for e in g], dtype=np.uint64)
    hashes = np.array([e["hash"] for e in g], dtype=np.uint32)
    return vals, conv, hashes


@pytest.mark.parametrize("kind", ["float64", "float32"])
def test_float_weak_hash_golden(orc, kind):
    """Float keys hash as intHashCRC32(UInt64(x)) with the reference build's x86-64 conversion
    (NaN / +-inf / out of range -> 0x8000000000000000, negatives wrap), pinned by the fixture
    tests/golden/make_float_hash.cpp generated with clang on x86-64."""
    import ctypes
    vals, conv, hashes = _float_golden(kind)
    f = orc.lib().orc_float64_to_u64 if kind == "float64" else orc.lib().orc_float32_to_u64
    f.restype = ctypes.c_uint64
    f.argtypes = [ctypes.c_double if kind == "float64" else ctypes.c_float]
    assert [f(float(x)) for x in vals] == [int(c) for c in conv]
    h = orc.weak_hash([vals], [orc.FLOAT64 if kind == "float64" else orc.FLOAT32])
    np.testing.assert_array_equal(h, hashes)


@pytest.mark.parametrize("name,collator", [("general_ci", 3), ("unicode_ci", 4), ("uca0900_ai_ci", 5)])
def test_oracle_ci_sort_keys_match_reference_gtest(orc, name, collator):
    """utf8mb4_general_ci / utf8mb4_unicode_ci / utf8mb4_0900_ai_ci sort keys and comparisons: the
    reference's collator gtest answers (gtest_tidb_collator.cpp:49-65, 71-140;
    tests/golden/reference_cases.json).  UCA comparisons walk the same 16-bit weights the sort key
    holds (Collator.cpp:526-578), so the key order is the comparison's sign."""
    import ctypes
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_cases.json")))[name]
    lib = orc.lib()
    lib.orc_collate.restype = ctypes.c_size_t

    def key(s):
        b = s.encode("utf-8")
        out = ctypes.create_string_buffer(8 * len(b) + 16)
        n = lib.orc_collate(collator, b, ctypes.c_size_t(len(b)), ctypes.c_size_t(len(b) + 1), out)
        return out.raw[:n]

    for c in gold["sort_keys"]:
        assert key(c["s"]).hex() == c["key_hex"], c
    for c in gold["compare"]:
        ka, kb = key(c["a"]), key(c["b"])
        assert (ka > kb) - (ka < kb) == c["sign"], c


def test_oracle_uca_special_weights(orc):
    """UCA weight rules beyond the table lookup (Collator.cpp:703-727, 791-816): zero-weight
    characters vanish from the key, long weights (weightLutLongMap) emit both words, code points
    past the tables take 0xFFFD (4.0.0) or the implicit 9.0.0 weight."""
    import ctypes
    lib = orc.lib()
    lib.orc_collate.restype = ctypes.c_size_t

    def key(s, c):
        b = s.encode("utf-8")
        out = ctypes.create_string_buffer(8 * len(b) + 16)
        n = lib.orc_collate(c, b, ctypes.c_size_t(len(b)), ctypes.c_size_t(len(b) + 1), out)
        return out.raw[:n]

    for c in (4, 5):
        assert key("a\x01b", c) == key("ab", c)               # U+0001 weighs nothing
        assert len(key("\u321d", c)) > 8                       # a long weight: first and second words
        assert key("\u321d", c) != key("\u321e", c)
    assert key("\U00030000", 4) == bytes.fromhex("fffd")
    r = 0x30000
    w = (r >> 15) + 0xFBC0 + (((r & 0x7FFF) | 0x8000) << 16)
    assert key("\U00030000", 5) == bytes.fromhex("%04x%04x" % (w & 0xFFFF, w >> 16))


def test_oracle_decimal_wide_rules(orc):
    D128, D256, D64, I64 = 13, 14, 12, 4
    """The oracle's rules on hand-derived values (CPU-side restatement checks)."""
    assert orc.arith_decimal_wide(2, [-7], [3], D128, D128, 16, 16, D128, 30) == [0]      # -21 / 100 -> 0
    assert orc.arith_decimal_wide(2, [-700], [3], D128, D128, 16, 16, D128, 30) == [-21]  # truncation toward 0
    assert orc.arith_decimal_wide(0, [1], [2], D64, D256, 2, 0, D256, 2) == [201]
    with pytest.raises(OverflowError):
        orc.arith_decimal_wide(0, [10 ** 65 - 1], [1], D256, I64, 0, 0, D256, 0)
    # no Decimal256 operand: only the Int256 range applies (10^65 + x is representable)
    assert orc.arith_decimal_wide(0, [10 ** 38 - 1], [1], D128, D128, 0, 38, D256, 38) == [(10 ** 38 - 1) * 10 ** 38 + 1]
