"""CPU tests of the oracle's min / max / first_row over Decimal128 / Decimal256 / String (SURVEY §8
a15), pinned by the reference's own answers: the AggNull String max and the AggKeyOptimization
String first_row cases (gtest_aggregation_executor.cpp:740-750, 1160-1245), and the collators'
compare() signs (gtest_tidb_collator.cpp:71-140) that the String compare restates.

Reference semantics restated by the oracle (oracle.c ord_offer / ord_merge): SingleValueDataString
::less / greater compare the rows WITH their terminating zero (AggregateFunctionMinMaxAny.h:218-230,
getDataAtWithTerminatingZero), first_row keeps the first row even when it is NULL
(AggregateFunctionNull.h:193-330), min / max are strict (equal values keep the first)."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
COLL = {"none": 0, "binary": 1, "bin_padding": 2, "general_ci": 3, "unicode_ci": 4, "uca0900_ai_ci": 5}


def _cases():
    with open(os.path.join(GOLD, "reference_cases.json")) as f:
        return json.load(f)


def str_col(vals):
    """(chars, end offsets) of a ColumnString; None rows are empty (their null map says NULL)"""
    bs = [(v or "").encode() + b"\0" for v in vals]
    chars = np.frombuffer(b"".join(bs), dtype=np.uint8).copy() if bs else np.zeros(0, np.uint8)
    offs = np.cumsum([len(b) for b in bs]).astype(np.uint64)
    return chars, offs


def _cmp(orc, coll, a: bytes, b: bytes) -> int:
    return orc.lib().orc_min_max_str_compare(coll, a, len(a), b, len(b))


@pytest.mark.parametrize("name,coll", [("general_ci", 3), ("unicode_ci", 4), ("uca0900_ai_ci", 5)])
def test_string_compare_restates_reference_collator_compare(orc, name, coll):
    """the oracle's compare() restatement (used for min / max) reproduces the reference collator
    gtest's compare signs on the bare strings"""
    for c in _cases()[name]["compare"]:
        assert _cmp(orc, coll, c["a"].encode(), c["b"].encode()) == c["sign"], (name, c)


def test_string_compare_with_terminator(orc):
    """with the '\\0' each ColumnString row ends in, padding collators no longer trim: "a" < "a "
    under utf8_general_ci / utf8mb4_bin (equal on the bare strings)"""
    for coll in (2, 3, 4):
        assert _cmp(orc, coll, b"a", b"a ") == 0
        assert _cmp(orc, coll, b"a\0", b"a \0") == -1
    assert _cmp(orc, 3, b"A\0", b"a\0") == 0
    assert _cmp(orc, 0, b"A\0", b"a\0") == -1


def test_agg_null_max_string(orc):
    """AggNull: max(s1) without key over Nullable(String) {"banana", NULL, "banana"} = "banana";
    GROUP BY s1 -> {NULL, "banana"}"""
    c = _cases()["aggregates"]["agg_null"]
    chars, offs = str_col(c["s1"])
    nulls = np.array([v is None for v in c["s1"]], np.uint8)
    a = orc.Agg(0, [(orc.AGG_MAX, orc.STRING | orc.NULLABLE)])
    a.consume(None, [(chars, offs)], arg_nulls=[nulls], n=len(c["s1"]))
    r = a.result()
    ch, of = r["states"][0]
    assert r["state_null"][0][0] == 0 and bytes(ch[:int(of[0]) - 1]).decode() == c["max_s1"]
    k = orc.AggKeys([orc.STRING], [(orc.AGG_COUNT_ALL, 0)])
    k.consume([(chars, offs)], [None], key_nulls=[nulls])
    got = sorted((g[0][0] for g in k.result()), key=lambda v: (v is not None, v))
    assert [None if v is None else v.decode() for v in got] == c["group_by_s1"]


def test_first_row_string_reference_cases(orc):
    """AggKeyOptimization cases 3, 4, 6, 7: count(1), first_row(String) GROUP BY the case's keys"""
    c = _cases()["aggregates"]["first_row_string"]
    per = c["rows"] // c["row_types"]
    vals = [v for v in c["values"] for _ in range(per)]
    col_int = np.repeat(np.arange(c["row_types"], dtype=np.int32), per)
    strs = str_col(vals)
    cols = {"col_string_with_collator": (orc.STRING, strs, 3), "col_string_no_collator": (orc.STRING, strs, 0),
            "col_int": (orc.INT32, col_int, 0)}
    for case in c["cases"]:
        kt = [cols[k][0] for k in case["keys"]]
        kc = [cols[k][2] for k in case["keys"]]
        arg_coll = cols[case["arg"]][2]
        k = orc.AggKeys(kt, [(orc.AGG_COUNT_ALL, 0), (orc.AGG_FIRST_ROW, orc.STRING | (arg_coll << 24))],
                        collators=kc)
        k.consume([cols[x][1] for x in case["keys"]], [None, strs])
        res = sorted(k.result(), key=lambda g: g[1][1])
        assert [g[1][0] for g in res] == c["count"], case
        assert [g[1][1].decode() for g in res] == c["expected"], case


def _py_groups(keys, vals, nulls, kind, cmp=None):
    """reference semantics in pure Python: per group the first / min / max value in row order"""
    out = {}
    for k, v, n in zip(keys, vals, nulls):
        k = int(k)
        if kind == "first":
            out.setdefault(k, None if n else v)
            continue
        if n:
            out.setdefault(k, None)
            continue
        cur = out.get(k)
        if cur is None or (cmp(v, cur) < 0 if kind == "min" else cmp(v, cur) > 0):
            out[k] = v
    return out


def _limbs(xs, limbs):
    return np.array([[(x >> (64 * j)) & ((1 << 64) - 1) for j in range(limbs)] for x in xs], dtype=np.uint64).view(np.int64)


def _from_limbs(row):
    v = sum(int(x) << (64 * j) for j, x in enumerate(np.asarray(row).view(np.uint64)))
    return v - (1 << (64 * len(row))) if v >> (64 * len(row) - 1) else v


@pytest.mark.parametrize("t,limbs", [(13, 2), (14, 4)])
def test_decimal_min_max_first_vs_python(orc, t, limbs):
    rng = np.random.default_rng(t)
    n, groups = 4000, 300
    keys = rng.integers(0, groups, n).astype(np.int64)
    span = 1 << (120 if limbs == 2 else 250)
    vals = [int(x) for x in rng.integers(-1000, 1000, n)]
    vals = [v * (span // 1000) + int(rng.integers(0, 1 << 40)) for v in vals]
    nulls = (rng.random(n) < 0.2).astype(np.uint8)
    col = _limbs(vals, limbs)
    for kind, name in ((orc.AGG_MIN, "min"), (orc.AGG_MAX, "max"), (orc.AGG_FIRST_ROW, "first")):
        a = orc.Agg(orc.INT64, [(kind, t | orc.NULLABLE)])
        a.consume(keys, [col], arg_nulls=[nulls])
        r = a.result()
        got = {int(k): (None if r["state_null"][0][i] else _from_limbs(r["states"][0][i])) for i, k in enumerate(r["keys"].view(np.int64))}
        exp = _py_groups(keys, vals, nulls, name, lambda x, y: (x > y) - (x < y))
        assert got == exp, name


def test_string_min_max_first_vs_python(orc):
    rng = np.random.default_rng(5)
    n, groups = 3000, 200
    keys = rng.integers(0, groups, n).astype(np.int64)
    alphabet = ["a", "A", "b", " ", "é", "ß", "ss", "z"]
    vals = ["".join(rng.choice(alphabet, int(rng.integers(0, 5)))) for _ in range(n)]
    nulls = (rng.random(n) < 0.15).astype(np.uint8)
    col = str_col(vals)
    for coll in (0, 2, 3, 4, 5):
        cmp = lambda x, y: _cmp(orc, coll, x.encode() + b"\0", y.encode() + b"\0")  # noqa: E731
        for kind, name in ((orc.AGG_MIN, "min"), (orc.AGG_MAX, "max"), (orc.AGG_FIRST_ROW, "first")):
            a = orc.Agg(orc.INT64, [(kind, orc.STRING | orc.NULLABLE | (coll << 24))])
            a.consume(keys, [col], arg_nulls=[nulls])
            r = a.result()
            ch, of = r["states"][0]
            got = {}
            for i, k in enumerate(r["keys"].view(np.int64)):
                s = int(of[i - 1]) if i else 0
                got[int(k)] = None if r["state_null"][0][i] else bytes(ch[s:int(of[i]) - 1]).decode()
            assert got == _py_groups(keys, vals, nulls, name, cmp), (coll, name)


def test_first_row_null_first_and_merge(orc):
    """a NULL first row makes first_row NULL (later rows do not replace it); merge keeps dst's"""
    keys = np.array([1, 1, 2, 2, 3], np.int64)
    x = np.array([0, 5, 7, 8, 9], np.int64)
    nul = np.array([1, 0, 0, 0, 1], np.uint8)
    a = orc.Agg(orc.INT64, [(orc.AGG_FIRST_ROW, orc.INT64 | orc.NULLABLE)])
    a.consume(keys, [x], arg_nulls=[nul])
    r = a.result()
    got = {int(k): (None if r["state_null"][0][i] else int(r["states"][0][i])) for i, k in enumerate(r["keys"].view(np.int64))}
    assert got == {1: None, 2: 7, 3: None}
    b = orc.Agg(orc.INT64, [(orc.AGG_FIRST_ROW, orc.INT64 | orc.NULLABLE)])
    b.consume(np.array([1, 2, 4], np.int64), [np.array([11, 12, 14], np.int64)], arg_nulls=[np.zeros(3, np.uint8)])
    a.merge(b)
    r = a.result()
    got = {int(k): (None if r["state_null"][0][i] else int(r["states"][0][i])) for i, k in enumerate(r["keys"].view(np.int64))}
    assert got == {1: None, 2: 7, 3: None, 4: 14}


def test_min_max_without_key_empty_is_default(orc):
    """SingleValueDataFixed::insertResultInto without a value: insertDefault (0), not NULL, for a
    non-Nullable argument; first_row is NULL"""
    a = orc.Agg(0, [(orc.AGG_MIN, orc.INT64), (orc.AGG_MAX, orc.FLOAT64), (orc.AGG_FIRST_ROW, orc.INT32)])
    a.consume(None, [np.zeros(1, np.int64), np.zeros(1, np.float64), np.zeros(1, np.int32)],
              mask=np.zeros(1, np.uint8), n=1)
    r = a.result()
    assert r["states"][0][0] == 0 and r["states"][1][0] == 0.0
    assert r["state_null"][2][0] == 1
