"""Generates the committed golden fixtures in tests/golden/.

reference_cases.json — known answers TRANSCRIBED (as data) from the reference's own gtests:
  * groupby: dbms/src/Flash/tests/gtest_aggregation_executor.cpp:269-272 (columns) and :344-368
    (expected GROUP BY key sets for tinyint_/smallint_/int_/bigint_);
  * groupby_keys: the same file, :261-270 (columns incl. float_, double_, date_, datetime_ (MyDate /
    MyDateTime are packed UInt64), string_) with the expected key sets of GROUP BY string_
    (:408-415) and of the two-column GROUP BYs (:433-482);
  * join: dbms/src/Flash/tests/gtest_join_executor.cpp:114-200 (SimpleJoin tables t1/t2 and the
    expected inner / left / semi / anti results).  The reference keys are strings "1".."4"; join
    equality is unchanged when they are written as the integers 1..4, which is how they are stored;
  * exchange: dbms/src/Flash/Mpp/tests/gtest_mpp_exchange_writer.cpp:663-718 (64 blocks of keys
    0..63, 4 partitions -> 1024 rows each);
  * aggregates: aggregate VALUES the reference's tests pin — the clerk table
    (gtest_aggregation_executor.cpp:272-290) with AggregationCount's expected count columns
    (:562-585), test_table (:102-106) with RepeatedAggregateFunction's sum(s2) = 6 (:755-757);
  * sum_types: result types of sum — integer inputs per gtest_sum_int_agg_func.cpp:88-99
    (ReturnTypeForIntegerInputs), Decimal inputs per SumDecimalInferer (Common/Decimal.h:156-163,
    Decimal(min(p+22, 65), s)), the Decimal256 bound of 65 digits (gtest_decimal_type.cpp:52-62) and
    the +/-/* result scales of DataTypeDecimal_test A (gtest_funtions_decimal_arith.cpp:47-77).
  * general_ci: utf8mb4_general_ci sort keys and comparisons pinned by the reference's collator
    gtest (dbms/src/TiDB/tests/gtest_tidb_collator.cpp:49-65 cmp_cases and :71-140 sk_cases, the
    GeneralCI column of each answer tuple), as hex bytes;
  * unicode_ci / uca0900_ai_ci: the same for utf8mb4_unicode_ci and utf8mb4_0900_ai_ci (the
    UnicodeCI and Utf8Mb40900AICI columns).
crc_vectors.json — CRC32-C / WeakHash32 vectors computed with the x86 SSE4.2 crc32q instruction,
  the instruction the reference itself hashes with (Common/HashTable/Hash.h:70-95), via oracle.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

N = None
T1 = {"a": [1, 2, N, 1, N], "b": [3, 4, 3, N, N]}
T2 = {"a": [1, 3, N, 1, N], "b": [3, 4, 3, N, N]}


def join_cases():
    # (left, right, key) in the order of gtest_join_executor.cpp:126-131
    combos = [("t1", "t2", "a"), ("t2", "t1", "a"), ("t1", "t2", "b"), ("t2", "t1", "b")]
    inner = [
        [[1, 1, 1, 1], [N, 3, N, 3], [1, 1, 1, 1], [3, 3, N, N]],
        [[1, 1, 1, 1], [N, 3, N, 3], [1, 1, 1, 1], [3, 3, N, N]],
        [[N, 1, 2, N, 1], [3, 3, 4, 3, 3], [1, 1, 3, N, N], [3, 3, 4, 3, 3]],
        [[N, 1, 3, N, 1], [3, 3, 4, 3, 3], [1, 1, 2, N, N], [3, 3, 4, 3, 3]],
    ]
    left = [
        [[1, 1, 2, N, 1, 1, N], [3, 3, 4, 3, N, N, N], [1, 1, N, N, 1, 1, N], [N, 3, N, N, N, 3, N]],
        [[1, 1, 3, N, 1, 1, N], [3, 3, 4, 3, N, N, N], [1, 1, N, N, 1, 1, N], [N, 3, N, N, N, 3, N]],
        [[1, 1, 2, N, N, 1, N], [3, 3, 4, 3, 3, N, N], [N, 1, 3, N, 1, N, N], [3, 3, 4, 3, 3, N, N]],
        [[1, 1, 3, N, N, 1, N], [3, 3, 4, 3, 3, N, N], [N, 1, 2, N, 1, N, N], [3, 3, 4, 3, 3, N, N]],
    ]
    semi = [[[1, 1], [3, N]], [[1, 1], [3, N]], [[1, 2, N], [3, 4, 3]], [[1, 3, N], [3, 4, 3]]]
    anti = [[[2, N, N], [4, 3, N]], [[3, N, N], [4, 3, N]], [[1, N], [N, N]], [[1, N], [N, N]]]
    tables = {"t1": T1, "t2": T2}
    out = []
    for i, (l, r, key) in enumerate(combos):
        for kind, exp in (("inner", inner[i]), ("left", left[i]), ("semi", semi[i]), ("anti", anti[i])):
            out.append({"name": f"SimpleJoin {kind} {l} {r} on {key}", "kind": kind, "probe": tables[l],
                        "build": tables[r], "key": key, "expected_columns": exp})
    return out


def groupby_cases():
    cols = {  # gtest_aggregation_executor.cpp:269-272
        "tinyint_": ([1, 2, 3, N, N, 0, 0, -1, -2], 1, "int8", [-1, 2, N, 0, 1, 3, -2]),
        "smallint_": ([2, 3, N, N, 0, -1, -2, 4, 0], 2, "int16", [-1, 2, -2, N, 0, 4, 3]),
        "int_": ([4, N, N, 0, 123, -1, -1, 123, 4], 3, "int32", [-1, N, 4, 0, 123]),
        "bigint_": ([2, 2, N, 0, -1, N, -1, 0, 123], 4, "int64", [2, -1, 0, 123, N]),
    }
    return [{"name": k, "column": v[0], "type": v[1], "dtype": v[2], "expected": v[3]} for k, v in cols.items()]


def groupby_keys_cases():
    # gtest_aggregation_executor.cpp:261-270; type codes of include/tiflash_amd.h (MyDate /
    # MyDateTime = UInt64 8, Float32 9, Float64 10, String 20)
    cols = {
        "tinyint_": (1, [1, 2, 3, N, N, 0, 0, -1, -2]),
        "smallint_": (2, [2, 3, N, N, 0, -1, -2, 4, 0]),
        "int_": (3, [4, N, N, 0, 123, -1, -1, 123, 4]),
        "bigint_": (4, [2, 2, N, 0, -1, N, -1, 0, 123]),
        "float_": (9, [3.3, N, 0, 4.0, 3.3, 5.6, -0.1, -0.1, N]),
        "double_": (10, [0.1, 0, 1.1, 1.1, 1.2, N, N, -1.2, -1.2]),
        "date_": (8, [1000000, 2000000, N, 300000, 1000000, N, 0, 2000000, N]),
        "datetime_": (8, [2000000, 0, N, 3000000, 1000000, N, 0, 2000000, 1000000]),
        "string_": (20, [N, "pingcap", "PingCAP", N, "PINGCAP", "PingCAP", N, "Shanghai", "Shanghai"]),
    }
    expected = [  # (group by columns, expected columns) :408-415, :433-482
        (["string_"], [[N, "pingcap", "PingCAP", "PINGCAP", "Shanghai"]]),
        (["tinyint_", "float_"], [[1, 2, N, 3, 0, 0, -1, N, -2], [3.3, N, 4, 0, -0.1, 5.6, -0.1, 3.3, N]]),
        (["smallint_", "datetime_"], [[2, 3, N, N, 0, -1, -2, 4], [2000000, 0, N, 3000000, 1000000, N, 0, 2000000]]),
        (["int_", "double_"], [[N, 123, -1, 0, N, 4, 4, 123], [0, -1.2, N, 1.1, 1.1, -1.2, 0.1, 1.2]]),
        (["bigint_", "string_"], [[-1, 0, 0, 123, 2, N, -1, 2], [N, N, "Shanghai", "Shanghai", N, "PingCAP", "PINGCAP", "pingcap"]]),
        (["date_", "datetime_"], [[1000000, 2000000, N, 300000, 1000000, 0, 2000000, N],
                                  [2000000, 0, N, 3000000, 1000000, 0, 2000000, 1000000]]),
        (["datetime_", "string_"], [[2000000, 0, N, 3000000, 1000000, 0, 2000000, 1000000],
                                    [N, "pingcap", "PingCAP", N, "PINGCAP", N, "Shanghai", "Shanghai"]]),
    ]
    return {"columns": {k: {"type": t, "values": v} for k, (t, v) in cols.items()},
            "cases": [{"group_by": g, "expected": e} for g, e in expected]}


def aggregate_cases():
    clerk = {  # gtest_aggregation_executor.cpp:272-290
        "age": [30, N, 27, 32, 25, 36, N, 22, 34],
        "gender": ["male", "female", "female", "male", "female", "female", "male", "female", "male"],
        "country": ["russia", "korea", "usa", "usa", "usa", "china", "china", "china", "china"],
        "salary": [1000.1, 1300.2, 0.3, N, -200.4, 900.5, -999.6, 2000.7, -300.8],
        "pr": [1, 2, 0, 3290124, 968933, 3125, 31236, 4327, 80000],
    }
    counts = [  # AggregationCount (:562-585): expected count columns, in unspecified group order
        {"func": "count(age)", "group_by": ["country"], "expected": [3, 3, 1, 0]},
        {"func": "count(gender)", "group_by": ["country", "gender"], "expected": [2, 2, 2, 1, 1, 1]},
        {"func": "count(1)", "group_by": [], "expected": [9]},
        {"func": "count(1)", "group_by": ["country"], "expected": [4, 3, 1, 1]},
        {"func": "count(pr)", "group_by": ["country"], "expected": [4, 3, 1, 1]},
    ]
    test_table = {"s1": [1, 2, 3], "s2": [1, 2, 3]}  # :102-106
    # AggregationMaxAndMin (:503-545): max / min of a nullable column per group, expected values in
    # unspecified group order (N = a group whose values are all NULL)
    min_max = [
        {"func": "max(age)", "group_by": ["country"], "expected": [36, 32, 30, N]},
        {"func": "max(salary)", "group_by": ["country", "gender"], "expected": [2000.7, 1300.2, 1000.1, 0.3, -300.8, N]},
        {"func": "min(age)", "group_by": ["country"], "expected": [30, 25, 22, N]},
        {"func": "min(salary)", "group_by": ["country", "gender"], "expected": [1300.2, 1000.1, 900.5, -200.4, -999.6, N]},
    ]
    # AggKeyOptimization case 1 (:1053-1137): 1024 rows, four groups of 256 rows (col_int = i,
    # col_tinyint = i): count(1), first_row(col_tinyint) GROUP BY col_int, col_tinyint
    first_row = {"rows": 1024, "row_types": 4, "count": [256, 256, 256, 256], "first_row_tinyint": [0, 1, 2, 3]}
    # AggNull (:740-750, table aggnull_test.t1 :98-101): max(s1) without key over Nullable(String)
    # s1 = {"banana", NULL, "banana"} -> {"banana"}; GROUP BY s1 -> s1 = {NULL, "banana"}
    agg_null = {"s1": ["banana", N, "banana"], "s2": ["apple", N, "banana"], "max_s1": "banana",
                "group_by_s1": [N, "banana"]}
    # AggKeyOptimization cases 3, 4, 6, 7 (:1160-1245): 1024 rows in four runs of 256 ("a", 0), ("b", 1),
    # ("c", 2), ("d", 3) of (col_string_*, col_int); count(1) and first_row(String column) GROUP BY the
    # listed keys -> counts 256 and first_row = "a".."d"; col_string_with_collator is utf8_general_ci
    first_row_string = {
        "rows": 1024, "row_types": 4, "values": ["a", "b", "c", "d"], "count": [256, 256, 256, 256],
        "cases": [{"case": 3, "keys": ["col_string_no_collator"], "arg": "col_string_no_collator"},
                  {"case": 4, "keys": ["col_string_with_collator"], "arg": "col_string_with_collator"},
                  {"case": 6, "keys": ["col_string_with_collator", "col_int", "col_string_no_collator"],
                   "arg": "col_string_with_collator"},
                  {"case": 7, "keys": ["col_string_with_collator", "col_int"], "arg": "col_string_with_collator"}],
        "collators": {"col_string_with_collator": "utf8_general_ci", "col_string_no_collator": None},
        "expected": ["a", "b", "c", "d"]}
    # RepeatedAggregateFunction (:752-770): max(s1) = 3, min(s1) = 1 without key over test_table
    repeated = {"max_s1": 3, "min_s1": 1, "sum_s2": 6}
    return {"clerk": clerk, "counts": counts, "test_table": test_table,
            "sums": [{"func": "sum(s2)", "group_by": [], "expected": [6]}],  # :755-757
            "min_max": min_max, "first_row": first_row, "agg_null": agg_null, "first_row_string": first_row_string,
            "repeated": repeated}


def sum_type_cases():
    ints = [  # gtest_sum_int_agg_func.cpp:88-99 (tfg type codes of include/tiflash_amd.h)
        (1, "Int64"), (2, "Int64"), (3, "Int64"), (4, "Int64"),
        (5, "UInt64"), (6, "UInt64"), (7, "UInt64"), (8, "UInt64"),
    ]
    decimals = [{"arg_prec": p, "result_prec": min(p + 22, 65)} for p in (1, 9, 10, 15, 16, 17, 18, 19, 38, 43, 65)]
    return {"int": [{"arg_type": t, "result": r} for t, r in ints], "decimal": decimals,
            "decimal256_max_digits": 65,  # gtest_decimal_type.cpp:52-62: 65 nines parse, 66 digits do not
            "arith_scales": {"lhs": [10, 4], "rhs": [10, 6], "plus": 6, "minus": 6, "multiply": 10}}


def general_ci_cases():
    # (input, expected sort key) — the GeneralCI entry (index 2) of sk_cases
    sk = [("a", "0041"), ("A", "0041"), ("\U0001F603", "fffd"),
          ("Foo \u00a9 bar \U0001D306 baz \u2603 qux",
           "0046004f004f002000a900200042004100520020fffd00200042004100" "5a0020260300200051005500" "58"),
          ("a ", "0041"), ("", ""), ("\u00df", "0053")]
    # (a, b, expected sign of compare) — the GeneralCI entry of cmp_cases
    cmp = [("a", "b", -1), ("a", "A", 0), ("\u00c0", "A", 0), ("abc", "abc", 0), ("abc", "ab", 1),
           ("\U0001F61C", "\U0001F603", 0), ("a", "a ", 0), ("a ", "a  ", 0), ("a\t", "a", 1), ("", "a", -1),
           ("a", "", 1), ("\u00df", "ss", -1), ("\U0001042D", "\U00010428", 0), ("\u8b3a", "\u8b42", -1)]
    return {"sort_keys": [{"s": a, "key_hex": k} for a, k in sk],
            "compare": [{"a": a, "b": b, "sign": c} for a, b, c in cmp]}


def uca_cases():
    # the UnicodeCI (index 4: utf8mb4_unicode_ci, UCA 4.0.0, padding) and Utf8Mb40900AICI (index 5:
    # utf8mb4_0900_ai_ci, UCA 9.0.0, no padding) entries of sk_cases / cmp_cases
    # (gtest_tidb_collator.cpp:49-65, 71-140)
    foo = "Foo \u00a9 bar \U0001D306 baz \u2603 qux"
    sk = {
        "unicode_ci": [("a", "0e33"), ("A", "0e33"), ("\U0001F603", "fffd"),
                       (foo, "0eb90f820f82020902c502090e4a0e330fc00209fffd0209" "0e4a0e33" "106a020906ff02090fb4101f105a"),
                       ("a ", "0e33"), ("", ""), ("\u00df", "0fea0fea")],
        "uca0900_ai_ci": [("a", "1c47"), ("A", "1c47"), ("\U0001F603", "15fe"),
                          (foo, "1ce51ddd1ddd0209058402091c601c471e3302090ef00209" "1c601c47" "1f210209091b02091e211eb51eff"),
                          ("a ", "1c470209"), ("", ""), ("\u00df", "1e711e71")],
    }
    pairs = [("a", "b"), ("a", "A"), ("\u00c0", "A"), ("abc", "abc"), ("abc", "ab"), ("\U0001F61C", "\U0001F603"),
             ("a", "a "), ("a ", "a  "), ("a\t", "a"), ("", "a"), ("a", ""), ("\u00df", "ss"),
             ("\U0001042D", "\U00010428"), ("\u8b3a", "\u8b42")]
    signs = {"unicode_ci": [-1, 0, 0, 0, 1, 0, 0, 0, 1, -1, 1, 0, 0, -1],
             "uca0900_ai_ci": [-1, 0, 0, 0, 1, 1, -1, -1, 1, -1, 1, 0, 1, -1]}
    return {name: {"sort_keys": [{"s": a, "key_hex": k} for a, k in sk[name]],
                   "compare": [{"a": a, "b": b, "sign": c} for (a, b), c in zip(pairs, signs[name])]}
            for name in sk}


def crc_vectors():
    from oracle import oracle as orc
    rng = np.random.default_rng(2024)
    xs = [0, 1, 2**63, 2**64 - 1, 0x0123456789ABCDEF] + [int(x) for x in rng.integers(0, 2**63, 27, dtype=np.int64)]
    seeds = [0xFFFFFFFF, 0, 0x12345678]
    vec = [{"crc": s, "x": x, "out": orc.crc32c_u64(s, x)} for s in seeds for x in xs]
    keys = np.arange(64, dtype=np.int64)
    h = orc.weak_hash([keys])
    strs = [b"", b"a", b"abcdefg", b"abcdefgh", b"abcdefghi", b"k00000042", b"hello world  "]
    sh = [orc.lib().orc_update_weak_hash32_bytes(s, len(s), 0xFFFFFFFF) for s in strs]
    return {"crc32c_u64": vec, "weak_hash_int64_0_63": [int(x) for x in h],
            "selector_0_63_p4": [int(x) for x in orc.fill_selector(h, 4)],
            "weak_hash_bytes": [{"s": s.decode(), "h": int(v)} for s, v in zip(strs, sh)]}


if __name__ == "__main__":
    with open(os.path.join(HERE, "reference_cases.json"), "w") as f:
        json.dump({"groupby": groupby_cases(), "groupby_keys": groupby_keys_cases(), "join": join_cases(),
                   "exchange": {"block_rows": 64, "blocks": 64, "parts": 4, "rows_per_part": 1024},
                   # gtest_mpp_exchange_writer.cpp:391-450 (testBatchWriteFineGrainedShuffle) and
                   # :542-607 (testFineGrainedShuffleWriter): P = 4, S = 8, partition column 0
                   "fine_grained": {"parts": 4, "streams": 8,
                                    "batch": {"block_rows": 1024, "batch_size": 4096, "rows_per_chunk": 32},
                                    "blocks": {"block_rows": 64, "block_num": 64, "batch_size": 108,
                                               "rows_per_part": 1024, "rows_per_stream": 512}},
                   "aggregates": aggregate_cases(), "sum_types": sum_type_cases(),
                   "general_ci": general_ci_cases(), **uca_cases()}, f, indent=1)
    with open(os.path.join(HERE, "crc_vectors.json"), "w") as f:
        json.dump(crc_vectors(), f, indent=1)
    print("wrote", os.listdir(HERE))
