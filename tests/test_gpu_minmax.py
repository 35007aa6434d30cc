"""min / max / first_row on the device (TFG_AGG_MIN / MAX / FIRST_ROW) vs the oracle and the
reference's known answers.

Reference: AggregateFunctionMinMaxAny.cpp:39-46,155-159 (factory), AggregateFunctionMinMaxAny.h
(SingleValueDataFixed::changeIfLess / changeIfGreater / changeFirstTime), AggregateFunctionNull.h
(NULL arguments skipped; first_row keeps a NULL first row, AggregateFunctionFirstRowNull).
Known answers: gtest_aggregation_executor.cpp:503-545 (AggregationMaxAndMin over the clerk table)
and :1053-1137 (AggKeyOptimization: first_row of a GROUP BY column), transcribed into
tests/golden/reference_cases.json by tests/golden/make_golden.py.

min / max are exact: the device keeps the extreme value's order key.  first_row returns the
argument of SOME row of the group (the reference's "first" depends on thread and merge order), so
it is checked where every row of a group carries the same value — the reference's own
first_row-optimisation case — and otherwise for membership in the group's values."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
NP = {1: np.int8, 2: np.int16, 3: np.int32, 4: np.int64, 5: np.uint8, 6: np.uint16, 7: np.uint32, 8: np.uint64,
      9: np.float32, 10: np.float64, 11: np.int32, 12: np.int64}


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _by_key(keys, states, nulls):
    """{key: [value or None per aggregate]}"""
    out = {}
    for r, k in enumerate(keys):
        out[int(k)] = [None if (n is not None and n[r]) else s[r].item() for s, n in zip(states, nulls)]
    return out


def _dev_result(res, nullable, types=None):
    keys = res["keys"].cpu().numpy()
    states = [s.cpu().numpy() for s in res["states"]]
    if types:  # the argument's numpy type (UInt64 results come back in an int64 tensor)
        states = [s.view(NP[t & 0xFF]) for s, t in zip(states, types)]
    nulls = [res["state_null"][i].cpu().numpy() if nullable[i] else None for i in range(len(states))]
    return _by_key(keys, states, nulls)


def _orc_result(r, nullable):
    keys = r["keys"].view(np.int64)
    nulls = [r["state_null"][i] if nullable[i] else None for i in range(len(r["states"]))]
    return _by_key(keys, r["states"], nulls)


def _data(rng, n, groups, types, null_frac):
    k = rng.integers(-groups // 2, groups // 2, n).astype(np.int64)
    args, nulls = [], []
    for t in types:
        base = t & 0xFF
        dt = NP[base]
        if base in (9, 10):
            x = (rng.integers(-(1 << 20), 1 << 20, n) / 64.0).astype(dt)
            x[x == 0] = 1.0  # -0 / +0 ties are order-dependent in the reference
        elif np.issubdtype(dt, np.unsignedinteger):
            x = rng.integers(0, np.iinfo(dt).max, n, dtype=np.uint64, endpoint=True).astype(dt)
        else:
            info = np.iinfo(dt)
            x = rng.integers(info.min, info.max, n, dtype=np.int64, endpoint=True).astype(dt)
        args.append(x)
        nulls.append((rng.random(n) < null_frac).astype(np.uint8) if t & 0x100 else None)
    return k, args, nulls


TYPES = [3 | 0x100, 10, 4, 8, 9 | 0x100, 12, 1, 6]


@pytest.mark.parametrize("n,groups", [(200_000, 5_000), (3_000_000, 1_000_000)])
def test_min_max_vs_oracle(tfa, ctx, dev, orc, n, groups):
    rng = np.random.default_rng(n)
    kinds = [tfa.AGG_MIN, tfa.AGG_MAX, tfa.AGG_MIN, tfa.AGG_MAX, tfa.AGG_MAX, tfa.AGG_MIN, tfa.AGG_MAX, tfa.AGG_MIN]
    k, args, nulls = _data(rng, n, groups, TYPES, 0.3)
    nullable = [bool(t & 0x100) for t in TYPES]
    got, exp = {}, {}
    for lo in range(0, len(TYPES), 4):  # four aggregates per aggregator (AGG_MAX)
        sl = slice(lo, lo + 4)
        aggs = list(zip(kinds[sl], TYPES[sl]))
        agg = tfa.Aggregator(ctx, tfa.INT64, aggs)
        agg.consume(_t(k, dev), [_t(a, dev) for a in args[sl]],
                    arg_nullmaps=[_t(x, dev) if x is not None else None for x in nulls[sl]])
        g = _dev_result(agg.result(), nullable[sl], TYPES[sl])
        agg.close()
        ref = orc.Agg(orc.INT64, aggs)
        ref.consume(k, args[sl], arg_nulls=nulls[sl])
        e = _orc_result(ref.result(), nullable[sl])
        for key, v in g.items():
            got.setdefault(key, []).extend(v)
        for key, v in e.items():
            exp.setdefault(key, []).extend(v)
    assert len(got) == len(exp)
    assert got == exp


def test_min_max_without_key_and_all_null(tfa, ctx, dev, orc):
    rng = np.random.default_rng(3)
    n = 100_000
    x = rng.integers(-10**9, 10**9, n).astype(np.int64)
    f = (rng.integers(-10**6, 10**6, n) / 8.0).astype(np.float32)
    allnull = np.ones(n, dtype=np.uint8)
    aggs = [(tfa.AGG_MIN, tfa.INT64), (tfa.AGG_MAX, tfa.FLOAT32), (tfa.AGG_MAX, tfa.INT64 | tfa.NULLABLE),
            (tfa.AGG_FIRST_ROW, tfa.INT64 | tfa.NULLABLE)]
    agg = tfa.Aggregator(ctx, 0, aggs)
    agg.consume(None, [_t(x, dev), _t(f, dev), _t(x, dev), _t(x, dev)],
                arg_nullmaps=[None, None, _t(allnull, dev), _t(allnull, dev)])
    res = agg.result()
    agg.close()
    assert res["states"][0].item() == int(x.min())
    assert res["states"][1].item() == float(f.max())
    assert res["state_null"][2].item() == 1 and res["state_null"][3].item() == 1


def test_first_row_reference_key_optimisation(tfa, ctx, dev):
    """AggKeyOptimization case 1: count(1), first_row(col_tinyint) GROUP BY col_int, col_tinyint over
    four blocks of 256 equal rows -> counts 256 and first_row = the group's col_tinyint."""
    case = json.load(open(os.path.join(HERE, "golden", "reference_cases.json")))["aggregates"]["first_row"]
    rows, types = case["rows"], case["row_types"]
    col_int = np.repeat(np.arange(types, dtype=np.int32), rows // types)
    col_tiny = col_int.astype(np.int8)
    agg = tfa.KeysAggregator(ctx, [tfa.INT32, tfa.INT8], [(tfa.AGG_COUNT_ALL, 0), (tfa.AGG_FIRST_ROW, tfa.INT8)])
    agg.consume([_t(col_int, dev), _t(col_tiny, dev)], [None, _t(col_tiny, dev)])
    res = agg.result()
    got = sorted(zip(res["keys"][0].cpu().tolist(), res["states"][0].cpu().tolist(), res["states"][1].cpu().tolist()))
    assert [c for _, c, _ in got] == case["count"]
    assert [fr for _, _, fr in got] == case["first_row_tinyint"]
    assert all(k == fr for k, _, fr in got)


@pytest.mark.parametrize("n,groups", [(300_000, 20_000), (2_000_000, 600_000)])
def test_first_row_functionally_dependent(tfa, ctx, dev, n, groups):
    """first_row of columns that depend on the key only (one value per group, NULL-ness too) is
    unique whatever row is first; of a free column it must be one of the group's values."""
    rng = np.random.default_rng(groups)
    k = rng.integers(0, groups, n).astype(np.int64)
    dep = (k * 7919 % 100_003 - 50_000).astype(np.int32)
    depf = (k % 1000).astype(np.float64) / 4.0 + 0.5
    depn = (k % 5 == 0).astype(np.uint8)  # NULL for every row of every fifth group
    free = rng.integers(0, 1 << 30, n).astype(np.int64)
    aggs = [(tfa.AGG_FIRST_ROW, tfa.INT32), (tfa.AGG_FIRST_ROW, tfa.FLOAT64 | tfa.NULLABLE),
            (tfa.AGG_FIRST_ROW, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.Aggregator(ctx, tfa.INT64, aggs)
    agg.consume(_t(k, dev), [_t(dep, dev), _t(depf, dev), _t(free, dev), None],
                arg_nullmaps=[None, _t(depn, dev), None, None])
    res = agg.result()
    agg.close()
    keys = res["keys"].cpu().numpy()
    assert len(keys) == len(np.unique(k))
    np.testing.assert_array_equal(res["states"][0].cpu().numpy(), (keys * 7919 % 100_003 - 50_000).astype(np.int32))
    fn = res["state_null"][1].cpu().numpy()
    np.testing.assert_array_equal(fn, (keys % 5 == 0).astype(np.uint8))
    fv = res["states"][1].cpu().numpy()
    np.testing.assert_array_equal(fv[fn == 0], ((keys % 1000) / 4.0 + 0.5)[fn == 0])
    order = np.argsort(k, kind="stable")
    ks, fs = k[order], free[order]
    members = set(zip(ks.tolist(), fs.tolist()))
    assert all((int(a), int(b)) in members for a, b in zip(keys, res["states"][2].cpu().numpy()))


def test_min_max_two_phase_and_merge(tfa, ctx, dev, orc):
    """partial results -> consume_partial (two-phase final) and tfg_agg_merge = one aggregation."""
    rng = np.random.default_rng(11)
    n, groups = 400_000, 50_000
    types = [tfa.INT32 | tfa.NULLABLE, tfa.FLOAT64, tfa.UINT16]
    kinds = [tfa.AGG_MIN, tfa.AGG_MAX, tfa.AGG_MAX]
    k, args, nulls = _data(rng, n, groups, types, 0.5)
    aggs = list(zip(kinds, types))
    nullable = [True, False, False]
    half = n // 2
    parts = []
    for sl in (slice(0, half), slice(half, n)):
        a = tfa.Aggregator(ctx, tfa.INT64, aggs)
        a.consume(_t(k[sl], dev), [_t(x[sl], dev) for x in args],
                  arg_nullmaps=[_t(x[sl], dev) if x is not None else None for x in nulls])
        parts.append(a)
    ref = orc.Agg(orc.INT64, aggs)
    ref.consume(k, args, arg_nulls=nulls)
    exp = _orc_result(ref.result(), nullable)
    # two-phase: the partial result blocks into a final aggregator
    fin = tfa.Aggregator(ctx, tfa.INT64, aggs)
    for a in parts:
        r = a.result()
        fin.consume_partial(r["keys"], r["states"], state_nullmaps=r["state_null"])
    assert _dev_result(fin.result(), nullable, types) == exp
    fin.close()
    # merge of the two aggregators' states
    parts[0].merge(parts[1])
    assert _dev_result(parts[0].result(), nullable, types) == exp
    for a in parts:
        a.close()


def _clerk_groups(clerk, keys):
    """rows of the clerk table grouped by the key columns -> {key tuple: [row indices]}"""
    groups = {}
    for r in range(len(clerk["age"])):
        groups.setdefault(tuple(clerk[c][r] for c in keys), []).append(r)
    return groups


def _str_col(vals):
    b = b"".join(v.encode() + b"\0" for v in vals)
    chars = np.frombuffer(b, dtype=np.uint8).copy()
    offs = np.cumsum([len(v.encode()) + 1 for v in vals]).astype(np.int64)
    return chars, offs


def test_min_max_reference_clerk(tfa, ctx, dev):
    """AggregationMaxAndMin: max / min of age (Nullable Int32) GROUP BY country, of salary
    (Nullable Float64) GROUP BY country, gender — the expected columns in unspecified order."""
    agg_cases = json.load(open(os.path.join(HERE, "golden", "reference_cases.json")))["aggregates"]
    clerk = agg_cases["clerk"]
    for case in agg_cases["min_max"]:
        fn, col = case["func"].split("(")
        col = col.rstrip(")")
        kind = tfa.AGG_MAX if fn == "max" else tfa.AGG_MIN
        vals = clerk[col]
        nulls = np.array([v is None for v in vals], dtype=np.uint8)
        if col == "age":
            t, x = tfa.INT32, np.array([v or 0 for v in vals], dtype=np.int32)
        else:
            t, x = tfa.FLOAT64, np.array([v or 0.0 for v in vals], dtype=np.float64)
        kc = [_str_col(clerk[c]) for c in case["group_by"]]
        agg = tfa.KeysAggregator(ctx, [tfa.STRING] * len(kc), [(kind, t | tfa.NULLABLE)])
        agg.consume([(_t(c, dev), _t(o, dev)) for c, o in kc], [_t(x, dev)], arg_nullmaps=[_t(nulls, dev)])
        res = agg.result()
        sn = res["state_null"][0].cpu().numpy()
        got = [None if sn[i] else v for i, v in enumerate(res["states"][0].cpu().tolist())]
        key = lambda v: (v is None, v if v is not None else 0)  # noqa: E731
        assert sorted(got, key=key) == sorted(case["expected"], key=key), case
        assert len(got) == len(_clerk_groups(clerk, case["group_by"]))
