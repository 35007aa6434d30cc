"""min / max / first_row over Decimal128 / Decimal256 / String, and first_row of every type, on the
device (row-reference states, agg_dev.h ACC_REF) vs the oracle and the reference's answers.

Reference: AggregateFunctionMinMaxAny.cpp:39-46,85-98,155-159 (factory), AggregateFunctionMinMaxAny.h
:40-456 (SingleValueDataFixed / SingleValueDataString: strict changeIfLess / changeIfGreater,
changeFirstTime; String compares with the collator over the row with its '\\0'),
AggregateFunctionNull.h:193-330 (AggregateFunctionFirstRowNull: a NULL first row is the answer).
Known answers: gtest_aggregation_executor.cpp:740-750 (AggNull: max(s1) = "banana") and
:1160-1245 (AggKeyOptimization cases 3, 4, 6, 7: first_row of a String column), transcribed into
tests/golden/reference_cases.json.  The oracle keeps the reference's single-thread answer (the
first row in input order); the device is exact against it, ties and first rows included."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
NP = {1: np.int8, 2: np.int16, 3: np.int32, 4: np.int64, 5: np.uint8, 6: np.uint16, 7: np.uint32, 8: np.uint64,
      9: np.float32, 10: np.float64, 11: np.int32, 12: np.int64}
DEC = {13: 2, 14: 4}
STR = 20


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def str_col(vals):
    bs = [(v or "").encode() + b"\0" for v in vals]
    chars = np.frombuffer(b"".join(bs), dtype=np.uint8).copy()
    offs = np.cumsum([len(b) for b in bs]).astype(np.int64)
    return chars, offs


def _limbs(xs, limbs):
    return np.array([[(x >> (64 * j)) & ((1 << 64) - 1) for j in range(limbs)] for x in xs],
                    dtype=np.uint64).view(np.int64)


def _int_of(row):
    row = np.asarray(row).view(np.uint64)
    v = sum(int(x) << (64 * j) for j, x in enumerate(row))
    return v - (1 << (64 * len(row))) if v >> (64 * len(row) - 1) else v


def _values(state, t, g):
    """per-group Python values of a result state (device tensors or oracle arrays)"""
    base = t & 0xFF
    if base == STR:
        ch, of = state
        ch = ch.cpu().numpy() if torch.is_tensor(ch) else ch
        of = (of.cpu().numpy() if torch.is_tensor(of) else of).astype(np.int64)
        return [bytes(ch[(of[i - 1] if i else 0):of[i] - 1]) for i in range(g)]
    s = state.cpu().numpy() if torch.is_tensor(state) else state
    if base in DEC:
        return [_int_of(r) for r in s.view(np.int64).reshape(-1, DEC[base])[:g]]
    return [x.item() for x in s.view(NP[base])[:g]]


def _by_key(keys, states, nulls, types):
    g = len(keys)
    cols = [_values(s, t, g) for s, t in zip(states, types)]
    out = {}
    for r, k in enumerate(keys):
        out[int(k)] = [None if (n is not None and n[r]) else c[r] for c, n in zip(cols, nulls)]
    return out


def _dev(res, types):
    keys = res["keys"].cpu().numpy().view(np.int64) if res["keys"] is not None else np.zeros(1, np.int64)
    nulls = [res["state_null"][i].cpu().numpy() for i in range(len(types))]
    return _by_key(keys, res["states"], nulls, types)


def _orc(r, types):
    keys = r["keys"].view(np.int64)
    return _by_key(keys, r["states"], r["state_null"], types)


def _gen(rng, n, t):
    base = t & 0xFF
    if base in DEC:
        top = 1 << (100 if base == 13 else 240)
        # few distinct magnitudes per group so ties (equal values) are common
        vals = [int(a) * (top // 64) + int(b) for a, b in zip(rng.integers(-64, 64, n), rng.integers(0, 4, n))]
        return vals, _limbs(vals, DEC[base])
    if base == STR:
        alphabet = ["a", "A", "b", "B", " ", "é", "É", "ß", "ss", "z", "0"]
        vals = ["".join(rng.choice(alphabet, int(rng.integers(0, 6)))) for _ in range(n)]
        return vals, str_col(vals)
    dt = NP[base]
    if base in (9, 10):
        x = (rng.integers(-1000, 1000, n) / 8.0).astype(dt)
    else:
        info = np.iinfo(dt)
        x = rng.integers(max(info.min, -(1 << 40)), min(info.max, 1 << 40), n, dtype=np.int64).astype(dt)
    return x, x


def _arg(col, t, dev, sl=slice(None)):
    if (t & 0xFF) == STR:
        chars, offs = col
        o = offs[sl]
        start = int(offs[sl.start - 1]) if sl.start else 0
        end = int(o[-1]) if len(o) else start
        return (_t(chars[start:end], dev), _t(o - start, dev))
    return _t(col[sl], dev)


def _orc_arg(col, t, sl=slice(None)):
    if (t & 0xFF) == STR:
        chars, offs = col
        o = offs[sl]
        start = int(offs[sl.start - 1]) if sl.start else 0
        return (chars[start:int(o[-1]) if len(o) else start], (o - start).astype(np.uint64))
    return np.ascontiguousarray(col[sl])


def _run(tfa, orc, ctx, dev, aggs, k, cols, nulls, blocks=1):
    """consume in `blocks` blocks on the device and in the oracle; -> (device dict, oracle dict)"""
    types = [t for _, t in aggs]
    n = len(k)
    agg = tfa.Aggregator(ctx, tfa.INT64, aggs)
    ref = orc.Agg(orc.INT64, aggs)
    cuts = np.linspace(0, n, blocks + 1).astype(int)
    for b in range(blocks):
        sl = slice(int(cuts[b]), int(cuts[b + 1]))
        agg.consume(_t(k[sl], dev), [_arg(c, t, dev, sl) for c, t in zip(cols, types)],
                    arg_nullmaps=[_t(x[sl], dev) if x is not None else None for x in nulls])
        ref.consume(k[sl], [_orc_arg(c, t, sl) for c, t in zip(cols, types)],
                    arg_nulls=[np.ascontiguousarray(x[sl]) if x is not None else None for x in nulls])
    got, exp = _dev(agg.result(), types), _orc(ref.result(), types)
    agg.close()
    return got, exp


@pytest.mark.parametrize("t", [13, 14])
@pytest.mark.parametrize("n,groups,blocks", [(200_000, 5_000, 1), (300_000, 20_000, 3), (2_000_000, 1_000_000, 2)])
def test_decimal_min_max_first_vs_oracle(tfa, ctx, dev, orc, t, n, groups, blocks):
    rng = np.random.default_rng(n + t)
    k = rng.integers(0, groups, n).astype(np.int64)
    _, col = _gen(rng, n, t)
    nul = (rng.random(n) < 0.2).astype(np.uint8)
    aggs = [(tfa.AGG_MIN, t | tfa.NULLABLE), (tfa.AGG_MAX, t | tfa.NULLABLE), (tfa.AGG_FIRST_ROW, t | tfa.NULLABLE),
            (tfa.AGG_MAX, t)]
    got, exp = _run(tfa, orc, ctx, dev, aggs, k, [col] * 4, [nul, nul, nul, None], blocks)
    assert len(got) == len(exp)
    assert got == exp


@pytest.mark.parametrize("coll", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("n,groups,blocks", [(100_000, 3_000, 2), (1_500_000, 1_000_000, 1)])
def test_string_min_max_first_vs_oracle(tfa, ctx, dev, orc, coll, n, groups, blocks):
    if n > 200_000 and coll not in (0, 3):
        pytest.skip("the 1M-group size runs on the byte and general_ci compares")
    rng = np.random.default_rng(n + coll)
    k = rng.integers(0, groups, n).astype(np.int64)
    _, col = _gen(rng, n, STR)
    nul = (rng.random(n) < 0.2).astype(np.uint8)
    t = STR | (coll << 24)
    aggs = [(tfa.AGG_MIN, t | tfa.NULLABLE), (tfa.AGG_MAX, t | tfa.NULLABLE), (tfa.AGG_FIRST_ROW, t | tfa.NULLABLE),
            (tfa.AGG_MIN, t)]
    got, exp = _run(tfa, orc, ctx, dev, aggs, k, [col] * 4, [nul, nul, nul, None], blocks)
    assert len(got) == len(exp)
    assert got == exp


@pytest.mark.parametrize("types", [[3 | 0x100, 10, 8, 12 | 0x100], [1, 6 | 0x100, 9, 4]])
def test_first_row_numeric_is_the_first_row(tfa, ctx, dev, orc, types):
    """first_row of numeric arguments: exactly the first row in input order, a NULL first row NULL"""
    rng = np.random.default_rng(len(types) + types[0])
    n, groups = 400_000, 30_000
    k = rng.integers(0, groups, n).astype(np.int64)
    cols = [_gen(rng, n, t)[1] for t in types]
    nulls = [(rng.random(n) < 0.3).astype(np.uint8) if t & 0x100 else None for t in types]
    aggs = [(tfa.AGG_FIRST_ROW, t) for t in types]
    got, exp = _run(tfa, orc, ctx, dev, aggs, k, cols, nulls, blocks=2)
    assert got == exp


@pytest.mark.parametrize("t", [13, 14, STR, STR | (3 << 24), 4])
def test_wide_two_phase_and_merge(tfa, ctx, dev, orc, t):
    """partial results -> consume_partial (two-phase final) and tfg_agg_merge = one aggregation over
    the concatenated input (partials in input order: the first row stays the first row)"""
    rng = np.random.default_rng(t & 0xFFFF)
    n, groups = 300_000, 40_000
    k = rng.integers(0, groups, n).astype(np.int64)
    _, col = _gen(rng, n, t)
    nul = (rng.random(n) < 0.4).astype(np.uint8)
    aggs = [(tfa.AGG_MIN, t | tfa.NULLABLE), (tfa.AGG_MAX, t | tfa.NULLABLE), (tfa.AGG_FIRST_ROW, t | tfa.NULLABLE)]
    types = [a[1] for a in aggs]
    ref = orc.Agg(orc.INT64, aggs)
    ref.consume(k, [_orc_arg(col, t)] * 3, arg_nulls=[nul] * 3)
    exp = _orc(ref.result(), types)
    half = n // 2
    parts = []
    for sl in (slice(0, half), slice(half, n)):
        a = tfa.Aggregator(ctx, tfa.INT64, aggs)
        a.consume(_t(k[sl], dev), [_arg(col, t, dev, sl)] * 3, arg_nullmaps=[_t(nul[sl], dev)] * 3)
        parts.append(a)
    fin = tfa.Aggregator(ctx, tfa.INT64, aggs)
    for a in parts:
        r = a.result()
        fin.consume_partial(r["keys"], r["states"], state_nullmaps=r["state_null"])
    assert _dev(fin.result(), types) == exp
    fin.close()
    parts[0].merge(parts[1])
    assert _dev(parts[0].result(), types) == exp
    for a in parts:
        a.close()


def test_without_key_wide_and_empty(tfa, ctx, dev, orc):
    """without key: Decimal / String min / max / first_row; an empty input gives min / max the
    type's default (non-Nullable argument) and first_row NULL; reset restores that"""
    rng = np.random.default_rng(9)
    n = 50_000
    dv, dcol = _gen(rng, n, 14)
    sv, scol = _gen(rng, n, STR)
    x = rng.integers(-10**9, 10**9, n).astype(np.int64)
    aggs = [(tfa.AGG_MAX, 14), (tfa.AGG_MIN, STR | (4 << 24)), (tfa.AGG_FIRST_ROW, STR), (tfa.AGG_MIN, tfa.INT64)]
    types = [a[1] for a in aggs]
    agg = tfa.Aggregator(ctx, 0, aggs)
    empty = _dev(agg.result(), types)[0]
    assert empty[0] == 0 and empty[3] == 0
    assert empty[2] is None  # first_row of nothing is NULL
    agg.consume(None, [_t(dcol, dev), _arg(scol, STR, dev), _arg(scol, STR, dev), _t(x, dev)])
    ref = orc.Agg(0, aggs)
    ref.consume(None, [dcol, _orc_arg(scol, STR), _orc_arg(scol, STR), x], n=n)
    assert _dev(agg.result(), types) == _orc(ref.result(), types)
    assert _dev(agg.result(), types)[0][2] == sv[0].encode()
    agg.reset()
    again = _dev(agg.result(), types)[0]
    assert again[0] == 0 and again[2] is None
    # a filter that keeps nothing (min / max of no row without key = default 0)
    agg2 = tfa.Aggregator(ctx, 0, [(tfa.AGG_MIN, tfa.INT32), (tfa.AGG_MAX, tfa.FLOAT64), (tfa.AGG_MAX, tfa.INT64),
                                   (tfa.AGG_FIRST_ROW, tfa.INT64)])
    z = np.zeros(n, np.uint8)
    agg2.consume(None, [_t(x.astype(np.int32), dev), _t(x.astype(np.float64), dev), _t(x, dev), _t(x, dev)],
                 mask=_t(z, dev))
    r = agg2.result()
    assert r["states"][0].item() == 0 and r["states"][1].item() == 0.0 and r["states"][2].item() == 0
    assert r["state_null"][3].item() == 1
    agg.close()
    agg2.close()


def test_agg_null_reference_max_string(tfa, ctx, dev):
    """AggNull: max(s1) without key over Nullable(String) {"banana", NULL, "banana"} = "banana"."""
    c = json.load(open(os.path.join(HERE, "golden", "reference_cases.json")))["aggregates"]["agg_null"]
    chars, offs = str_col(c["s1"])
    nul = np.array([v is None for v in c["s1"]], np.uint8)
    agg = tfa.Aggregator(ctx, 0, [(tfa.AGG_MAX, STR | tfa.NULLABLE)])
    agg.consume(None, [(_t(chars, dev), _t(offs, dev))], arg_nullmaps=[_t(nul, dev)])
    r = agg.result()
    ch, of = r["states"][0]
    assert r["state_null"][0].item() == 0
    assert bytes(ch.cpu().numpy()[:int(of[0].item()) - 1]).decode() == c["max_s1"]
    agg.close()


def test_first_row_string_reference_cases(tfa, ctx, dev):
    """AggKeyOptimization cases 3, 4, 6, 7: count(1), first_row(String) GROUP BY one String key
    (key_string), several keys (serialized) -> counts 256, first_row "a".."d"."""
    c = json.load(open(os.path.join(HERE, "golden", "reference_cases.json")))["aggregates"]["first_row_string"]
    per = c["rows"] // c["row_types"]
    vals = [v for v in c["values"] for _ in range(per)]
    chars, offs = str_col(vals)
    s = (_t(chars, dev), _t(offs, dev))
    col_int = _t(np.repeat(np.arange(c["row_types"], dtype=np.int32), per), dev)
    cols = {"col_string_with_collator": (STR, s, 3), "col_string_no_collator": (STR, s, 0),
            "col_int": (3, col_int, 0)}
    for case in c["cases"]:
        kt = [cols[x][0] for x in case["keys"]]
        kc = [cols[x][2] for x in case["keys"]]
        arg_coll = cols[case["arg"]][2]
        agg = tfa.KeysAggregator(ctx, kt, [(tfa.AGG_COUNT_ALL, 0), (tfa.AGG_FIRST_ROW, STR | (arg_coll << 24))],
                                 collators=kc)
        agg.consume([cols[x][1] for x in case["keys"]], [None, s])
        r = agg.result()
        g = agg.size()
        firsts = _values(r["states"][1], STR, g)
        got = sorted(zip(firsts, r["states"][0].cpu().tolist()))
        assert [f.decode() for f, _ in got] == c["expected"], case
        assert [n for _, n in got] == c["count"], case
        agg.close()


def test_string_first_row_with_long_keys_serialized(tfa, ctx, dev, orc):
    """String min / first_row under the serialized method (String keys past 15 bytes) vs the oracle"""
    rng = np.random.default_rng(21)
    n = 60_000
    kv = [f"customer-name-{int(x):08d}" for x in rng.integers(0, 4000, n)]
    kch, kof = str_col(kv)
    _, col = _gen(rng, n, STR)
    aggs = [(tfa.AGG_FIRST_ROW, STR), (tfa.AGG_MIN, STR | (3 << 24)), (tfa.AGG_MAX, 13)]
    _, dcol = _gen(rng, n, 13)
    agg = tfa.KeysAggregator(ctx, [STR], aggs)
    agg.consume([(_t(kch, dev), _t(kof, dev))], [_arg(col, STR, dev), _arg(col, STR, dev), _t(dcol, dev)])
    r = agg.result()
    g = agg.size()
    kc_, ko_ = r["keys"][0]
    keys = _values((kc_, ko_), STR, g)
    got = {}
    cols = [_values(r["states"][i], aggs[i][1], g) for i in range(3)]
    for i, key in enumerate(keys):
        got[key] = [c[i] for c in cols]
    ref = orc.AggKeys([orc.STRING], aggs)
    ref.consume([(kch, kof.astype(np.uint64))], [_orc_arg(col, STR), _orc_arg(col, STR), dcol])
    exp = {}
    for key, vals in ref.result():
        exp[key[0]] = [vals[0], vals[1], vals[2]]
    assert got == exp


def test_min_max_unsupported_types(tfa, ctx):
    for t in (tfa.KEYS128,):
        with pytest.raises(tfa.TfgError) as e:
            tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_MIN, t)])
        assert e.value.code == -6
    with pytest.raises(tfa.TfgError) as e:
        tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_MAX, STR | (9 << 24))])
    assert e.value.code == -4


@pytest.mark.parametrize("nullmaps_of_nullable_only", [False, True])
def test_mixed_two_phase_with_count(tfa, ctx, dev, orc, nullmaps_of_nullable_only):
    """min(Nullable Int32), max(Float64), first_row(Int16), count(*) — the C++ planner test's
    signature — through two partial aggregators and a final consume_partial, vs one oracle pass"""
    rng = np.random.default_rng(77)
    n = 120_000
    k = (rng.integers(0, 3000, n) - 1000).astype(np.int64)
    v = (rng.integers(0, 2_000_001, n) - 1_000_000).astype(np.int32)
    vn = ((k % 7 == 0) | (rng.integers(0, 4, n) == 0)).astype(np.uint8)
    x = ((rng.integers(0, 1 << 24, n) - (1 << 23)) / 64.0).astype(np.float64)
    y = (k % 1000).astype(np.int16)
    aggs = [(tfa.AGG_MIN, tfa.INT32 | tfa.NULLABLE), (tfa.AGG_MAX, tfa.FLOAT64), (tfa.AGG_FIRST_ROW, tfa.INT16),
            (tfa.AGG_COUNT_ALL, 0)]
    types = [tfa.INT32, tfa.FLOAT64, tfa.INT16, tfa.UINT64]
    ref = orc.Agg(orc.INT64, aggs)
    ref.consume(k, [v, x, y, None], arg_nulls=[vn, None, None, None])
    exp = _orc(ref.result(), types)
    fin = tfa.Aggregator(ctx, tfa.INT64, aggs)
    for sl in (slice(0, n // 2), slice(n // 2, n)):
        a = tfa.Aggregator(ctx, tfa.INT64, aggs)
        a.consume(_t(k[sl], dev), [_t(v[sl], dev), _t(x[sl], dev), _t(y[sl], dev), None],
                  arg_nullmaps=[_t(vn[sl], dev), None, None, None])
        r = a.result()
        # the Nullable results' null maps only, as the C++ Aggregator::mergeOnBlock passes them
        nm = [r["state_null"][0], None, r["state_null"][2], None] if nullmaps_of_nullable_only else r["state_null"]
        fin.consume_partial(r["keys"], r["states"], state_nullmaps=nm)
        a.close()
    got = _dev(fin.result(), types)
    fin.close()
    bad = [(kk, got.get(kk), ev) for kk, ev in exp.items() if got.get(kk) != ev][:5]
    assert len(got) == len(exp) and not bad, bad



def test_mixed_two_phase_negative_values(tfa, ctx, dev, orc):
    """the C++ PlanAggregateMinMaxFirstRow two-phase case with its value signs: first_row(y) with
    y = k % 1000 under C's truncating %, so negative keys carry negative first_row values;
    partial aggregators over the two halves (each checked against the oracle), merged with
    consume_partial (null maps of the Nullable results only)"""
    rng = np.random.default_rng(77)
    n = 120_000
    k = (rng.integers(0, 3000, n) - 1000).astype(np.int64)
    v = (rng.integers(0, 2_000_001, n) - 1_000_000).astype(np.int32)
    vn = ((np.fmod(k, 7) == 0) | (rng.integers(0, 4, n) == 0)).astype(np.uint8)
    x = ((rng.integers(0, 1 << 24, n) - (1 << 23)) / 64.0).astype(np.float64)
    y = np.fmod(k, 1000).astype(np.int16)
    aggs = [(tfa.AGG_MIN, tfa.INT32 | tfa.NULLABLE), (tfa.AGG_MAX, tfa.FLOAT64), (tfa.AGG_FIRST_ROW, tfa.INT16),
            (tfa.AGG_COUNT_ALL, 0)]
    types = [tfa.INT32, tfa.FLOAT64, tfa.INT16, tfa.UINT64]
    ref = orc.Agg(orc.INT64, aggs)
    ref.consume(k, [v, x, y, None], arg_nulls=[vn, None, None, None])
    exp = _orc(ref.result(), types)
    fin = tfa.Aggregator(ctx, tfa.INT64, aggs)
    for sl in (slice(0, n // 2), slice(n // 2, n)):
        a = tfa.Aggregator(ctx, tfa.INT64, aggs)
        a.consume(_t(k[sl], dev), [_t(v[sl], dev), _t(x[sl], dev), _t(y[sl], dev), None],
                  arg_nullmaps=[_t(vn[sl], dev), None, None, None])
        res = a.result()
        part = _dev(res, types)
        pref = orc.Agg(orc.INT64, aggs)
        pref.consume(k[sl], [v[sl], x[sl], y[sl], None], arg_nulls=[vn[sl], None, None, None])
        pexp = _orc(pref.result(), types)
        bad = [(kk, part.get(kk), ev) for kk, ev in pexp.items() if part.get(kk) != ev][:5]
        assert len(part) == len(pexp) and not bad, ("partial", bad)
        fin.consume_partial(res["keys"], res["states"],
                            state_nullmaps=[res["state_null"][0], None, res["state_null"][2], None])
        a.close()
    got = _dev(fin.result(), types)
    fin.close()
    bad = [(kk, got.get(kk), ev) for kk, ev in exp.items() if got.get(kk) != ev][:5]
    assert len(got) == len(exp) and not bad, bad


def test_mixed_collators_and_decimal_blocks(tfa, ctx, dev, orc):
    """the C++ PlanAggregateWideMinMaxFirstRow aggregate set in one aggregator: min(s) under
    utf8_general_ci, max(s) binary, first_row(s) over a Nullable String of 0-3 (multi-byte)
    characters, max(d) Decimal128 — three blocks, vs the oracle"""
    rng = np.random.default_rng(91)
    n, groups = 60_000, 2_000
    k = rng.integers(0, groups, n).astype(np.int64)
    alpha = ["a", "A", "b", "B", " ", "é", "É", "ss", "ß", "z"]
    vals = ["".join(rng.choice(alpha, int(rng.integers(0, 4)))) for _ in range(n)]
    scol = str_col(vals)
    nul = (rng.random(n) < 0.2).astype(np.uint8)
    _, dcol = _gen(rng, n, 13)
    gci = STR | (3 << 24)
    aggs = [(tfa.AGG_MIN, gci | tfa.NULLABLE), (tfa.AGG_MAX, STR | tfa.NULLABLE),
            (tfa.AGG_FIRST_ROW, STR | tfa.NULLABLE), (tfa.AGG_MAX, 13)]
    got, exp = _run(tfa, orc, ctx, dev, aggs, k, [scol, scol, scol, dcol], [nul, nul, nul, None], 3)
    assert len(got) == len(exp)
    assert got == exp


@pytest.mark.parametrize("which", [0, 1])
def test_mixed_collators_two_phase_three_slices(tfa, ctx, dev, orc, which):
    """the two-phase half of the C++ PlanAggregateWideMinMaxFirstRow: three slices, each through
    its own partial aggregator (closed after its merge), into one final consume_partial; which=0:
    min(s) general_ci, max(s), first_row(s), max(d); which=1: first_row(d), first_row(s)"""
    rng = np.random.default_rng(191 + which)
    n, groups = 60_000, 2_000
    k = rng.integers(0, groups, n).astype(np.int64)
    alpha = ["a", "A", "b", "B", " ", "é", "É", "ss", "ß", "z"]
    vals = ["".join(rng.choice(alpha, int(rng.integers(0, 4)))) for _ in range(n)]
    scol = str_col(vals)
    nul = (rng.random(n) < 0.2).astype(np.uint8)
    _, dcol = _gen(rng, n, 13)
    gci = STR | (3 << 24)
    if which == 0:
        aggs = [(tfa.AGG_MIN, gci | tfa.NULLABLE), (tfa.AGG_MAX, STR | tfa.NULLABLE),
                (tfa.AGG_FIRST_ROW, STR | tfa.NULLABLE), (tfa.AGG_MAX, 13)]
        cols, nulls = [scol, scol, scol, dcol], [nul, nul, nul, None]
    else:
        aggs = [(tfa.AGG_FIRST_ROW, 13), (tfa.AGG_FIRST_ROW, STR | tfa.NULLABLE)]
        cols, nulls = [dcol, scol], [None, nul]
    types = [t for _, t in aggs]
    ref = orc.Agg(orc.INT64, aggs)
    ref.consume(k, [_orc_arg(c, t) for c, t in zip(cols, types)], arg_nulls=nulls)
    exp = _orc(ref.result(), types)
    fin = tfa.Aggregator(ctx, tfa.INT64, aggs)
    cuts = np.linspace(0, n, 4).astype(int)
    for b in range(3):
        sl = slice(int(cuts[b]), int(cuts[b + 1]))
        a = tfa.Aggregator(ctx, tfa.INT64, aggs)
        a.consume(_t(k[sl], dev), [_arg(c, t, dev, sl) for c, t in zip(cols, types)],
                  arg_nullmaps=[_t(x[sl], dev) if x is not None else None for x in nulls])
        r = a.result()
        # the Nullable results' null maps only (first_row always; min / max of a Nullable argument)
        nm = [r["state_null"][i] if (types[i] & tfa.NULLABLE or aggs[i][0] == tfa.AGG_FIRST_ROW) else None
              for i in range(len(aggs))]
        fin.consume_partial(r["keys"], r["states"], state_nullmaps=nm)
        a.close()
    got = _dev(fin.result(), types)
    fin.close()
    bad = [(kk, got.get(kk), ev) for kk, ev in exp.items() if got.get(kk) != ev][:5]
    assert len(got) == len(exp) and not bad, bad
