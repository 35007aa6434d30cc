"""Case-insensitive String keys on the GPU (§8 f2): utf8mb4_general_ci, utf8mb4_unicode_ci and
utf8mb4_0900_ai_ci.  Weak hash (exchange routing), GROUP BY (key_string and the serialized method)
and join keys, each against the oracle's restatement of the collator's sortKey (oracle/oracle.c
orc_collate, pinned by the reference's collator gtest answers in tests/golden/reference_cases.json
"general_ci" / "unicode_ci" / "uca0900_ai_ci").

Reference: GeneralCICollator::convertImpl (TiDB/Collation/Collator.cpp:416-455), weight
(Collator.h:403-407); UCACICollator::convertImpl (Collator.cpp:580-629) with Unicode0400 /
Unicode0900::weight (:703-727, 791-816); consumers: ColumnString::updateWeakHash32 (ColumnString.cpp:1244),
HashMethodString (ColumnsHashing.h:233), serializeValueIntoArena (AggregationCommon.h:202),
the join's key_strbin path (JoinHashMap.cpp:83-112)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# letters in several cases and accents, CJK, astral characters (weight 0xFFFD), trailing spaces
# (UCA: a zero-weight control character, long weights U+321D / U+3307 / U+FDFB, a code point past
# the 9.0.0 table)
ALPHABET = ["a", "A", "à", "À", "á", "b", "B", "ß", "s", "S", "œ", "é", "E",
            "謺", "譂", "\U0001F603", "\U0001F61C", "z", "ё", "Ё", "ẞ", "1", "_",
            "\x01", "\u321d", "\u3307", "\ufdfb", "\U00030000"]
COLLATORS = [3, 4, 5]  # COLLATOR_GENERAL_CI, COLLATOR_UNICODE_CI, COLLATOR_UCA0900_AI_CI


def _random_strings(rng, n, maxlen):
    out = []
    for _ in range(n):
        k = int(rng.integers(0, maxlen + 1))
        s = "".join(ALPHABET[int(i)] for i in rng.integers(0, len(ALPHABET), k))
        if rng.random() < 0.2:
            s += " " * int(rng.integers(1, 3))
        out.append(s.encode("utf-8"))
    return out


def _column(strs):
    chars = np.frombuffer(b"".join(s + b"\0" for s in strs), dtype=np.uint8).copy()
    offsets = np.cumsum([len(s) + 1 for s in strs]).astype(np.uint64)
    return chars, offsets


def _sort_key(orc, s, collator):
    lib = orc.lib()
    lib.orc_collate.restype = ctypes.c_size_t
    out = ctypes.create_string_buffer(8 * len(s) + 16)
    n = lib.orc_collate(collator, s, ctypes.c_size_t(len(s)), ctypes.c_size_t(len(s) + 1), out)
    return out.raw[:n]


@pytest.mark.parametrize("collator", COLLATORS)
@pytest.mark.parametrize("selective", [False, True])
def test_ci_weak_hash(tfa, ctx, dev, orc, selective, collator):
    rng = np.random.default_rng(71 + selective)
    strs = _random_strings(rng, 20_000, 12)
    chars, offs = _column(strs)
    nulls = (rng.random(len(strs)) < 0.05).astype(np.uint8)
    n = len(strs)
    exp = orc.weak_hash_string(chars, offs.view(np.int64), np.full(n, 0xFFFFFFFF, np.uint32), nulls, collator)
    h = torch.full((n,), -1, dtype=torch.int32, device=dev)
    sel = None
    if selective:
        rows = np.sort(rng.choice(n, n // 3, replace=False)).astype(np.uint64)
        sel = torch.from_numpy(rows.view(np.int64)).to(dev)
        h = torch.full((rows.shape[0],), -1, dtype=torch.int32, device=dev)
        exp = exp[rows.astype(np.int64)]
    got = tfa.weak_hash_string(ctx, torch.from_numpy(chars).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev), h,
                               nullmap=torch.from_numpy(nulls).to(dev), collator=collator, selective=sel)
    assert np.array_equal(got.cpu().numpy().view(np.uint32), exp.view(np.uint32))
    # equal sort keys hash equal: 'a' / 'A' / 'à' ...
    eq = [b"abc", b"ABC", "àBC".encode(), b"a\x01bc"] if collator == 5 else [b"abc", b"ABC", "àBC".encode(), b"abc  "]
    c2, o2 = _column(eq)
    h2 = torch.full((4,), -1, dtype=torch.int32, device=dev)
    g2 = tfa.weak_hash_string(ctx, torch.from_numpy(c2).to(dev), torch.from_numpy(o2.view(np.int64)).to(dev), h2,
                              collator=collator).cpu().numpy()
    assert len(set(g2.tolist())) == 1


@pytest.mark.parametrize("collator", COLLATORS)
@pytest.mark.parametrize("maxlen", [6, 20])  # 6: mostly packed key_string keys (<= 15 key bytes); 20: serialized
def test_ci_group_by_string(tfa, ctx, dev, orc, maxlen, collator):
    rng = np.random.default_rng(81 + maxlen)
    strs = _random_strings(rng, 30_000, maxlen)
    chars, offs = _column(strs)
    v = rng.integers(-1000, 1000, len(strs)).astype(np.int64)
    aggs = [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, collators=[collator])
    agg.consume([(torch.from_numpy(chars).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev))],
                [torch.from_numpy(v).to(dev), None])
    res = agg.result()
    gc, go = (t.cpu().numpy() for t in res["keys"][0])
    starts = np.concatenate([[0], go.view(np.uint64)[:-1]]).astype(np.int64)
    got = {}
    for i in range(len(go)):
        key = gc[starts[i]:int(go[i]) - 1].tobytes()  # the sort key (the Aggregator's key column)
        assert key not in got
        got[key] = (int(res["states"][0][i].item()), int(res["states"][1][i].item()))
    agg.close()
    exp = {}
    for s, x in zip(strs, v):
        k = _sort_key(orc, s, collator)
        a, c = exp.get(k, (0, 0))
        exp[k] = (a + int(x), c + 1)
    assert got == exp
    # the oracle's own GROUP BY under the collator agrees
    ref = orc.AggKeys([orc.STRING], [(0, orc.INT64), (2, 0)], collators=[collator])
    ref.consume([(chars, offs)], [v, None])
    assert ref.size() == len(exp)


@pytest.mark.parametrize("collator", COLLATORS)
def test_ci_group_by_string_and_int(tfa, ctx, dev, orc, collator):
    """String + Int64 keys: the serialized method, the String part as its sort key."""
    rng = np.random.default_rng(91)
    strs = _random_strings(rng, 20_000, 5)
    chars, offs = _column(strs)
    k2 = rng.integers(0, 3, len(strs)).astype(np.int64)
    agg = tfa.KeysAggregator(ctx, [tfa.STRING, tfa.INT64], [(tfa.AGG_COUNT_ALL, 0)],
                             collators=[collator, 0])
    agg.consume([(torch.from_numpy(chars).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev)),
                 torch.from_numpy(k2).to(dev)], [None])
    res = agg.result()
    gc, go = (t.cpu().numpy() for t in res["keys"][0])
    gk2 = res["keys"][1].cpu().numpy()
    starts = np.concatenate([[0], go.view(np.uint64)[:-1]]).astype(np.int64)
    got = {(gc[starts[i]:int(go[i]) - 1].tobytes(), int(gk2[i])): int(res["states"][0][i].item()) for i in range(len(go))}
    agg.close()
    exp = {}
    for s, x in zip(strs, k2):
        key = (_sort_key(orc, s, collator), int(x))
        exp[key] = exp.get(key, 0) + 1
    assert got == exp


@pytest.mark.parametrize("collator", COLLATORS)
def test_ci_join_keys(tfa, ctx, dev, orc, collator):
    rng = np.random.default_rng(101)
    bs = _random_strings(rng, 3000, 4)
    ps = _random_strings(rng, 12_000, 4)
    bc, bo = _column(bs)
    pc, po = _column(ps)
    t = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    ci = [collator]
    fb, nbm = tfa.join_key_hash(ctx, [t(bc)], [tfa.STRING], offsets=[t(bo.view(np.int64))], collators=ci)
    fp, npm = tfa.join_key_hash(ctx, [t(pc)], [tfa.STRING], offsets=[t(po.view(np.int64))], collators=ci)
    j = tfa.Join(ctx, tfa.UINT64)
    j.build(fb, key_nullmap=nbm)
    pi, bi = j.probe(fp, kind=tfa.JOIN_INNER, key_nullmap=npm)
    ok = tfa.join_keys_equal(ctx, [tfa.STRING], [t(pc)], [t(bc)], pi, bi, probe_offsets=[t(po.view(np.int64))],
                             build_offsets=[t(bo.view(np.int64))], collators=ci).cpu().numpy().astype(bool)
    got = sorted(zip(pi.cpu().numpy().view(np.uint32)[ok].tolist(), bi.cpu().numpy().view(np.uint32)[ok].tolist()))
    idx = {}
    for r, s in enumerate(bs):
        idx.setdefault(_sort_key(orc, s, collator), []).append(r)
    exp = sorted((i, r) for i, s in enumerate(ps) for r in idx.get(_sort_key(orc, s, collator), []))
    assert got == exp and len(exp) > 1000
