"""GPU parity: general join keys (§8 f2) and the String gather of joined rows.

chooseJoinMapMethod (dbms/src/Interpreters/JoinHashMap.cpp:33-116) joins several fixed keys as
keys128 / keys256, one String key as key_strbin / key_strbinpadding by collator, and anything
else as serialized.  Here those key sets join on device fingerprints (tfg_join_key_hash) through
the UInt64 table, and tfg_join_keys_equal keeps the key-equal candidate pairs.  The expected pairs
come from a pure-Python nested loop over the same rows (small sizes); a NULL in any key column
never matches (extractNestedColumnsAndNullMap ORs the key null maps).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _strings(strs):
    chars = np.frombuffer(b"".join(s + b"\0" for s in strs), dtype=np.uint8).copy()
    offsets = np.cumsum([len(s) + 1 for s in strs]).astype(np.int64)
    return chars, offsets


def _sort_key(s, collator):
    return s.rstrip(b" ") if collator == 2 else s


def _device_pairs(tfa, ctx, dev, fp_b, null_b, fp_p, null_p):
    j = tfa.Join(ctx, tfa.UINT64)
    if fp_b.shape[0]:
        j.build(fp_b, key_nullmap=null_b)
    return j.probe(fp_p, kind=tfa.JOIN_INNER, key_nullmap=null_p)


@pytest.mark.parametrize("nb,np_", [(0, 50), (1, 1), (300, 2000), (5000, 40_000)])
def test_join_two_fixed_keys(tfa, ctx, dev, nb, np_):
    rng = np.random.default_rng(nb + np_)
    ba = rng.integers(0, 7, nb).astype(np.int32)
    bb = rng.integers(-3, 3, nb).astype(np.int64)
    bn = (rng.random(nb) < 0.1).astype(np.uint8)
    pa = rng.integers(0, 8, np_).astype(np.int32)
    pb = rng.integers(-3, 4, np_).astype(np.int64)
    pn = (rng.random(np_) < 0.1).astype(np.uint8)
    t = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    types = [tfa.INT32, tfa.INT64]
    fb, nbm = tfa.join_key_hash(ctx, [t(ba), t(bb)], types, nullmaps=[None, t(bn)]) if nb else (t(bb), t(bn))
    fp, npm = tfa.join_key_hash(ctx, [t(pa), t(pb)], types, nullmaps=[None, t(pn)])
    assert np.array_equal(npm.cpu().numpy(), pn)
    pi, bi = _device_pairs(tfa, ctx, dev, fb, nbm, fp, npm)
    ok = tfa.join_keys_equal(ctx, types, [t(pa), t(pb)], [t(ba), t(bb)], pi, bi) if nb else pi.new_zeros(0)
    ok = ok.cpu().numpy().astype(bool)
    got = sorted(zip(pi.cpu().numpy()[ok].tolist(), bi.cpu().numpy()[ok].tolist()))
    idx = {}
    for r in range(nb):
        if not bn[r]:
            idx.setdefault((int(ba[r]), int(bb[r])), []).append(r)
    exp = sorted((i, r) for i in range(np_) if not pn[i] for r in idx.get((int(pa[i]), int(pb[i])), []))
    assert got == exp


@pytest.mark.parametrize("collator", [0, 1, 2])
def test_join_string_key(tfa, ctx, dev, collator):
    rng = np.random.default_rng(30 + collator)
    words = [b"", b"a", b"a ", b"a  ", b"k%08d" % 3, b"k%08d " % 3, b"x" * 40, b"x" * 39 + b"y", b" a", b"z" * 16]
    bs = [words[i] for i in rng.integers(0, len(words), 400)]
    ps = [words[i] for i in rng.integers(0, len(words), 3000)]
    bc, bo = _strings(bs)
    pc, po = _strings(ps)
    t = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    fb, nbm = tfa.join_key_hash(ctx, [t(bc)], [tfa.STRING], offsets=[t(bo)], collators=[collator])
    fp, npm = tfa.join_key_hash(ctx, [t(pc)], [tfa.STRING], offsets=[t(po)], collators=[collator])
    pi, bi = _device_pairs(tfa, ctx, dev, fb, nbm, fp, npm)
    ok = tfa.join_keys_equal(ctx, [tfa.STRING], [t(pc)], [t(bc)], pi, bi, probe_offsets=[t(po)],
                             build_offsets=[t(bo)], collators=[collator]).cpu().numpy().astype(bool)
    got = sorted(zip(pi.cpu().numpy()[ok].tolist(), bi.cpu().numpy()[ok].tolist()))
    exp = sorted((i, r) for i in range(len(ps)) for r in range(len(bs))
                 if _sort_key(ps[i], collator) == _sort_key(bs[r], collator))
    assert got == exp
    # equal sort keys hash equally (the fingerprint is a function of the sort key alone)
    fpn, fbn = fp.cpu().numpy(), fb.cpu().numpy()
    for i, s in enumerate(ps[:50]):
        for r, u in enumerate(bs[:50]):
            if _sort_key(s, collator) == _sort_key(u, collator):
                assert fpn[i] == fbn[r]


def test_keys_equal_rejects_unequal_pairs(tfa, ctx, dev):
    """Verification is exact whatever pairs the table proposes (stands in for a fingerprint
    collision): every (i, j) over a small cross product is checked against Python equality."""
    a = np.array([1, 1, 2, 2, 0], dtype=np.int32)
    d = np.array([[5, 0], [5, 1], [5, 0], [-1, -1], [0, 0]], dtype=np.int64)  # Decimal128 limbs
    n = len(a)
    pi = torch.tensor([i for i in range(n) for _ in range(n)], dtype=torch.int32, device=dev)
    bi = torch.tensor([j for _ in range(n) for j in range(n)], dtype=torch.int32, device=dev)
    t = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    passin = torch.ones(n * n, dtype=torch.uint8, device=dev)
    passin[0] = 0
    ok = tfa.join_keys_equal(ctx, [tfa.INT32, tfa.DECIMAL128], [t(a), t(d)], [t(a), t(d)], pi, bi,
                             pass_in=passin).cpu().numpy()
    exp = [int(a[i] == a[j] and (d[i] == d[j]).all() and not (i == 0 and j == 0)) for i in range(n) for j in range(n)]
    assert ok.tolist() == exp


def test_gather_string(tfa, ctx, dev):
    strs = [b"", b"abc", b"k%08d" % 9, b"y" * 300, b"q"]
    c, o = _strings(strs)
    perm = np.array([3, 0, -1, 2, 2, 4, -1, 1], dtype=np.int32)
    oc, oo = tfa.gather_string(ctx, torch.from_numpy(perm).to(dev), torch.from_numpy(c).to(dev),
                               torch.from_numpy(o).to(dev))
    ec, eo = _strings([strs[p] if p >= 0 else b"" for p in perm])
    assert np.array_equal(oc.cpu().numpy(), ec)
    assert np.array_equal(oo.cpu().numpy(), eo)
