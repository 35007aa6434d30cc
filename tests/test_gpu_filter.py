"""GPU parity: comparison, mask logic, countBytesInFilter, filter compaction (a1-a8) vs the oracle.

Mirrors dbms/src/Flash/tests/gtest_filter_executor.cpp (equals / andOr / convertBool) and the
selectivity sweep of dbms/src/Columns/tests/bench_column_filter.cpp:251-290.  Bit-exact.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

OPS = [0, 1, 2, 3, 4, 5]  # EQ NE LT LE GT GE
NP_TO_T = {np.int8: 1, np.int16: 2, np.int32: 3, np.int64: 4, np.uint8: 5, np.uint16: 6, np.uint32: 7,
           np.uint64: 8, np.float32: 9, np.float64: 10}


def _t(x, dev):
    if x.dtype == np.uint64:
        return torch.from_numpy(x.view(np.int64)).to(dev)
    if x.dtype == np.uint32:
        return torch.from_numpy(x.view(np.int32)).to(dev)
    if x.dtype == np.uint16:
        return torch.from_numpy(x.view(np.int16)).to(dev)
    return torch.from_numpy(x).to(dev)


def _col(rng, dtype, n):
    if np.issubdtype(dtype, np.floating):
        x = rng.normal(0, 100, n).astype(dtype)
        if n:
            x[rng.integers(0, n, max(1, n // 50))] = np.nan
        x[: min(n, 4)] = [0.0, -0.0, np.inf, -np.inf][: min(n, 4)]
        return x
    info = np.iinfo(dtype)
    x = rng.integers(info.min, info.max, n, dtype=dtype, endpoint=True)
    x[: min(n, 4)] = np.array([info.min, info.max, 0, 1], dtype=dtype)[: min(n, 4)]
    return x


@pytest.mark.parametrize("dtype", list(NP_TO_T))
@pytest.mark.parametrize("n", [0, 1, 17, 4096, 100_003])
def test_cmp_const_all_types(tfa, ctx, dev, orc, dtype, n):
    rng = np.random.default_rng(n + NP_TO_T[dtype])
    a = _col(rng, dtype, n)
    ct = NP_TO_T[dtype]
    scalars = [(tfa.INT64, 0), (tfa.INT64, -1), (tfa.UINT64, 2**63 + 5), (tfa.FLOAT64, 0.5), (tfa.FLOAT64, float("nan")),
               (tfa.INT64, 2**53 + 1), (tfa.FLOAT64, 9.3e18), (tfa.UINT8, 255)]
    for st, sv in scalars:
        for op in OPS:
            got = tfa.cmp_const(ctx, _t(a, dev), op, sv, scalar_type=st, col_type=ct).cpu().numpy()
            ctype = {tfa.INT64: np.int64, tfa.UINT64: np.uint64, tfa.FLOAT64: np.float64, tfa.UINT8: np.uint8}[st]
            exp = orc.cmp(a, op, np.array([sv], dtype=ctype), a_type=ct, b_type=st, b_const=True, n=n)
            np.testing.assert_array_equal(got, exp, err_msg=f"{dtype} {op} {st}:{sv}")


def test_accurate_comparison_known_answers(tfa, ctx, dev):
    # Core/AccurateComparison.h:27-29 "Int8(-1) != UInt8(255)"; int vs float exact; NaN false
    a = torch.tensor([-1], dtype=torch.int8, device=dev)
    assert tfa.cmp_const(ctx, a, tfa.EQ, 255, scalar_type=tfa.UINT8).item() == 0
    assert tfa.cmp_const(ctx, a, tfa.LT, 255, scalar_type=tfa.UINT8).item() == 1
    big = torch.tensor([2**53 + 1], dtype=torch.int64, device=dev)
    assert tfa.cmp_const(ctx, big, tfa.GT, float(2**53), scalar_type=tfa.FLOAT64).item() == 1
    assert tfa.cmp_const(ctx, big, tfa.EQ, float(2**53), scalar_type=tfa.FLOAT64).item() == 0
    nan = torch.tensor([float("nan")], dtype=torch.float64, device=dev)
    for op, exp in [(tfa.EQ, 0), (tfa.NE, 1), (tfa.LT, 0), (tfa.LE, 0), (tfa.GT, 0), (tfa.GE, 0)]:
        assert tfa.cmp_const(ctx, nan, op, 1, scalar_type=tfa.INT64).item() == exp


@pytest.mark.parametrize("pair", [(np.int64, np.int64), (np.int32, np.uint32), (np.int64, np.float64),
                                  (np.uint64, np.int8), (np.float32, np.float64), (np.uint16, np.float32)])
def test_cmp_vector(tfa, ctx, dev, orc, pair):
    rng = np.random.default_rng(7)
    n = 50_001
    a, b = _col(rng, pair[0], n), _col(rng, pair[1], n)
    b[::3] = b[::3].astype(pair[1])  # some equal values
    nulls = (rng.random(n) < 0.1).astype(np.uint8)
    for op in OPS:
        got = tfa.cmp_vector(ctx, _t(a, dev), op, _t(b, dev), a_nullmap=torch.from_numpy(nulls).to(dev),
                             a_type=NP_TO_T[pair[0]], b_type=NP_TO_T[pair[1]]).cpu().numpy()
        exp = orc.cmp(a, op, b, a_type=NP_TO_T[pair[0]], b_type=NP_TO_T[pair[1]], a_null=nulls)
        np.testing.assert_array_equal(got, exp)


def test_mask_logic_and_count(tfa, ctx, dev, orc):
    rng = np.random.default_rng(3)
    n = 123_457
    a = rng.integers(0, 3, n).astype(np.uint8)
    b = rng.integers(0, 2, n).astype(np.uint8)
    ad, bd = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    np.testing.assert_array_equal(tfa.mask_logic(ctx, tfa.AND, ad, bd).cpu().numpy(), ((a != 0) & (b != 0)).astype(np.uint8))
    np.testing.assert_array_equal(tfa.mask_logic(ctx, tfa.OR, ad, bd).cpu().numpy(), ((a != 0) | (b != 0)).astype(np.uint8))
    np.testing.assert_array_equal(tfa.mask_logic(ctx, tfa.NOT, ad).cpu().numpy(), (a == 0).astype(np.uint8))
    nulls = (rng.random(n) < 0.2).astype(np.uint8)
    assert tfa.count_mask(ctx, ad) == orc.count_bytes_in_filter(a)
    assert tfa.count_mask(ctx, ad, torch.from_numpy(nulls).to(dev)) == orc.count_bytes_in_filter(a, nulls)


@pytest.mark.parametrize("sel", [0.0, 0.01, 0.1, 0.5, 0.96, 1.0])
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 4095, 4096, 4097, 1_000_003])
def test_filter_selectivity_sweep(tfa, ctx, dev, orc, sel, n):
    rng = np.random.default_rng(int(sel * 100) + n)
    mask = (rng.random(n) < sel).astype(np.uint8) * rng.integers(1, 255, n).astype(np.uint8)  # any nonzero keeps
    c8 = rng.integers(-2**62, 2**62, n, dtype=np.int64)
    c4 = rng.random(n).astype(np.float32)
    c1 = rng.integers(0, 255, n).astype(np.uint8)
    c16 = rng.integers(-2**62, 2**62, (n, 2), dtype=np.int64)
    outs = tfa.filter(ctx, torch.from_numpy(mask).to(dev), [torch.from_numpy(x).to(dev) for x in (c8, c4, c1, c16)])
    for x, o in zip((c8, c4, c1, c16), outs):
        np.testing.assert_array_equal(o.cpu().numpy(), orc.filter(x, mask))


def test_filter_misaligned_columns(tfa, ctx, dev, orc):
    rng = np.random.default_rng(11)
    n = 10_000
    base = torch.from_numpy(rng.integers(0, 1000, n + 3, dtype=np.int64)).to(dev)
    col = base[3:]  # 24-byte offset: not 16-byte aligned
    mask_full = torch.from_numpy((rng.random(n + 1) < 0.5).astype(np.uint8)).to(dev)
    mask = mask_full[1:]
    out, = tfa.filter(ctx, mask, [col])
    np.testing.assert_array_equal(out.cpu().numpy(), orc.filter(col.cpu().numpy(), mask.cpu().numpy()))


@pytest.mark.parametrize("n", [0, 5, 4096, 300_001])
def test_fused_filter_cmp_const(tfa, ctx, dev, orc, n):
    rng = np.random.default_rng(n)
    f = rng.integers(0, 100, n, dtype=np.int64)
    k = rng.integers(0, 10**6, n, dtype=np.int64)
    v = rng.random(n)
    nulls = (rng.random(n) < 0.05).astype(np.uint8)
    ko, vo = tfa.filter_cmp_const(ctx, torch.from_numpy(f).to(dev), tfa.LT, 96,
                                  [torch.from_numpy(k).to(dev), torch.from_numpy(v).to(dev)],
                                  pred_nullmap=torch.from_numpy(nulls).to(dev))
    mask = orc.cmp(f, 2, np.array([96]), b_const=True, a_null=nulls, n=n)
    np.testing.assert_array_equal(ko.cpu().numpy(), orc.filter(k, mask))
    np.testing.assert_array_equal(vo.cpu().numpy(), orc.filter(v, mask))


def test_filter_string(tfa, ctx, dev, orc):
    rng = np.random.default_rng(1)
    n = 20_000
    strs = [b"k%08d" % i if i % 7 else b"x" * (i % 130) for i in range(n)]
    chars = np.frombuffer(b"".join(s + b"\0" for s in strs), dtype=np.uint8).copy()
    offsets = np.cumsum([len(s) + 1 for s in strs]).astype(np.uint64)
    mask = (rng.random(n) < 0.3).astype(np.uint8)
    gc, go = tfa.filter_string(ctx, torch.from_numpy(mask).to(dev), torch.from_numpy(chars).to(dev),
                               torch.from_numpy(offsets.view(np.int64)).to(dev))
    ec, eo = orc.filter_string(chars, offsets, mask)
    np.testing.assert_array_equal(gc.cpu().numpy(), ec)
    np.testing.assert_array_equal(go.cpu().numpy().view(np.uint64), eo)
