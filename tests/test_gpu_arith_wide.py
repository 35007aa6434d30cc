"""GPU parity of tfg_arith's wide path (a3, §8 f): Decimal256 results and operands, and multiplies
whose result scale is capped below sa + sb (decimal_max_scale 30), against the oracle's exact
integer restatement (oracle.oracle.arith_decimal_wide) of DecimalBinaryOperation
(Functions/FunctionBinaryArithmetic.h:231-640) with the inferers of Common/Decimal.h:109-163.

The reference's own gtests hold no Decimal256 +, -, * answers (gtest_arithmetic_functions.cpp:
311-358 covers Decimal256 division only), so beyond the inferers' result types (pinned in
tests/golden/reference_cases.json "sum_types" / "arith_scales") these values are parity unpinned:
the oracle is the rules as read from the code, checked here against hand-derived values.
Overflow (DECIMAL_OVERFLOW: a value past Int256, or past 10^65 - 1 when an operand is Decimal256)
fails the call with TfgError, never a wrapped value."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

I32, I64, D32, D64, D128, D256 = 3, 4, 11, 12, 13, 14
LIMBS = {D128: 2, D256: 4}
INT_PREC = {I32: 10, I64: 19}
# (type, precision, scale) operands: integers, narrow decimals, Decimal128 and Decimal256
OPERANDS = [(I64, None, 0), (I32, None, 0), (D32, 9, 2), (D64, 18, 4), (D128, 30, 3), (D128, 38, 10),
            (D256, 50, 5), (D256, 65, 0), (D256, 65, 30), (D256, 40, 20)]
N = 1031


def _result(op, pa, sa, pb, sb):
    if op == 2:
        p, s = min(pa + pb, 65), min(sa + sb, 30)
    else:
        s = max(sa, sb)
        p = min(max(pa - sa, pb - sb) + s + 1, 65)
    return (D32 if p <= 9 else D64 if p <= 18 else D128 if p <= 38 else D256), p, s


def _vals(rng, t, prec, n, small):
    if t in (I32, I64):
        bits = 31 if t == I32 else 63
        v = [int(x) for x in rng.integers(-(1 << bits), (1 << bits) - 1, n)]
        v[:3] = [-(1 << bits), (1 << bits) - 1, 0]
    else:
        lim = 10 ** (min(prec, 6) if small else prec)
        v = [int(x) % lim * (1 if i % 2 else -1) for i, x in enumerate(rng.integers(0, 1 << 62, n))]
        v = [x * (lim // (1 << 62) + 1) % lim if not small and lim > (1 << 62) else x for x in v]
        v[:3] = [lim - 1, -(lim - 1), 0]
    return v


def _tensor(t, vals, dev):
    if t in LIMBS:
        k = LIMBS[t]
        m = (1 << (64 * k)) - 1
        arr = np.array([[((v & m) >> (64 * j)) & ((1 << 64) - 1) for j in range(k)] for v in vals], dtype=np.uint64)
        return torch.from_numpy(arr.view(np.int64)).to(dev)
    return torch.from_numpy(np.array(vals, dtype=np.int32 if t in (I32, D32) else np.int64)).to(dev)


def _ints(t, got):
    a = got.cpu().numpy()
    if t in LIMBS:
        u = a.view(np.uint64)
        k = LIMBS[t]
        out = []
        for row in u:
            v = sum(int(row[j]) << (64 * j) for j in range(k))
            out.append(v - (1 << (64 * k)) if v >> (64 * k - 1) else v)
        return out
    return [int(x) for x in a]


def _cases():
    for ta, pa, sa in OPERANDS:
        for tb, pb, sb in OPERANDS:
            if pa is None and pb is None:
                continue
            for op in (0, 1, 2):
                rt, _, rs = _result(op, pa or INT_PREC[ta], sa, pb or INT_PREC[tb], sb)
                capped = op == 2 and rs != sa + sb
                if rt == D256 or D256 in (ta, tb) or capped:
                    yield ta, pa, sa, tb, pb, sb, op, rt, rs


@pytest.mark.parametrize("mode", [0, 1, 2], ids=["vector_vector", "const_vector", "vector_const"])
@pytest.mark.parametrize("small", [True, False], ids=["small", "full_range"])
def test_wide_arith_matches_oracle(tfa, ctx, dev, mode, small):
    rng = np.random.default_rng(7 + mode + 10 * small)
    ran = overflowed = 0
    for ta, pa, sa, tb, pb, sb, op, rt, rs in _cases():
        a = _vals(rng, ta, pa, N, small)
        b = _vals(rng, tb, pb, N, small)
        if mode == 1:
            a = [a[int(rng.integers(0, N))]] * N
        elif mode == 2:
            b = [b[int(rng.integers(0, N))]] * N
        da = a[0] if mode == 1 else _tensor(ta, a, dev)
        db = b[0] if mode == 2 else _tensor(tb, b, dev)
        try:
            exp = orc.arith_decimal_wide(op, a, b, ta, tb, sa, sb, rt, rs)
        except OverflowError:
            exp = None
        if exp is None:
            with pytest.raises(tfa.TfgError) as ei:
                tfa.arith(ctx, op, da, db, rt, a_type=ta, b_type=tb, a_scale=sa, b_scale=sb, res_scale=rs, n=N,
                          device=dev)
            assert ei.value.code == tfa.TFG_ERR_OVERFLOW
            overflowed += 1
            continue
        got = tfa.arith(ctx, op, da, db, rt, a_type=ta, b_type=tb, a_scale=sa, b_scale=sb, res_scale=rs, n=N,
                        device=dev)
        bits = {D32: 32, D64: 64, D128: 128, D256: 256}[rt]
        wrap = lambda v: (v + (1 << (bits - 1))) % (1 << bits) - (1 << (bits - 1))  # noqa: E731
        assert _ints(rt, got) == [wrap(v) for v in exp], (ta, pa, sa, tb, pb, sb, op, rt, rs, mode)
        ran += 1
    assert ran > 60
    if not small:
        assert overflowed > 0  # Decimal(65) +/- Decimal(65) at full range leaves 10^65 - 1


def test_wide_arith_known_values(tfa, ctx, dev):
    """Hand-derived: Decimal(65,0) (10^65 - 1) + 1 overflows; (10^65 - 1) - 1 does not;
    Decimal(38,10) x Decimal(38,25) -> Decimal(65,30): the raw product / 10^5, truncated toward 0;
    Decimal(38,0) + Decimal(38,38) -> Decimal(65,38): the first operand scaled by 10^38."""
    big = 10 ** 65 - 1
    a = _tensor(D256, [big], dev)
    with pytest.raises(tfa.TfgError):
        tfa.arith(ctx, 0, a, 1, D256, a_type=D256, b_type=I64, a_scale=0, res_scale=0)
    r = tfa.arith(ctx, 1, a, 1, D256, a_type=D256, b_type=I64, a_scale=0, res_scale=0)
    assert _ints(D256, r) == [big - 1]
    x = _tensor(D128, [123456789, -123456789], dev)
    y = _tensor(D128, [100001, 100001], dev)
    m = tfa.arith(ctx, 2, x, y, D256, a_type=D128, b_type=D128, a_scale=10, b_scale=25, res_scale=30)
    assert _ints(D256, m) == [123456789 * 100001 // 10 ** 5, -(123456789 * 100001 // 10 ** 5)]
    p = tfa.arith(ctx, 0, _tensor(D128, [10 ** 38 - 1], dev), _tensor(D128, [1], dev), D256, a_type=D128,
                  b_type=D128, a_scale=0, b_scale=38, res_scale=38)
    assert _ints(D256, p) == [(10 ** 38 - 1) * 10 ** 38 + 1]
    # capped scale with a Decimal128 result: Decimal(18,16) x Decimal(18,16) -> Decimal(36,30)
    q = tfa.arith(ctx, 2, torch.tensor([-123456789012345678], dtype=torch.int64, device=dev),
                  torch.tensor([3], dtype=torch.int64, device=dev), D128, a_type=D64, b_type=D64, a_scale=16,
                  b_scale=16, res_scale=30)
    assert _ints(D128, q) == [-(123456789012345678 * 3 // 100)]
