"""GPU parity of tfg_arith (a3: FunctionBinaryArithmetic / DecimalBinaryOperation,
Functions/FunctionBinaryArithmetic.h:72-215, 231-500) against the oracle's restatement
(oracle/oracle.c orc_arith) for every pair of numeric / decimal operand types, +, - and *,
vector-vector, vector-constant and constant-vector, with the edge values of every type.

Result types follow the reference: integers by NumberTraits (ResultOfAdditionMultiplication /
ResultOfSubtraction: the next wider integer, signed unless both are unsigned and the op is not
minus; 64-bit stays 64-bit, so the result wraps like the reference's native ops), any float
operand -> Float64, decimals by PlusDecimalInferer / MulDecimalInferer (Common/Decimal.h:109-163)
with integer operands as Decimal(IntPrec, 0) (:45-93).  Bit-exact for every type (float results
are single IEEE operations in double on both sides)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

I8, I16, I32, I64, U8, U16, U32, U64, F32, F64 = range(1, 11)
D32, D64, D128 = 11, 12, 13
NP = {I8: np.int8, I16: np.int16, I32: np.int32, I64: np.int64, U8: np.uint8, U16: np.uint16, U32: np.uint32,
      U64: np.uint64, F32: np.float32, F64: np.float64, D32: np.int32, D64: np.int64}
WIDTH = {I8: 1, I16: 2, I32: 4, I64: 8, U8: 1, U16: 2, U32: 4, U64: 8, F32: 4, F64: 8, D32: 4, D64: 8, D128: 16}
INT_PREC = {I8: 3, U8: 3, I16: 5, U16: 5, I32: 10, U32: 10, I64: 19, U64: 20}
# (type, precision, scale) of the decimal operands exercised
DECS = [(D32, 9, 2), (D64, 15, 2), (D64, 18, 4), (D128, 30, 3)]
N = 4099  # ragged: not a multiple of the 256-thread workgroup


def _int_result(op, a, b):
    signed = (a not in (U8, U16, U32, U64)) or (b not in (U8, U16, U32, U64)) or op == 1
    w = min(8, 2 * max(WIDTH[a], WIDTH[b]))
    return {(1, True): I8, (2, True): I16, (4, True): I32, (8, True): I64,
            (1, False): U8, (2, False): U16, (4, False): U32, (8, False): U64}[(w, signed)]


def _dec_result(op, pa, sa, pb, sb):
    if op == 2:
        p, s = min(pa + pb, 65), min(sa + sb, 30)
    else:
        s = max(sa, sb)
        p = min(max(pa - sa, pb - sb) + s + 1, 65)
    if p > 38:
        return None, p, s
    return (D32 if p <= 9 else D64 if p <= 18 else D128), p, s


def _values(t, n, rng, prec=None):
    if t == D128:
        lim = 10 ** prec
        vals = [int(x) for x in rng.integers(-2**62, 2**62, n)]
        vals = [v * (lim // 2**62 + 1) % lim * (1 if i % 3 else -1) for i, v in enumerate(vals)]
        vals[:3] = [lim - 1, -(lim - 1), 0]
        m = (1 << 128) - 1
        return np.array([[(v & m) & ((1 << 64) - 1), (v & m) >> 64] for v in vals], dtype=np.uint64).view(np.int64)
    dt = np.dtype(NP[t])
    if t in (F32, F64):
        x = (rng.standard_normal(n) * 1e6).astype(dt)
        x[:4] = [0.0, -0.0, np.finfo(dt).max, np.finfo(dt).tiny]
        return x
    if prec is not None:  # decimal payload below 10^prec
        lim = min(10 ** prec - 1, np.iinfo(dt).max)
        x = rng.integers(-lim, lim, n, dtype=dt, endpoint=True)
        x[:2] = [lim, -lim]
        return x
    info = np.iinfo(dt)
    x = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    x[:4] = [info.min, info.max, 0, 1 if info.min == 0 else -1]
    return x


def _operands():
    ops = [(t, None, 0) for t in (I8, I16, I32, I64, U8, U16, U32, U64, F32, F64)]
    return ops + [(t, p, s) for t, p, s in DECS]


def _cases():
    for ta, pa, sa in _operands():
        for tb, pb, sb in _operands():
            for op in (0, 1, 2):
                dec = pa is not None or pb is not None
                flt = ta in (F32, F64) or tb in (F32, F64)
                if dec and flt:
                    continue  # decimal with a float operand: ILLEGAL_TYPE_OF_ARGUMENT
                yield ta, pa, sa, tb, pb, sb, op


def _run_case(tfa, ctx, dev, orc, rng, ta, pa, sa, tb, pb, sb, op, mode):
    a = _values(ta, N, rng, pa)
    b = _values(tb, N, rng, pb)
    if pa is not None or pb is not None:
        rt, _, rs = _dec_result(op, pa if pa is not None else INT_PREC[ta], sa, pb if pb is not None else INT_PREC[tb], sb)
        if rt is None:
            return False  # Decimal256 result: tests/test_gpu_arith_wide.py
    elif ta in (F32, F64) or tb in (F32, F64):
        rt, rs = F64, 0
    else:
        rt, rs = _int_result(op, ta, tb), 0
    a_const, b_const = mode == 1, mode == 2
    if (a_const and ta == D128) or (b_const and tb == D128):
        return False  # the Python binding passes 8-byte host constants only
    ga = a[:1] if a_const else a
    gb = b[:1] if b_const else b
    pyval = lambda x, t: float(x[0]) if t in (F32, F64) else int(x[0])  # noqa: E731
    da = pyval(ga, ta) if a_const else torch.from_numpy(np.ascontiguousarray(ga)).to(dev)
    db = pyval(gb, tb) if b_const else torch.from_numpy(np.ascontiguousarray(gb)).to(dev)
    got = tfa.arith(ctx, op, da, db, rt, a_type=ta, b_type=tb, a_scale=sa, b_scale=sb, res_scale=rs, n=N, device=dev)
    exp = orc.arith(op, ga, gb, rt, a_type=ta, b_type=tb, a_const=a_const, b_const=b_const, a_scale=sa, b_scale=sb,
                    res_scale=rs, n=N)
    g = got.cpu().contiguous().numpy().view(np.uint8).reshape(-1)
    assert g.tobytes() == exp.tobytes(), (ta, pa, sa, tb, pb, sb, op, mode)
    return True


@pytest.mark.parametrize("mode", [0, 1, 2], ids=["vector_vector", "const_vector", "vector_const"])
def test_arith_every_type_pair(tfa, ctx, dev, orc, mode):
    rng = np.random.default_rng(100 + mode)
    ran = 0
    for case in _cases():
        ran += _run_case(tfa, ctx, dev, orc, rng, *case, mode)
    assert ran > 400


def test_arith_decimal_scale_alignment_known_values(tfa, ctx, dev):
    """applyScaled: Decimal(10,4) 1.2345 + Decimal(10,6) 0.000001 = 1.234501 (scale 6);
    * gives scale 10; Int64 7 + Decimal(15,2) 0.05 = 7.05."""
    a = torch.tensor([12345, -12345], dtype=torch.int64, device=dev)
    b = torch.tensor([1, 1], dtype=torch.int64, device=dev)
    p = tfa.arith(ctx, 0, a, b, D64, a_type=D64, b_type=D64, a_scale=4, b_scale=6, res_scale=6)
    assert p.cpu().tolist() == [1234501, -1234499]
    m = tfa.arith(ctx, 1, a, b, D64, a_type=D64, b_type=D64, a_scale=4, b_scale=6, res_scale=6)
    assert m.cpu().tolist() == [1234499, -1234501]
    x = tfa.arith(ctx, 2, a, b, D128, a_type=D64, b_type=D64, a_scale=4, b_scale=6, res_scale=10)
    assert x.cpu().numpy()[:, 0].tolist() == [12345, -12345] and x.cpu().numpy()[:, 1].tolist() == [0, -1]
    s = tfa.arith(ctx, 0, 7, torch.tensor([5], dtype=torch.int64, device=dev), D64, a_type=I64, b_type=D64,
                  a_scale=0, b_scale=2, res_scale=2)
    assert s.cpu().tolist() == [705]


def test_arith_rejects_float_decimal(tfa, ctx, dev):
    a = torch.zeros(4, dtype=torch.int64, device=dev)
    f = torch.zeros(4, dtype=torch.float64, device=dev)
    with pytest.raises(tfa.TfgError):
        tfa.arith(ctx, 0, a, f, D64, a_type=D64, b_type=F64)
