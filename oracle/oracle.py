"""ctypes wrapper of oracle/liboracle.so — the CPU restatement of the reference's hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / CPU baseline, never by the product (tiflash_amd/).
Arrays are numpy arrays in host memory.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(_HERE, "liboracle.so")
_L = None

INT8, INT16, INT32, INT64, UINT8, UINT16, UINT32, UINT64, FLOAT32, FLOAT64 = range(1, 11)
DECIMAL32, DECIMAL64, DECIMAL128, DECIMAL256 = 11, 12, 13, 14
STRING = 20
NULLABLE = 0x100
AGG_SUM, AGG_COUNT, AGG_COUNT_ALL, AGG_MIN, AGG_MAX, AGG_FIRST_ROW = range(6)
NP_DTYPE = {INT8: np.int8, INT16: np.int16, INT32: np.int32, INT64: np.int64, UINT8: np.uint8, UINT16: np.uint16,
            UINT32: np.uint32, UINT64: np.uint64, FLOAT32: np.float32, FLOAT64: np.float64, DECIMAL32: np.int32,
            DECIMAL64: np.int64}


def prec(t: int, p: int) -> int:
    """Aggregate argument type word of a Decimal column with precision p (TFG_ARG_PREC)."""
    return t | (p << 16)


def sum_result_prec(t: int) -> int:
    """SumDecimalInferer (Common/Decimal.h:156-163): min(p + 22, 65); 0 for non-decimal args."""
    return lib().orc_sum_result_prec(int(t) & ~NULLABLE)


def sum_limbs(kind: int, t: int) -> int:
    """Words of a sum result: 1 (Int64 / UInt64 / Float64), 2 (Decimal128) or 4 (Decimal256)."""
    base = t & 0xFF
    if kind != 0 or base not in (DECIMAL32, DECIMAL64, DECIMAL128, DECIMAL256):
        return 1
    return 4 if sum_result_prec(t) > 38 else 2


def limbs_to_int(row) -> int:
    """Little-endian two's complement 64-bit limbs -> Python int."""
    v = 0
    for i, w in enumerate(row):
        v |= (int(w) & ((1 << 64) - 1)) << (64 * i)
    bits = 64 * len(row)
    return v - (1 << bits) if v >> (bits - 1) else v


def int_to_limbs(v: int, n: int) -> np.ndarray:
    m = v & ((1 << (64 * n)) - 1)
    return np.array([(m >> (64 * i)) & ((1 << 64) - 1) for i in range(n)], dtype=np.uint64).view(np.int64)
NP_TYPE = {np.dtype(np.int8): INT8, np.dtype(np.int16): INT16, np.dtype(np.int32): INT32, np.dtype(np.int64): INT64,
           np.dtype(np.uint8): UINT8, np.dtype(np.uint16): UINT16, np.dtype(np.uint32): UINT32,
           np.dtype(np.uint64): UINT64, np.dtype(np.float32): FLOAT32, np.dtype(np.float64): FLOAT64}


def build():
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)


def lib():
    global _L
    if _L is None:
        if not os.path.exists(_PATH):
            build()
        L = ctypes.CDLL(_PATH)
        L.orc_crc32c_u64.restype = ctypes.c_uint32
        L.orc_crc32c_u64.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
        L.orc_crc32c_u64_sw.restype = ctypes.c_uint32
        L.orc_crc32c_u64_sw.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
        L.orc_update_weak_hash32_bytes.restype = ctypes.c_uint32
        L.orc_update_weak_hash32_bytes.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
        L.orc_count_bytes_in_filter.restype = ctypes.c_size_t
        L.orc_filter.restype = ctypes.c_size_t
        L.orc_filter_string.restype = ctypes.c_size_t
        L.orc_agg_create.restype = ctypes.c_void_p
        L.orc_agg_size.restype = ctypes.c_size_t
        L.orc_agg_size.argtypes = [ctypes.c_void_p]
        L.orc_agg_destroy.argtypes = [ctypes.c_void_p]
        L.orc_aggk_create.restype = ctypes.c_void_p
        L.orc_aggk_destroy.argtypes = [ctypes.c_void_p]
        L.orc_aggk_size.restype = ctypes.c_size_t
        L.orc_aggk_size.argtypes = [ctypes.c_void_p]
        L.orc_aggk_result.restype = ctypes.c_size_t
        L.orc_agg_result_chars.restype = ctypes.c_size_t
        L.orc_agg_result_chars.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_aggk_result_chars.restype = ctypes.c_size_t
        L.orc_aggk_result_chars.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_min_max_str_compare.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                              ctypes.c_size_t]
        L.orc_join_create.restype = ctypes.c_void_p
        L.orc_join_destroy.argtypes = [ctypes.c_void_p]
        L.orc_join_probe.restype = ctypes.c_size_t
        L.orc_bench_filter_agg.restype = ctypes.c_size_t
        L.orc_bench_join.restype = ctypes.c_size_t
        L.orc_bench_filter_agg_ref.restype = ctypes.c_size_t
        L.orc_bench_string_agg.restype = ctypes.c_size_t
        L.orc_join_ref_build.restype = ctypes.c_void_p
        L.orc_join_ref_probe.restype = ctypes.c_size_t
        L.orc_join_ref_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_int, ctypes.c_void_p]
        L.orc_join_ref_destroy.argtypes = [ctypes.c_void_p]
        L.orc_codec_encode.restype = ctypes.c_size_t
        L.orc_codec_decode_strings.restype = ctypes.c_size_t
        L.orc_lz4_decompress_block.restype = ctypes.c_int64
        L.orc_lz4_decompress_block.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        L.orc_lz4_bound.restype = ctypes.c_size_t
        L.orc_lz4_bound.argtypes = [ctypes.c_size_t]
        L.orc_lz4_compress_block.restype = ctypes.c_size_t
        L.orc_lz4_compress_block.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_lz4_packet_compress.restype = ctypes.c_size_t
        L.orc_lz4_packet_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_lz4_packet_decompress.restype = ctypes.c_int64
        L.orc_lz4_packet_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        _L = L
    return _L


def _p(a):
    return ctypes.c_void_p(0) if a is None else a.ctypes.data_as(ctypes.c_void_p)


class _StrCol(ctypes.Structure):  # orc_str_col / orc_str_out: a String column's chars + end offsets
    _fields_ = [("chars", ctypes.c_void_p), ("offsets", ctypes.c_void_p)]


def _ptrs(arrs):
    """Pointer array of numpy arrays; a (chars, offsets) pair becomes a host orc_str_col (kept alive
    on the array object)."""
    out = (ctypes.c_void_p * max(1, len(arrs)))()
    keep = []
    for i, a in enumerate(arrs):
        if isinstance(a, (tuple, list)):
            c, o = np.ascontiguousarray(a[0], dtype=np.uint8), np.ascontiguousarray(a[1], dtype=np.uint64)
            sc = _StrCol(c.ctypes.data, o.ctypes.data)
            keep += [c, o, sc]
            out[i] = ctypes.addressof(sc)
        else:
            out[i] = 0 if a is None else a.ctypes.data
    out._keep = keep
    return out


def type_of(a: np.ndarray) -> int:
    return NP_TYPE[a.dtype]


def crc32c_u64(crc: int, x: int) -> int:
    return lib().orc_crc32c_u64(crc, x & 0xFFFFFFFFFFFFFFFF)


def crc32c_u64_sw(crc: int, x: int) -> int:
    return lib().orc_crc32c_u64_sw(crc, x & 0xFFFFFFFFFFFFFFFF)


def weak_hash(cols, types=None, nullmaps=None, h=None) -> np.ndarray:
    n = len(cols[0])
    if h is None:
        h = np.full(n, 0xFFFFFFFF, dtype=np.uint32)
    for j, c in enumerate(cols):
        c = np.ascontiguousarray(c)
        t = types[j] if types else type_of(c)
        nm = None if not nullmaps or nullmaps[j] is None else np.ascontiguousarray(nullmaps[j], dtype=np.uint8)
        lib().orc_weak_hash_update(t, _p(c), _p(nm), ctypes.c_size_t(n), _p(h))
    return h


def weak_hash_string(chars: np.ndarray, offsets: np.ndarray, h: np.ndarray, nullmap=None, collator=0):
    lib().orc_weak_hash_update_string(_p(chars), _p(offsets), _p(nullmap), ctypes.c_size_t(len(offsets)), collator,
                                      _p(h))
    return h


def fill_selector(h: np.ndarray, part_num: int, fgs: int = 0) -> np.ndarray:
    sel = np.empty(len(h), dtype=np.uint32)
    lib().orc_fill_selector(_p(h), ctypes.c_size_t(len(h)), ctypes.c_uint32(part_num), ctypes.c_uint32(fgs), _p(sel))
    return sel


def partition(sel: np.ndarray, parts: int):
    perm = np.empty(len(sel), dtype=np.uint32)
    offs = np.empty(parts + 1, dtype=np.uint64)
    lib().orc_partition(_p(sel), ctypes.c_size_t(len(sel)), ctypes.c_uint32(parts), _p(perm), _p(offs))
    return perm, offs


def cmp(a, op, b, a_type=None, b_type=None, a_const=False, b_const=False, a_null=None, b_null=None, n=None):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    n = n if n is not None else (len(b) if a_const else len(a))
    out = np.empty(n, dtype=np.uint8)
    lib().orc_cmp(a_type or type_of(a), _p(a), int(a_const), op, b_type or type_of(b), _p(b), int(b_const),
                  _p(a_null), _p(b_null), ctypes.c_size_t(n), _p(out))
    return out


def count_bytes_in_filter(f: np.ndarray, nullmap=None) -> int:
    return lib().orc_count_bytes_in_filter(_p(f), _p(nullmap), ctypes.c_size_t(len(f)))


def filter(col: np.ndarray, f: np.ndarray) -> np.ndarray:  # noqa: A001
    col = np.ascontiguousarray(col)
    out = np.empty_like(col)
    width = col.dtype.itemsize * (col.shape[1] if col.ndim == 2 else 1)
    k = lib().orc_filter(width, _p(col), _p(f), ctypes.c_size_t(len(f)), _p(out))
    return out[:k]


def filter_string(chars, offsets, f):
    out_chars = np.empty(max(1, len(chars)), dtype=np.uint8)
    out_offsets = np.empty(max(1, len(offsets)), dtype=np.uint64)
    nbytes = ctypes.c_size_t()
    rows = lib().orc_filter_string(_p(chars), _p(offsets), _p(f), ctypes.c_size_t(len(f)), _p(out_chars),
                                   _p(out_offsets), ctypes.byref(nbytes))
    return out_chars[:nbytes.value], out_offsets[:rows]


def arith(op, a, b, res_type, a_type=None, b_type=None, a_const=False, b_const=False, a_scale=0, b_scale=0,
          res_scale=0, n=None):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    n = n if n is not None else (len(b) if a_const else len(a))
    width = {1: 1, 2: 2, 3: 4, 4: 8, 5: 1, 6: 2, 7: 4, 8: 8, 9: 4, 10: 8, 11: 4, 12: 8, 13: 16}[res_type]
    out = np.zeros(n * width, dtype=np.uint8)
    rc = lib().orc_arith(op, a_type or type_of(a), _p(a), int(a_const), a_scale, b_type or type_of(b), _p(b),
                         int(b_const), b_scale, res_type, res_scale, ctypes.c_size_t(n), _p(out))
    assert rc == 0
    return out


def arith_decimal_wide(op, a, b, a_type, b_type, a_scale, b_scale, res_type, res_scale):
    """Decimal arithmetic with exact integers (Python ints in, Python ints out) for Decimal256
    results / operands and multiplies with a capped result scale: DecimalBinaryOperation
    (Functions/FunctionBinaryArithmetic.h:231-640).  +/-: the operand of lower scale is scaled up to
    the result scale (DataTypeDecimal::getScales, DataTypes/DataTypeDecimal.h:96-123, applyScaled);
    *: the raw product divided by 10^(sa + sb - res_scale), truncating toward zero (applyScaledMul).
    A Decimal256 result must fit Int256 (boost checked_int256_t, common/types.h:35), and when an
    operand is Decimal256 too (need_promote_type) must not exceed 10^65 - 1 (check_overflow,
    DecimalMaxValue): else OverflowError, the reference's DECIMAL_OVERFLOW.  Small inputs only
    (pure Python)."""
    dec = (11, 12, 13, 14)
    sa = a_scale if a_type in dec else 0
    sb = b_scale if b_type in dec else 0
    promote = res_type == 14 and 14 in (a_type, b_type)
    out = []
    for x, y in zip(a, b):
        if op == 2:
            r = x * y
            k = 10 ** (sa + sb - res_scale)
            r = abs(r) // k * (1 if r >= 0 else -1)
        else:
            x *= 10 ** (res_scale - sa)
            y *= 10 ** (res_scale - sb)
            r = x + y if op == 0 else x - y
        if res_type == 14 and (not -(1 << 255) <= r < (1 << 255) or (promote and r > 10 ** 65 - 1)):
            raise OverflowError("Decimal math overflow")
        out.append(r)
    return out


def _ord_state(h, i, t, g, strs, keys_agg=False):
    """Result buffer of a min / max / first_row state: the argument's type; Decimal128 / Decimal256
    as (g, 2 / 4) int64 limbs; a String as a (chars, offsets) pair (recorded in strs[i])."""
    base = t & 0xFF
    if base == STRING:
        nb = (lib().orc_aggk_result_chars if keys_agg else lib().orc_agg_result_chars)(h, i)
        c, o = np.zeros(max(nb, 1), np.uint8), np.zeros(max(g, 1), np.uint64)
        strs[i] = (c[:nb], o[:g])
        return (c, o)
    if base in (DECIMAL128, DECIMAL256):
        return np.zeros((max(g, 1), 2 if base == DECIMAL128 else 4), np.int64)
    return np.zeros(max(g, 1), NP_DTYPE[base])


class Agg:
    """Reference-semantics Aggregator (HashMap key64 + sum/count states)."""

    def __init__(self, key_type: int, aggs):
        kinds = (ctypes.c_int * len(aggs))(*[k for k, _ in aggs])
        types = (ctypes.c_int * len(aggs))(*[t & ~NULLABLE for _, t in aggs])
        self.aggs = list(aggs)
        self.h = ctypes.c_void_p(lib().orc_agg_create(key_type, len(aggs), kinds, types))
        self.key_type = key_type

    def consume(self, keys, args, key_null=None, arg_nulls=None, mask=None, n=None):
        if n is None:
            if keys is not None:
                n = len(keys)
            else:
                a0 = next(a for a in args if a is not None)
                n = len(a0[1]) if isinstance(a0, (tuple, list)) else len(a0)
        lib().orc_agg_consume(self.h, _p(keys), _p(key_null), _ptrs(args), _ptrs(arg_nulls) if arg_nulls else None,
                              _p(mask), ctypes.c_size_t(n))

    def merge(self, other: "Agg"):
        lib().orc_agg_merge(self.h, other.h)

    def size(self) -> int:
        return lib().orc_agg_size(self.h)

    def result(self):
        g = self.size()
        keys = np.empty(g, dtype=np.uint64)
        key_null = np.empty(g, dtype=np.uint8)
        states, snull = [], []
        strs = {}
        for i, (kind, t) in enumerate(self.aggs):
            limbs = sum_limbs(kind, t)
            if kind in (AGG_MIN, AGG_MAX, AGG_FIRST_ROW):  # the argument's type
                states.append(_ord_state(self.h, i, t, g, strs))
            elif kind != 0:
                states.append(np.empty(g, dtype=np.uint64))
            elif (t & 0xFF) in (FLOAT32, FLOAT64):
                states.append(np.empty(g, dtype=np.float64))
            elif limbs > 1:
                states.append(np.empty((g, limbs), dtype=np.int64))
            else:
                states.append(np.empty(g, dtype=np.int64))
            snull.append(np.empty(g, dtype=np.uint8))
        lib().orc_agg_result(self.h, _p(keys), _p(key_null), _ptrs(states), _ptrs(snull))
        for i, (c, o) in strs.items():
            states[i] = (c, o)
        return {"keys": keys, "key_null": key_null, "states": states, "state_null": snull}

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_agg_destroy(self.h)
            self.h = None


_SIGNED = {INT8, INT16, INT32, INT64, DECIMAL32, DECIMAL64, DECIMAL128, DECIMAL256}
_KW = {INT8: 1, INT16: 2, INT32: 4, INT64: 8, UINT8: 1, UINT16: 2, UINT32: 4, UINT64: 8, FLOAT32: 4, FLOAT64: 8,
       DECIMAL32: 4, DECIMAL64: 8, DECIMAL128: 16, DECIMAL256: 32}


class AggKeys:
    """orc_aggk: GROUP BY several keys or one String key (keys128 / key_string / serialized).
    A String key column is a (chars uint8, offsets uint64) pair.  result() returns the groups as
    (key tuple, [state_i]) with key values int / bytes / None (NULL)."""

    def __init__(self, key_types, aggs, collators=None):
        self.key_types = list(key_types)
        self.aggs = list(aggs)
        kt = (ctypes.c_int * len(key_types))(*key_types)
        co = (ctypes.c_int * len(key_types))(*(collators or [0] * len(key_types)))
        kinds = (ctypes.c_int * len(aggs))(*[k for k, _ in aggs])
        types = (ctypes.c_int * len(aggs))(*[t & ~NULLABLE for _, t in aggs])
        self.h = ctypes.c_void_p(lib().orc_aggk_create(len(key_types), kt, co, len(aggs), kinds, types))

    def consume(self, keys, args, key_nulls=None, arg_nulls=None, mask=None):
        cols, offs = [], []
        for t, k in zip(self.key_types, keys):
            if t == STRING:
                cols.append(np.ascontiguousarray(k[0]))
                offs.append(np.ascontiguousarray(k[1], dtype=np.uint64))
            else:
                cols.append(np.ascontiguousarray(k))
                offs.append(None)
        n = len(offs[0]) if self.key_types[0] == STRING else cols[0].nbytes // _KW[self.key_types[0]]
        self._keep = (cols, offs, args, key_nulls, arg_nulls, mask)
        lib().orc_aggk_consume(self.h, _ptrs(cols), _ptrs(offs), _ptrs(key_nulls) if key_nulls else None, _ptrs(args),
                               _ptrs(arg_nulls) if arg_nulls else None, _p(mask), ctypes.c_size_t(n))

    def size(self) -> int:
        return lib().orc_aggk_size(self.h)

    def _decode(self, b: bytes):
        out, o = [], 0
        for t in self.key_types:
            isnull = b[o]
            o += 1
            if isnull:
                out.append(None)
                continue
            if t == STRING:
                ln = int.from_bytes(b[o:o + 8], "little")
                out.append(bytes(b[o + 8:o + 8 + ln]))
                o += 8 + ln
            else:
                w = _KW[t]
                if t in (FLOAT32, FLOAT64):
                    out.append(float(np.frombuffer(b[o:o + w], np.float32 if t == FLOAT32 else np.float64)[0]))
                else:
                    out.append(int.from_bytes(b[o:o + w], "little", signed=t in _SIGNED))
                o += w
        return tuple(out)

    def result_arrays(self):
        """-> (key bytes, key end offsets, [state arrays], [state null arrays]) without building
        Python tuples: the serialised keys (per key a NULL byte, then the value bytes, or a String's
        u64 length + bytes) for callers that decode millions of groups with numpy."""
        g = self.size()
        total = lib().orc_aggk_result(self.h, None, None, None, None)
        kb = np.zeros(max(total, 1), np.uint8)
        ko = np.zeros(max(g, 1), np.uint64)
        states, snull = [], []
        strs = {}
        for i, (kind, t) in enumerate(self.aggs):
            limbs = sum_limbs(kind, t)
            if kind in (AGG_MIN, AGG_MAX, AGG_FIRST_ROW):  # the argument's type
                states.append(_ord_state(self.h, i, t, g, strs, keys_agg=True))
                snull.append(np.zeros(max(g, 1), np.uint8))
                continue
            t &= 0xFF
            if limbs > 1:
                states.append(np.zeros((max(g, 1), limbs), np.int64))
            elif kind == 0 and t in (FLOAT32, FLOAT64):
                states.append(np.zeros(max(g, 1), np.float64))
            else:
                states.append(np.zeros(max(g, 1), np.int64))
            snull.append(np.zeros(max(g, 1), np.uint8))
        lib().orc_aggk_result(self.h, _p(kb), _p(ko), _ptrs(states), _ptrs(snull))
        for i, co in strs.items():
            states[i] = co
        return kb[:total], ko[:g], [st if i in strs else st[:g] for i, st in enumerate(states)], [sn[:g] for sn in snull]

    def result(self):
        g = self.size()
        total = lib().orc_aggk_result(self.h, None, None, None, None)
        kb = np.zeros(max(total, 1), np.uint8)
        ko = np.zeros(max(g, 1), np.uint64)
        states, snull = [], []
        strs = {}
        for i, (kind, t) in enumerate(self.aggs):
            limbs = sum_limbs(kind, t)
            if kind in (AGG_MIN, AGG_MAX, AGG_FIRST_ROW):  # the argument's type
                states.append(_ord_state(self.h, i, t, g, strs, keys_agg=True))
                snull.append(np.zeros(max(g, 1), np.uint8))
                continue
            t &= 0xFF
            if limbs > 1:
                states.append(np.zeros((max(g, 1), limbs), np.int64))
            elif kind == 0 and t in (FLOAT32, FLOAT64):
                states.append(np.zeros(max(g, 1), np.float64))
            else:
                states.append(np.zeros(max(g, 1), np.int64))
            snull.append(np.zeros(max(g, 1), np.uint8))
        lib().orc_aggk_result(self.h, _p(kb), _p(ko), _ptrs(states), _ptrs(snull))
        groups = []
        s = 0
        for i in range(g):
            e = int(ko[i])
            key = self._decode(kb[s:e].tobytes())
            s = e
            vals = []
            for j, st in enumerate(states):
                if j in strs:  # String min / max / first_row: the value's bytes without the '\0'
                    c, o = strs[j]
                    vals.append(bytes(c[(int(o[i - 1]) if i else 0):int(o[i]) - 1]))
                    continue
                v = st[i]
                vals.append(limbs_to_int(v) if st.ndim == 2 else v.item())
            groups.append((key, vals))
        return groups

    def __del__(self):
        try:
            lib().orc_aggk_destroy(self.h)
        except Exception:
            pass


class JoinRef:
    def __init__(self, key_type: int):
        self.h = ctypes.c_void_p(lib().orc_join_create(key_type))

    def build(self, keys, key_null=None):
        keys = np.ascontiguousarray(keys)
        lib().orc_join_build(self.h, _p(keys), _p(key_null), ctypes.c_size_t(len(keys)))

    def probe(self, keys, kind=0, key_null=None):
        keys = np.ascontiguousarray(keys)
        n = len(keys)
        total = lib().orc_join_probe(self.h, kind, _p(keys), _p(key_null), ctypes.c_size_t(n), None, None,
                                     ctypes.c_size_t(0))
        pi = np.empty(max(total, 1), dtype=np.uint32)
        bi = np.empty(max(total, 1), dtype=np.uint32)
        lib().orc_join_probe(self.h, kind, _p(keys), _p(key_null), ctypes.c_size_t(n), _p(pi), _p(bi),
                             ctypes.c_size_t(total))
        return pi[:total], bi[:total]

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_join_destroy(self.h)
            self.h = None


def bench_filter_agg(f, threshold, k, v, nthreads, block_rows=65536):
    cs = ctypes.c_double()
    g = lib().orc_bench_filter_agg(_p(f), ctypes.c_int64(threshold), _p(k), _p(v), ctypes.c_size_t(len(k)),
                                   nthreads, ctypes.c_size_t(block_rows), ctypes.byref(cs))
    return g, cs.value


def bench_filter_agg_ref(f, threshold, k, v, nthreads, block_rows=65536):
    cs = ctypes.c_double()
    g = lib().orc_bench_filter_agg_ref(_p(f), ctypes.c_int64(threshold), _p(k), _p(v), ctypes.c_size_t(len(k)),
                                       nthreads, ctypes.c_size_t(block_rows), ctypes.byref(cs))
    return g, cs.value


class JoinBench:
    """C3 CPU leg: build once (timed separately), probe + materialise timed by the caller."""

    def __init__(self, build_keys, build_pay, nthreads):
        self.bk, self.bp = np.ascontiguousarray(build_keys), np.ascontiguousarray(build_pay)
        self.threads = nthreads
        self.h = ctypes.c_void_p(lib().orc_join_ref_build(_p(self.bk), _p(self.bp), ctypes.c_size_t(len(self.bk)),
                                                          nthreads))

    def probe(self, probe_keys, probe_pay):
        cs = ctypes.c_uint64()
        m = lib().orc_join_ref_probe(self.h, _p(probe_keys), _p(probe_pay), ctypes.c_size_t(len(probe_keys)),
                                     self.threads, ctypes.byref(cs))
        return m, cs.value

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_join_ref_destroy(self.h)
            self.h = None


def bench_string_agg(chars, offsets, v, nthreads, block_rows=65536):
    """C5 partial aggregation on the CPU (cpu_baseline_str.c) -> (groups, sum of counts)."""
    cs = ctypes.c_uint64()
    g = lib().orc_bench_string_agg(_p(chars), _p(offsets), _p(v), ctypes.c_size_t(len(v)), nthreads,
                                   ctypes.c_size_t(block_rows), ctypes.byref(cs))
    return g, cs.value


def bench_join(build_keys, probe_keys, nthreads):
    cs = ctypes.c_uint64()
    m = lib().orc_bench_join(_p(build_keys), ctypes.c_size_t(len(build_keys)), _p(probe_keys),
                             ctypes.c_size_t(len(probe_keys)), nthreads, ctypes.byref(cs))
    return m, cs.value


# ---- (f1) MPP packet codec (oracle/codec.c) --------------------------------------------------
CODEC_CHBLOCK, CODEC_V1 = 0, 1


def codec_encode(columns, n, version=CODEC_V1, part_rows=None) -> bytes:
    """CHBlockChunkCodec(V1) encode of host columns: (name, type_name, data, offsets, nullmap)."""
    nc = len(columns)
    names = (ctypes.c_char_p * max(nc, 1))(*[c[0].encode() for c in columns])
    types = (ctypes.c_char_p * max(nc, 1))(*[c[1].encode() for c in columns])
    keep = [np.ascontiguousarray(x) if x is not None else None for c in columns for x in c[2:5]]
    data = _ptrs([keep[3 * i] for i in range(nc)])
    offs = _ptrs([keep[3 * i + 1] for i in range(nc)])
    nms = _ptrs([keep[3 * i + 2] for i in range(nc)])
    np_ = len(part_rows) if part_rows else 0
    pr = (ctypes.c_int64 * max(np_, 1))(*(part_rows or [0]))
    L = lib()
    size = L.orc_codec_encode(version, nc, names, types, data, offs, nms, ctypes.c_int64(n), np_, pr, None,
                              ctypes.c_size_t(0))
    assert size != ctypes.c_size_t(-1).value, "unsupported type"
    out = np.zeros(max(size, 1), np.uint8)
    got = L.orc_codec_encode(version, nc, names, types, data, offs, nms, ctypes.c_int64(n), np_, pr, _p(out),
                             ctypes.c_size_t(out.size))
    assert got == size
    return out[:size].tobytes()


def codec_decode_strings(buf: bytes, rows: int, chars_cap: int):
    """Legacy String bulk decode -> (chars with terminators, end offsets, bytes consumed)."""
    src = np.frombuffer(buf, np.uint8)
    chars = np.zeros(max(chars_cap, 1), np.uint8)
    offs = np.zeros(max(rows, 1), np.uint64)
    used = lib().orc_codec_decode_strings(_p(src), ctypes.c_size_t(src.size), ctypes.c_int64(rows), _p(chars),
                                          _p(offs))
    assert used != ctypes.c_size_t(-1).value, "truncated"
    return chars[:int(offs[rows - 1]) if rows else 0], offs[:rows], used


# ---- (f1) LZ4 packets (oracle/lz4.c) ---------------------------------------------------------
def lz4_decompress_block(block: bytes, raw_cap: int):
    """LZ4_decompress_safe restated: decoded bytes, or None when the block is malformed."""
    src = np.frombuffer(block, np.uint8) if block else np.zeros(1, np.uint8)
    dst = np.zeros(max(raw_cap, 1), np.uint8)
    got = lib().orc_lz4_decompress_block(_p(src), len(block), _p(dst), raw_cap)
    return None if got < 0 else dst[:got].tobytes()


def lz4_compress_block(raw: bytes) -> bytes:
    src = np.frombuffer(raw, np.uint8) if raw else np.zeros(1, np.uint8)
    dst = np.zeros(lib().orc_lz4_bound(len(raw)), np.uint8)
    n = lib().orc_lz4_compress_block(_p(src), len(raw), _p(dst))
    return dst[:n].tobytes()


def lz4_packet_compress(packet: bytes, frame_raw: int = 0) -> bytes:
    """Uncompressed V1 packet (0x02 + body) -> LZ4 frames of frame_raw body bytes (0: one frame)."""
    src = np.frombuffer(packet, np.uint8)
    L = lib()
    cap = L.orc_lz4_packet_compress(_p(src), src.size, frame_raw, None)
    out = np.zeros(max(cap, 1), np.uint8)
    n = L.orc_lz4_packet_compress(_p(src), src.size, frame_raw, _p(out))
    return out[:n].tobytes()


def lz4_packet_decompress(packet: bytes):
    """LZ4 frames -> the uncompressed V1 packet (0x02 + body); None when malformed."""
    src = np.frombuffer(packet, np.uint8) if packet else np.zeros(1, np.uint8)
    L = lib()
    size = L.orc_lz4_packet_decompress(_p(src), len(packet), None, 0)
    if size < 0:
        return None
    out = np.zeros(size, np.uint8)
    got = L.orc_lz4_packet_decompress(_p(src), len(packet), _p(out), size)
    return None if got < 0 else out.tobytes()
