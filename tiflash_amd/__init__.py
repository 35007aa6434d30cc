"""tiflash_amd — MI355X (gfx950) execution layer for TiFlash's Block/Column hot path.

This Python module is plumbing only: it loads ``libtiflash_amd.so`` (hand-written HIP kernels
behind the C-ABI declared in ``include/tiflash_amd.h``) with ctypes and passes device pointers
of torch tensors.  There is no CPU fallback: every entry point goes through the HIP library and
raises if it is missing.  The C++ operator layer that mirrors the reference's
FilterTransformAction / Aggregator / Join / HashPartitionWriter lives in ``tiflash_amd/host``.
"""
from __future__ import annotations

import ctypes
import os
import sys
import weakref
from typing import Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
# TFA_LIB_PATH: an instrumented build of the same library (profiling experiments, tools/)
LIB_PATH = os.environ.get("TFA_LIB_PATH") or os.path.join(_HERE, "libtiflash_amd.so")

# ---- constants mirrored from include/tiflash_amd.h --------------------------------------------
TFG_OK = 0
ERRORS = {
    -1: "INVALID_ARG", -2: "HIP", -3: "OOM", -4: "NOT_IMPLEMENTED", -5: "SIZE_MISMATCH",
    -6: "ILLEGAL_TYPE", -7: "LOGICAL", -8: "CAPACITY", -9: "NO_DEVICE", -10: "FAULT_INJECTED", -11: "OVERFLOW",
}
TFG_ERR_NOT_IMPLEMENTED = -4
TFG_ERR_CAPACITY = -8
TFG_ERR_NO_DEVICE = -9
TFG_ERR_OVERFLOW = -11

INT8, INT16, INT32, INT64, UINT8, UINT16, UINT32, UINT64, FLOAT32, FLOAT64 = range(1, 11)
DECIMAL32, DECIMAL64, DECIMAL128, DECIMAL256 = 11, 12, 13, 14
STRING, KEYS128 = 20, 21  # String GROUP BY keys (chars, offsets); packed 16-byte key (tfg_agg_create_keys)
NULLABLE = 0x100  # or-ed into an aggregate argument type: the argument may carry a null map


def collate(t: int, c: int) -> int:
    """Aggregate argument type word of a String min / max argument under collator c
    (TFG_ARG_COLLATOR): SingleValueDataString compares with the collator."""
    return t | (int(c) << 24)


def prec(t: int, p: int) -> int:
    """Aggregate argument type word of a Decimal column of precision p (TFG_ARG_PREC): sum over
    Decimal(p, s) returns Decimal(min(p + 22, 65), s) — Decimal128 up to 38 digits, else
    Decimal256 (4 int64 limbs per value).  Without it the type's maximum precision is assumed."""
    return t | (int(p) << 16)

EQ, NE, LT, LE, GT, GE = range(6)
PLUS, MINUS, MULTIPLY = range(3)
AND, OR, NOT = range(3)
AGG_SUM, AGG_COUNT, AGG_COUNT_ALL, AGG_MIN, AGG_MAX, AGG_FIRST_ROW = range(6)
JOIN_INNER, JOIN_LEFT, JOIN_SEMI, JOIN_ANTI = range(4)
JOIN_V2_TAGGED = 1  # tfg_join_create_v2 flags
COLLATOR_NONE, COLLATOR_BINARY, COLLATOR_BIN_PADDING, COLLATOR_GENERAL_CI, COLLATOR_UNICODE_CI, COLLATOR_UCA0900_AI_CI = range(6)

WIDTH = {INT8: 1, INT16: 2, INT32: 4, INT64: 8, UINT8: 1, UINT16: 2, UINT32: 4, UINT64: 8,
         FLOAT32: 4, FLOAT64: 8, DECIMAL32: 4, DECIMAL64: 8, DECIMAL128: 16, DECIMAL256: 32, KEYS128: 16}
_CTYPE = {INT8: ctypes.c_int8, INT16: ctypes.c_int16, INT32: ctypes.c_int32, INT64: ctypes.c_int64,
          UINT8: ctypes.c_uint8, UINT16: ctypes.c_uint16, UINT32: ctypes.c_uint32, UINT64: ctypes.c_uint64,
          FLOAT32: ctypes.c_float, FLOAT64: ctypes.c_double, DECIMAL32: ctypes.c_int32,
          DECIMAL64: ctypes.c_int64}


class TfgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"tfg error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


_lib = None


def lib() -> ctypes.CDLL:
    """The HIP library.  Raises (never falls back) when it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        # torch first: the library then binds to the HIP runtime torch already loaded (one
        # runtime per process; loading ours first made torch see no device)
        import torch  # noqa: F401
        L = ctypes.CDLL(LIB_PATH)
        L.tfg_last_error.restype = ctypes.c_char_p
        L.tfg_version.restype = ctypes.c_char_p
        L.tfg_type_width.restype = ctypes.c_size_t
        L.tfg_type_width.argtypes = [ctypes.c_int]
        L.tfg_codec_compress_bound.restype = ctypes.c_size_t
        L.tfg_codec_compress_bound.argtypes = [ctypes.c_size_t]
        _lib = L
    return _lib


def check(rc: int) -> int:
    if rc != TFG_OK:
        raise TfgError(rc, lib().tfg_last_error().decode(errors="replace"))
    return rc


def _p(t) -> ctypes.c_void_p:
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(t.data_ptr())


def _ptr_array(ts) -> ctypes.Array:
    arr = (ctypes.c_void_p * max(1, len(ts)))()
    for i, t in enumerate(ts):
        arr[i] = t.data_ptr() if t is not None else 0
    return arr


class _StrCol(ctypes.Structure):  # tfg_str_col
    _fields_ = [("chars", ctypes.c_void_p), ("offsets", ctypes.c_void_p)]


class _StrOut(ctypes.Structure):  # tfg_str_out
    _fields_ = [("chars", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("chars_capacity", ctypes.c_uint64)]


def _arg_array(ts):
    """Aggregate arguments / partial states: a tensor, None, or a String column as a (chars, offsets)
    tensor pair, passed as a host tfg_str_col.  Returns (array, keep-alive list)."""
    arr = (ctypes.c_void_p * max(1, len(ts)))()
    keep = []
    for i, t in enumerate(ts):
        if isinstance(t, (tuple, list)):
            sc = _StrCol(t[0].data_ptr(), t[1].data_ptr())
            keep.append(sc)
            arr[i] = ctypes.addressof(sc)
        else:
            arr[i] = t.data_ptr() if t is not None else 0
    return arr, keep


def _agg_states(h, n_aggs: int, g: int, dev):
    """Result buffers of an aggregator's states: (pointer array, keep-alive, finish) — finish()
    returns the state list (a String state as a (chars, offsets) pair)."""
    import torch
    arr = (ctypes.c_void_p * max(1, n_aggs))()
    keep, outs = [], []
    for i in range(n_aggs):
        t, w = ctypes.c_int(), ctypes.c_int()
        check(lib().tfg_agg_result_type(h, i, ctypes.byref(t), ctypes.byref(w)))
        if t.value == STRING:
            nb = ctypes.c_uint64()
            check(lib().tfg_agg_result_chars(h, i, ctypes.byref(nb)))
            chars = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=dev)
            offs = torch.empty(max(g, 1), dtype=torch.int64, device=dev)
            so = _StrOut(chars.data_ptr(), offs.data_ptr(), nb.value)
            keep.append(so)
            arr[i] = ctypes.addressof(so)
            outs.append((chars[:nb.value], offs[:g]))
            continue
        s = _empty(g, w.value, dev)
        if t.value == FLOAT64:
            s = s.view(torch.float64)
        elif t.value == FLOAT32:
            s = s.view(torch.float32)
        arr[i] = s.data_ptr()
        outs.append(s)
    return arr, keep, outs


def _int_array(xs) -> ctypes.Array:
    arr = (ctypes.c_int * max(1, len(xs)))()
    for i, x in enumerate(xs):
        arr[i] = int(x)
    return arr


def _scalar(type_: int, value):
    if type_ in (DECIMAL128, DECIMAL256):  # a Python int as little-endian two's complement limbs
        limbs = 2 if type_ == DECIMAL128 else 4
        v = int(value) % (1 << (64 * limbs))
        return (ctypes.c_uint64 * limbs)(*[(v >> (64 * k)) & ((1 << 64) - 1) for k in range(limbs)])
    return _CTYPE[type_](value)


def torch_type(t) -> int:
    import torch
    m = {torch.int8: INT8, torch.int16: INT16, torch.int32: INT32, torch.int64: INT64, torch.uint8: UINT8,
         torch.float32: FLOAT32, torch.float64: FLOAT64}
    if hasattr(torch, "uint16"):
        m[torch.uint16] = UINT16
        m[torch.uint32] = UINT32
        m[torch.uint64] = UINT64
    return m[t.dtype]


def _empty(n, width, device):
    import torch
    dt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}.get(width)
    if dt is None:  # 16- / 32-byte values (Decimal128 / Decimal256) as (n, 2) / (n, 4) int64
        return torch.empty((max(n, 1), width // 8), dtype=torch.int64, device=device)[:n]
    return torch.empty(max(n, 1), dtype=dt, device=device)[:n]


def _alloc(n, width, device, dtype):
    """n >= 1 elements of `width` bytes viewed as `dtype` (2-D (n, 2) / (n, 4) int64 for 16- / 32-byte values)."""
    import torch
    if width in (16, 32):
        return torch.empty((n, width // 8), dtype=torch.int64, device=device)
    return torch.empty(n, dtype=dtype, device=device)


class Context:
    """tfg_ctx bound to a device and the current torch stream of that device."""

    def __init__(self, device: int = 0, stream=None):
        import torch
        self.device = device
        if stream is None:
            stream = torch.cuda.current_stream(device)
        self.stream = stream
        h = ctypes.c_void_p()
        check(lib().tfg_ctx_create(ctypes.c_int(device), ctypes.c_void_p(stream.cuda_stream), ctypes.byref(h)))
        self.h = h
        self._children = weakref.WeakSet()  # aggregators / joins: destroyed before the context

    def sync(self):
        check(lib().tfg_ctx_sync(self.h))

    def reserve(self, nbytes: int):
        check(lib().tfg_ctx_reserve(self.h, ctypes.c_size_t(nbytes)))

    # kernel profiler (HIP events on this context's stream)
    def profile(self, on: bool = True):
        check(lib().tfg_profile_enable(self.h, int(on)))

    def profile_reset(self):
        check(lib().tfg_profile_reset(self.h))

    def profile_read(self) -> dict:
        """{phase name: (total_ms, launches)} accumulated since the last reset."""
        out, i = {}, 0
        name = ctypes.create_string_buffer(64)
        ms, cnt = ctypes.c_double(), ctypes.c_uint64()
        while lib().tfg_profile_read(self.h, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)) == TFG_OK:
            out[name.value.decode()] = (ms.value, cnt.value)
            i += 1
        return out

    def close(self):
        if getattr(self, "h", None) and not sys.is_finalizing():
            for c in list(self._children):
                c.close()
            lib().tfg_ctx_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ---- a1/a2 comparison -------------------------------------------------------------------------
def cmp_const(ctx: Context, col, op: int, scalar, scalar_type: Optional[int] = None, nullmap=None,
              col_type: Optional[int] = None, out=None):
    import torch
    ct = col_type or torch_type(col)
    st = scalar_type or (FLOAT64 if isinstance(scalar, float) else INT64)
    n = col.shape[0]
    out = out if out is not None else torch.empty(n, dtype=torch.uint8, device=col.device)
    s = _scalar(st, scalar)
    check(lib().tfg_cmp_const(ctx.h, ct, _p(col), _p(nullmap), ctypes.c_int64(n), op, st, ctypes.byref(s), _p(out)))
    return out


def cmp_vector(ctx: Context, a, op: int, b, a_nullmap=None, b_nullmap=None, a_type=None, b_type=None):
    import torch
    n = a.shape[0]
    out = torch.empty(n, dtype=torch.uint8, device=a.device)
    check(lib().tfg_cmp_vector(ctx.h, a_type or torch_type(a), _p(a), _p(a_nullmap), op, b_type or torch_type(b),
                               _p(b), _p(b_nullmap), ctypes.c_int64(n), _p(out)))
    return out


def mask_logic(ctx: Context, op: int, a, b=None):
    import torch
    out = torch.empty_like(a)
    check(lib().tfg_mask_logic(ctx.h, op, _p(a), _p(b), ctypes.c_int64(a.shape[0]), _p(out)))
    return out


def count_mask(ctx: Context, mask, nullmap=None) -> int:
    c = ctypes.c_uint64()
    check(lib().tfg_count_mask(ctx.h, _p(mask), _p(nullmap), ctypes.c_int64(mask.shape[0]), ctypes.c_void_p(0),
                               ctypes.byref(c)))
    return c.value


def _col_width(c) -> int:
    return c.element_size() * (c.shape[1] if c.dim() == 2 else 1)


def filter(ctx: Context, mask, cols: Sequence):  # noqa: A001 - mirrors IColumn::filter
    """Stable compaction of every column by one UInt8 filter (ColumnVector<T>::filter)."""
    n = mask.shape[0]
    widths = [_col_width(c) for c in cols]
    cnt = ctypes.c_uint64()
    # count first so outputs are exactly sized (sync), then compact
    check(lib().tfg_count_mask(ctx.h, _p(mask), ctypes.c_void_p(0), ctypes.c_int64(n), ctypes.c_void_p(0),
                               ctypes.byref(cnt)))
    k = cnt.value
    outs = [_alloc(max(k, 1), w, mask.device, c.dtype) for c, w in zip(cols, widths)]
    check(lib().tfg_filter(ctx.h, _p(mask), ctypes.c_int64(n), len(cols), _ptr_array(cols), _int_array(widths),
                           _ptr_array(outs), ctypes.c_void_p(0), ctypes.byref(cnt)))
    return [o[:k] for o in outs]


def filter_cmp_const(ctx: Context, pred_col, op: int, scalar, cols: Sequence, scalar_type=None, pred_nullmap=None,
                     pred_type=None, out_capacity: Optional[int] = None):
    """Fused FilterTransformAction for `pred_col op scalar`; outputs sized to n unless given."""
    import torch
    n = pred_col.shape[0]
    st = scalar_type or (FLOAT64 if isinstance(scalar, float) else INT64)
    widths = [_col_width(c) for c in cols]
    cap = n if out_capacity is None else out_capacity
    outs = [_alloc(max(cap, 1), w, pred_col.device, c.dtype) for c, w in zip(cols, widths)]
    cnt = ctypes.c_uint64()
    s = _scalar(st, scalar)
    check(lib().tfg_filter_cmp_const(ctx.h, pred_type or torch_type(pred_col), _p(pred_col), _p(pred_nullmap), op, st,
                                     ctypes.byref(s), ctypes.c_int64(n), len(cols), _ptr_array(cols),
                                     _int_array(widths), _ptr_array(outs), ctypes.c_void_p(0), ctypes.byref(cnt)))
    return [o[:cnt.value] for o in outs]


def filter_string(ctx: Context, mask, chars, offsets):
    import torch
    n = mask.shape[0]
    out_chars = torch.empty(max(1, chars.shape[0]), dtype=torch.uint8, device=mask.device)
    out_offsets = torch.empty(max(1, n), dtype=torch.int64, device=mask.device)
    rows, nbytes = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().tfg_filter_string(ctx.h, _p(mask), ctypes.c_int64(n), _p(chars), _p(offsets), _p(out_chars),
                                  _p(out_offsets), ctypes.byref(rows), ctypes.byref(nbytes)))
    return out_chars[:nbytes.value], out_offsets[:rows.value]


# ---- a3 arithmetic ----------------------------------------------------------------------------
def arith(ctx: Context, op: int, a, b, res_type: int, a_type=None, b_type=None, a_scale=0, b_scale=0, res_scale=0,
          n=None, device=None):
    """a/b: tensors or Python scalars (constants); Decimal128 / Decimal256 operands and results are
    (n, 2) / (n, 4) int64 tensors of little-endian limbs (constants: Python ints)."""
    import torch
    a_const, b_const = not hasattr(a, "data_ptr"), not hasattr(b, "data_ptr")
    if n is None:
        n = (b if a_const else a).shape[0]
    dev = device or (b if a_const else a).device
    at = a_type or (torch_type(a) if not a_const else INT64)
    bt = b_type or (torch_type(b) if not b_const else INT64)
    out = _empty(n, WIDTH[res_type], dev)
    ap = ctypes.byref(_scalar(at, a)) if a_const else _p(a)
    bp = ctypes.byref(_scalar(bt, b)) if b_const else _p(b)
    check(lib().tfg_arith(ctx.h, op, at, ap, int(a_const), a_scale, bt, bp, int(b_const), b_scale, res_type,
                          res_scale, ctypes.c_int64(n), _p(out)))
    if res_type == FLOAT64:
        out = out.view(torch.float64)
    elif res_type == FLOAT32:
        out = out.view(torch.float32)
    return out


# ---- a22-a24 hash / partition -----------------------------------------------------------------
def weak_hash(ctx: Context, cols: Sequence, types: Optional[Sequence[int]] = None, nullmaps=None, h=None,
              selective=None):
    """WeakHash32 over key columns (IColumn::updateWeakHash32); returns an int32 tensor of u32 bits.
    selective (int64 tensor of row ids, BlockInfo::selective): one hash per listed row."""
    import torch
    n = selective.shape[0] if selective is not None else cols[0].shape[0]
    if h is None:
        h = torch.empty(n, dtype=torch.int32, device=cols[0].device)
        check(lib().tfg_weak_hash_init(ctx.h, _p(h), ctypes.c_int64(n)))
    for j, c in enumerate(cols):
        t = types[j] if types else torch_type(c)
        nm = nullmaps[j] if nullmaps else None
        check(lib().tfg_weak_hash_update_selective(ctx.h, t, _p(c), _p(nm), _p(selective), ctypes.c_int64(n), _p(h)))
    return h


def weak_hash_string(ctx: Context, chars, offsets, h, nullmap=None, collator=COLLATOR_NONE, selective=None):
    n = selective.shape[0] if selective is not None else offsets.shape[0]
    check(lib().tfg_weak_hash_update_string_selective(ctx.h, _p(chars), _p(offsets), _p(nullmap), _p(selective),
                                                      ctypes.c_int64(n), collator, _p(h)))
    return h


def selective_perm(ctx: Context, selective, perm=None):
    """tfg_selective_perm: out[i] = selective[perm[i]] (perm None: selective[i]) as int32 row ids."""
    import torch
    n = perm.shape[0] if perm is not None else selective.shape[0]
    out = torch.empty(max(n, 1), dtype=torch.int32, device=selective.device)[:n]
    check(lib().tfg_selective_perm(ctx.h, _p(selective), _p(perm), ctypes.c_int64(n), _p(out)))
    return out


def fill_selector(ctx: Context, h, part_num: int, fine_grained_stream_count: int = 0):
    import torch
    sel = torch.empty_like(h)
    check(lib().tfg_fill_selector(ctx.h, _p(h), ctypes.c_int64(h.shape[0]), ctypes.c_uint32(part_num),
                                  ctypes.c_uint32(fine_grained_stream_count), _p(sel)))
    return sel


def partition(ctx: Context, selector, num_parts: int):
    """Stable partition permutation + offsets (the row order IColumn::scatter produces)."""
    import torch
    n = selector.shape[0]
    perm = torch.empty(max(n, 1), dtype=torch.int32, device=selector.device)[:n]
    offs = torch.empty(num_parts + 1, dtype=torch.int64, device=selector.device)
    host = (ctypes.c_uint64 * (num_parts + 1))()
    check(lib().tfg_partition(ctx.h, _p(selector), ctypes.c_int64(n), ctypes.c_uint32(num_parts), _p(perm), _p(offs),
                              host))
    return perm, list(host)


def gather(ctx: Context, perm, cols: Sequence):
    n = perm.shape[0]
    widths = [_col_width(c) for c in cols]
    outs = [_alloc(max(n, 1), w, perm.device, c.dtype) for c, w in zip(cols, widths)]
    check(lib().tfg_gather(ctx.h, _p(perm), ctypes.c_int64(n), len(cols), _ptr_array(cols), _int_array(widths),
                           _ptr_array(outs)))
    return [o[:n] for o in outs]


def hash_partition(ctx: Context, cols: Sequence, key_idx: Sequence[int], part_num: int, types=None, nullmaps=None):
    """HashBaseWriterHelper::scatterColumns: returns (partition-major columns, host offsets[P+1])."""
    n = cols[0].shape[0]
    types = types or [torch_type(c) for c in cols]
    outs = [_alloc(max(n, 1), WIDTH[t], c.device, c.dtype) for c, t in zip(cols, types)]
    import torch
    offs = torch.empty(part_num + 1, dtype=torch.int64, device=cols[0].device)
    host = (ctypes.c_uint64 * (part_num + 1))()
    nm = _ptr_array(nullmaps) if nullmaps else ctypes.c_void_p(0)
    check(lib().tfg_hash_partition(ctx.h, ctypes.c_int64(n), len(key_idx), _int_array(key_idx), len(cols),
                                   _int_array(types), _ptr_array(cols), nm, ctypes.c_uint32(part_num),
                                   _ptr_array(outs), _p(offs), host))
    return [o[:n] for o in outs], list(host)


# ---- a9-a17 aggregation -----------------------------------------------------------------------
class _AggParams(ctypes.Structure):
    _fields_ = [("bucket_bits", ctypes.c_int), ("expected_groups", ctypes.c_int64)]


class Aggregator:
    """tfg_agg: hash GROUP BY with one fixed-width key (key_type=0: without key)."""

    def __init__(self, ctx: Context, key_type: int, aggs: Sequence[tuple], bucket_bits: int = 0,
                 expected_groups: int = 0):
        """aggs: sequence of (kind, arg_type[|NULLABLE]) — arg_type ignored for AGG_COUNT_ALL."""
        self.ctx = ctx
        self.key_type = key_type
        self.aggs = list(aggs)
        kinds = _int_array([k for k, _ in aggs])
        types = _int_array([t for _, t in aggs])
        params = _AggParams(bucket_bits, expected_groups)
        h = ctypes.c_void_p()
        check(lib().tfg_agg_create(ctx.h, key_type, len(aggs), kinds, types, ctypes.c_void_p(0), ctypes.byref(params),
                                   ctypes.byref(h)))
        self.h = h
        ctx._children.add(self)

    def consume(self, keys, args: Sequence, key_nullmap=None, arg_nullmaps=None, mask=None, n=None):
        if n is None:
            if keys is not None:
                n = keys.shape[0]
            else:
                a0 = next(a for a in args if a is not None)
                n = a0[1].shape[0] if isinstance(a0, (tuple, list)) else a0.shape[0]
        av, _keep = _arg_array(args)
        check(lib().tfg_agg_consume(self.h, _p(keys), _p(key_nullmap), av,
                                    _ptr_array(arg_nullmaps) if arg_nullmaps else ctypes.c_void_p(0), _p(mask),
                                    ctypes.c_int64(n)))

    def consume_filtered(self, pred_col, op: int, scalar, keys, args: Sequence, scalar_type=None, pred_nullmap=None,
                         key_nullmap=None, arg_nullmaps=None, pred_type=None):
        st = scalar_type or (FLOAT64 if isinstance(scalar, float) else INT64)
        s = _scalar(st, scalar)
        av, _keep = _arg_array(args)
        check(lib().tfg_agg_consume_filtered(self.h, pred_type or torch_type(pred_col), _p(pred_col), _p(pred_nullmap),
                                             op, st, ctypes.byref(s), _p(keys), _p(key_nullmap), av,
                                             _ptr_array(arg_nullmaps) if arg_nullmaps else ctypes.c_void_p(0),
                                             ctypes.c_int64(pred_col.shape[0])))

    def consume_partial(self, keys, states: Sequence, key_nullmap=None, state_nullmaps=None):
        if keys is not None:
            n = keys.shape[0]
        else:
            n = states[0][1].shape[0] if isinstance(states[0], (tuple, list)) else states[0].shape[0]
        av, _keep = _arg_array(states)
        check(lib().tfg_agg_consume_partial(self.h, _p(keys), _p(key_nullmap), av,
                                            _ptr_array(state_nullmaps) if state_nullmaps else ctypes.c_void_p(0),
                                            ctypes.c_int64(n)))

    def reset(self):
        check(lib().tfg_agg_reset(self.h))

    def merge(self, other: "Aggregator"):
        check(lib().tfg_agg_merge(self.h, other.h))

    def size(self) -> int:
        g = ctypes.c_uint64()
        check(lib().tfg_agg_size(self.h, ctypes.byref(g)))
        return g.value

    def result(self, device=None, capacity_hint: Optional[int] = None):
        """-> dict(keys, key_null, states[i], state_null[i]) with exactly size() rows.
        capacity_hint (e.g. the previous result's group count): buffers of that many groups are
        handed over before the count is known, so the device runs the result without waiting for
        a host round trip; a count above the hint falls back to the exact call."""
        import torch
        dev = device or torch.device("cuda", self.ctx.device)
        kw = WIDTH.get(self.key_type, 8)

        def run(g):
            keys = _empty(g, kw, dev) if self.key_type else None
            key_null = torch.empty(max(g, 1), dtype=torch.uint8, device=dev)[:g]
            sarr, _keep, states = _agg_states(self.h, len(self.aggs), g, dev)
            snulls = [torch.empty(max(g, 1), dtype=torch.uint8, device=dev)[:g] for _ in self.aggs]
            cnt = ctypes.c_uint64()
            rc = lib().tfg_agg_result(self.h, _p(keys), _p(key_null), sarr, _ptr_array(snulls),
                                      ctypes.c_uint64(g), ctypes.byref(cnt))
            return rc, cnt.value, keys, key_null, states, snulls

        if capacity_hint:
            rc, n, keys, key_null, states, snulls = run(int(capacity_hint))
            if rc == TFG_OK:
                cut = lambda t: t if t is None else ((t[0], t[1][:n]) if isinstance(t, tuple) else t[:n])
                return {"keys": cut(keys), "key_null": key_null[:n], "states": [cut(s) for s in states],
                        "state_null": [x[:n] for x in snulls]}
            if rc != TFG_ERR_CAPACITY:
                check(rc)
        rc, _, keys, key_null, states, snulls = run(self.size())
        check(rc)
        return {"keys": keys, "key_null": key_null, "states": states, "state_null": snulls}

    def close(self):
        if getattr(self, "h", None) and not sys.is_finalizing():
            lib().tfg_agg_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class KeysAggregator(Aggregator):
    """tfg_agg_create_keys: GROUP BY several fixed-width keys (keys128) or one String key
    (key_string; a String column is a (chars uint8, offsets int64/uint64) pair of device tensors).
    result() restores the key columns; result_packed() / consume_partial_packed() carry the packed
    16-byte keys between the phases of a two-phase aggregation."""

    def __init__(self, ctx: Context, key_types: Sequence[int], aggs: Sequence[tuple], collators=None,
                 bucket_bits: int = 0, expected_groups: int = 0):
        self.ctx = ctx
        self.key_types = list(key_types)
        self.key_type = KEYS128 if (len(key_types) > 1 or key_types[0] == STRING) else key_types[0]
        self.aggs = list(aggs)
        params = _AggParams(bucket_bits, expected_groups)
        h = ctypes.c_void_p()
        check(lib().tfg_agg_create_keys(ctx.h, len(key_types), _int_array(key_types),
                                        _int_array(collators) if collators else ctypes.c_void_p(0), len(aggs),
                                        _int_array([k for k, _ in aggs]), _int_array([t for _, t in aggs]),
                                        ctypes.c_void_p(0), ctypes.byref(params), ctypes.byref(h)))
        self.h = h
        ctx._children.add(self)

    def _key_arrays(self, keys):
        cols, offs = [], []
        for t, k in zip(self.key_types, keys):
            if t == STRING:
                cols.append(k[0])
                offs.append(k[1])
            else:
                cols.append(k)
                offs.append(None)
        t0 = self.key_types[0]  # rows: a Decimal128 / Decimal256 key may come as flat int64 limbs
        n = offs[0].shape[0] if t0 == STRING else cols[0].numel() * cols[0].element_size() // WIDTH[t0]
        return _ptr_array(cols), _ptr_array(offs), n

    def consume(self, keys, args: Sequence, key_nullmaps=None, arg_nullmaps=None, mask=None):
        kc, ko, n = self._key_arrays(keys)
        av, _keep = _arg_array(args)
        check(lib().tfg_agg_consume_keys(self.h, kc, ko, _ptr_array(key_nullmaps) if key_nullmaps else ctypes.c_void_p(0),
                                         av, _ptr_array(arg_nullmaps) if arg_nullmaps else ctypes.c_void_p(0),
                                         _p(mask), ctypes.c_int64(n)))

    def consume_partial(self, keys, states: Sequence, key_nullmaps=None, state_nullmaps=None):
        kc, ko, n = self._key_arrays(keys)
        av, _keep = _arg_array(states)
        check(lib().tfg_agg_consume_partial_keys(
            self.h, kc, ko, _ptr_array(key_nullmaps) if key_nullmaps else ctypes.c_void_p(0), av,
            _ptr_array(state_nullmaps) if state_nullmaps else ctypes.c_void_p(0), ctypes.c_int64(n)))

    def consume_partial_packed(self, keys16, states: Sequence, state_nullmaps=None):
        Aggregator.consume_partial(self, keys16, states, None, state_nullmaps)

    def result_packed(self, device=None):
        """-> dict as Aggregator.result() with keys = (G, 2) int64 packed keys."""
        return Aggregator.result(self, device)

    def holds_packed(self) -> bool:
        """True while the keys are held packed (16 bytes), False once the serialized method holds
        them (String sort keys past 15 bytes, String + fixed tuples, wide tuples)."""
        rc = lib().tfg_agg_weak_hash_packed(self.h, ctypes.c_void_p(0), ctypes.c_int64(0), ctypes.c_void_p(0))
        if rc == TFG_ERR_NOT_IMPLEMENTED:
            return False
        check(rc)
        return True

    def weak_hash_packed(self, keys16, h):
        """h (int32, n) updated with IColumn::updateWeakHash32 of the key columns the packed keys
        (result_packed()["keys"]) stand for."""
        check(lib().tfg_agg_weak_hash_packed(self.h, _p(keys16), ctypes.c_int64(keys16.shape[0]), _p(h)))
        return h

    def result(self, device=None, chars_capacity=None, capacity_hint: Optional[int] = None):
        """-> dict(keys=[col or (chars, offsets)], key_null=[uint8], states=[...], state_null=[...]).
        String keys of the serialized method may need more than 16 bytes a group: the call is
        repeated with the size TFG_ERR_CAPACITY reports.  capacity_hint: as Aggregator.result —
        buffers of that many groups (16 chars bytes a group) handed over before the count is read;
        a count above it falls back to the exact call."""
        import torch
        dev = device or torch.device("cuda", self.ctx.device)
        hinted = bool(capacity_hint) and chars_capacity is None
        g = int(capacity_hint) if hinted else self.size()
        ccap = max(16 * g, 1) if chars_capacity is None else max(chars_capacity, 1)
        cols, offs, nulls = [], [], []
        for t in self.key_types:
            if t == STRING:
                cols.append(torch.empty(ccap, dtype=torch.uint8, device=dev))
                offs.append(torch.empty(max(g, 1), dtype=torch.int64, device=dev))
            else:
                cols.append(_empty(g, WIDTH[t], dev))
                offs.append(None)
            nulls.append(torch.empty(max(g, 1), dtype=torch.uint8, device=dev))
        sarr, _keep, states = _agg_states(self.h, len(self.aggs), g, dev)
        snulls = [torch.empty(max(g, 1), dtype=torch.uint8, device=dev)[:g] for _ in self.aggs]
        cnt, chars = ctypes.c_uint64(), ctypes.c_uint64()
        rc = lib().tfg_agg_result_keys(self.h, _ptr_array(cols), _ptr_array(offs), _ptr_array(nulls), sarr,
                                       _ptr_array(snulls), ctypes.c_uint64(g), ctypes.c_uint64(ccap),
                                       ctypes.byref(cnt), ctypes.byref(chars))
        if hinted and rc == TFG_ERR_CAPACITY:
            # more groups than the hint (the exact call sizes them), or String keys needing more
            # than 16 chars bytes a group (the serialized method): retry with the reported chars
            return self.result(device, chars.value if cnt.value <= g and chars.value > ccap else None)
        if not hinted and rc == TFG_ERR_CAPACITY and chars.value > ccap:
            return self.result(device, chars.value)
        check(rc)
        n = cnt.value if hinted else g
        # each String key column ends at its own last offset (chars reports the largest column's)
        ends = iter(torch.stack([o[n - 1] for t, o in zip(self.key_types, offs) if t == STRING]).tolist()
                    if n and STRING in self.key_types else [])
        keys = []
        for t, c, o in zip(self.key_types, cols, offs):
            keys.append((c[:next(ends)] if n else c[:0], o[:n]) if t == STRING else c[:n])
        cut = lambda x: (x[0], x[1][:n]) if isinstance(x, tuple) else x[:n]
        return {"keys": keys, "key_null": [x[:n] for x in nulls], "states": [cut(x) for x in states] if hinted else states,
                "state_null": [x[:n] for x in snulls]}


# ---- a18-a21 join -----------------------------------------------------------------------------
class Join:
    """tfg_join: hash join v1 semantics (strictness ALL) on one fixed-width key."""

    def __init__(self, ctx: Context, key_type: int, expected_build_rows: int = 0, v2: bool = False,
                 tagged: bool = True):
        """v2: JoinV2's pointer table (tfg_join_create_v2; tagged = tagged heads) instead of the
        radix-partitioned v1 table."""
        self.ctx = ctx
        h = ctypes.c_void_p()
        if v2:
            check(lib().tfg_join_create_v2(ctx.h, key_type, ctypes.c_int64(expected_build_rows),
                                           JOIN_V2_TAGGED if tagged else 0, ctypes.byref(h)))
        else:
            check(lib().tfg_join_create(ctx.h, key_type, ctypes.c_int64(expected_build_rows), ctypes.byref(h)))
        self.h = h
        ctx._children.add(self)

    def build(self, keys, key_nullmap=None, payload: Optional[Sequence] = None):
        """payload: 1-2 8-byte columns carried with the build rows (materialising probe_rows)."""
        if payload:
            check(lib().tfg_join_build_rows(self.h, _p(keys), _p(key_nullmap), ctypes.c_int64(keys.shape[0]),
                                            len(payload), _ptr_array(payload)))
        else:
            check(lib().tfg_join_build(self.h, _p(keys), _p(key_nullmap), ctypes.c_int64(keys.shape[0])))

    def finalize(self):
        check(lib().tfg_join_finalize(self.h))

    def probe(self, keys, kind: int = JOIN_INNER, key_nullmap=None, capacity: Optional[int] = None,
              out_probe=None, out_build=None):
        """-> (probe_idx, build_idx) int32 tensors (u32 bits; build -1 = no match)."""
        import torch
        n = keys.shape[0]
        cap = capacity if capacity is not None else max(n, 1)
        while True:
            pi = out_probe if out_probe is not None else torch.empty(max(cap, 1), dtype=torch.int32, device=keys.device)
            bi = out_build if out_build is not None else torch.empty(max(cap, 1), dtype=torch.int32, device=keys.device)
            cnt = ctypes.c_uint64()
            rc = lib().tfg_join_probe(self.h, kind, _p(keys), _p(key_nullmap), ctypes.c_int64(n), _p(pi), _p(bi),
                                      ctypes.c_uint64(cap), ctypes.c_void_p(0), ctypes.byref(cnt))
            if rc == TFG_ERR_CAPACITY and out_probe is None:
                cap = cnt.value
                continue
            check(rc)
            return pi[:cnt.value], bi[:cnt.value]

    def probe_rows(self, keys, payload: Sequence, build_words: int, kind: int = JOIN_INNER, key_nullmap=None,
                   capacity: Optional[int] = None, outs=None):
        """Materialising probe -> (probe payload columns, build payload columns, build_null).
        Columns are 8-byte tensors of the payload dtypes; build_null (LEFT) marks unmatched rows."""
        import torch
        n = keys.shape[0]
        cap = capacity if capacity is not None else max(n, 1)
        pairs = kind in (JOIN_INNER, JOIN_LEFT)
        while True:
            if outs is not None:
                op, ob, bnull = outs
            else:
                op = [torch.empty(max(cap, 1), dtype=c.dtype, device=keys.device) for c in payload]
                ob = [torch.empty(max(cap, 1), dtype=torch.int64, device=keys.device)
                      for _ in range(build_words if pairs else 0)]
                bnull = torch.empty(max(cap, 1), dtype=torch.uint8, device=keys.device)
            cnt = ctypes.c_uint64()
            rc = lib().tfg_join_probe_rows(self.h, kind, _p(keys), _p(key_nullmap), ctypes.c_int64(n), len(payload),
                                           _ptr_array(payload), _ptr_array(op),
                                           _ptr_array(ob) if ob else ctypes.c_void_p(0),
                                           _p(bnull) if kind == JOIN_LEFT else ctypes.c_void_p(0),
                                           ctypes.c_uint64(cap), ctypes.byref(cnt))
            if rc == TFG_ERR_CAPACITY and outs is None:
                cap = cnt.value
                continue
            check(rc)
            m = cnt.value
            return [o[:m] for o in op], [o[:m] for o in ob], bnull[:m]

    def stats(self):
        r, p = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().tfg_join_stats(self.h, ctypes.byref(r), ctypes.byref(p)))
        return r.value, p.value

    def close(self):
        if getattr(self, "h", None) and not sys.is_finalizing():
            lib().tfg_join_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def join_key_hash(ctx: Context, cols: Sequence, types: Sequence[int], offsets: Optional[Sequence] = None,
                  nullmaps: Optional[Sequence] = None, collators: Optional[Sequence[int]] = None):
    """tfg_join_key_hash: UInt64 fingerprints of the key tuples + the OR of the key null maps
    (general join keys: several columns, String, 16-byte; JoinHashMap.cpp:33-116)."""
    import torch
    n = int(offsets[0].shape[0]) if types[0] == STRING else int(cols[0].shape[0])
    dev = cols[0].device
    out = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    onull = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    k = len(cols)
    check(lib().tfg_join_key_hash(ctx.h, k, _int_array(types), _int_array(collators or [0] * k), _ptr_array(cols),
                                  _ptr_array(offsets or [None] * k), _ptr_array(nullmaps or [None] * k),
                                  ctypes.c_int64(n), _p(out), _p(onull)))
    return out[:n], onull[:n]


def join_keys_equal(ctx: Context, types: Sequence[int], probe_cols: Sequence, build_cols: Sequence, probe_idx,
                    build_idx, probe_offsets: Optional[Sequence] = None, build_offsets: Optional[Sequence] = None,
                    collators: Optional[Sequence[int]] = None, pass_in=None):
    """tfg_join_keys_equal: 1 where pass_in (default 1) and the pair's full key tuples are equal."""
    import torch
    n = int(probe_idx.shape[0])
    out = torch.empty(max(n, 1), dtype=torch.uint8, device=probe_idx.device)
    k = len(types)
    check(lib().tfg_join_keys_equal(ctx.h, k, _int_array(types), _int_array(collators or [0] * k),
                                    _ptr_array(probe_cols), _ptr_array(probe_offsets or [None] * k),
                                    _ptr_array(build_cols), _ptr_array(build_offsets or [None] * k), _p(probe_idx),
                                    _p(build_idx), _p(pass_in), ctypes.c_int64(n), _p(out)))
    return out[:n]


def gather_string(ctx: Context, perm, chars, offsets):
    """tfg_gather_string -> (chars, end offsets) of rows perm (-1 -> the empty String)."""
    import torch
    n = int(perm.shape[0])
    dev = perm.device
    oo = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    nbytes = ctypes.c_uint64()
    check(lib().tfg_gather_string(ctx.h, _p(perm), ctypes.c_int64(n), _p(chars), _p(offsets), _p(oo),
                                  ctypes.c_void_p(0), ctypes.c_uint64(0), ctypes.byref(nbytes)))
    oc = torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=dev)
    check(lib().tfg_gather_string(ctx.h, _p(perm), ctypes.c_int64(n), _p(chars), _p(offsets), _p(oo), _p(oc),
                                  ctypes.c_uint64(nbytes.value), ctypes.byref(nbytes)))
    return oc[:nbytes.value], oo[:n]


# ---- (f1) MPP packet codec: CHBlockChunkCodec / CHBlockChunkCodecV1 --------------------------
CODEC_CHBLOCK, CODEC_V1 = 0, 1


class _CodecColumn(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("type_name", ctypes.c_char_p), ("data", ctypes.c_void_p),
                ("offsets", ctypes.c_void_p), ("nullmap", ctypes.c_void_p)]


def codec_encode(ctx: Context, columns: Sequence, n: int, version: int = CODEC_V1):
    """CHBlockChunkCodec(V1)::encode of a Block held on the device.

    columns: sequence of (name, type_name, data, offsets, nullmap) — data / offsets / nullmap are
    device tensors (offsets and nullmap may be None).  Returns the packet as a uint8 device tensor.
    """
    import torch
    arr = (_CodecColumn * max(len(columns), 1))()
    for i, (name, tname, data, offs, nm) in enumerate(columns):
        arr[i] = _CodecColumn(name.encode(), tname.encode(), _p(data).value, _p(offs).value, _p(nm).value)
    size = ctypes.c_size_t()
    check(lib().tfg_codec_encode(ctx.h, version, len(columns), arr, ctypes.c_int64(n), None, ctypes.c_size_t(0),
                                 ctypes.byref(size)))
    dev = columns[0][2].device if columns and columns[0][2] is not None else torch.device("cuda", ctx.device)
    out = torch.empty(max(size.value, 1), dtype=torch.uint8, device=dev)
    check(lib().tfg_codec_encode(ctx.h, version, len(columns), arr, ctypes.c_int64(n), _p(out),
                                 ctypes.c_size_t(out.numel()), ctypes.byref(size)))
    return out[:size.value]


COMPRESSION_LZ4, COMPRESSION_LZ4HC, COMPRESSION_ZSTD, COMPRESSION_NONE = 1, 2, 3, 5


def codec_compress(ctx: Context, packet, method: int = COMPRESSION_LZ4):
    """CHBlockChunkCodecV1::encode(std::string_view, method) of an uncompressed V1 device packet
    (as MPPTunnelSetHelper::ToCompressedPacket re-encodes a chunk): LZ4 frames (LZ4 / LZ4HC) or ZSTD
    frames (COMPRESSION_ZSTD, the HIGH_COMPRESSION mode), 64 KB of body each, a device tensor."""
    import torch
    size = ctypes.c_size_t()
    check(lib().tfg_codec_compress(ctx.h, method, _p(packet), ctypes.c_size_t(packet.numel()), None,
                                   ctypes.c_size_t(0), ctypes.byref(size)))
    out = torch.empty(max(size.value, 1), dtype=torch.uint8, device=packet.device)
    check(lib().tfg_codec_compress(ctx.h, method, _p(packet), ctypes.c_size_t(packet.numel()), _p(out),
                                   ctypes.c_size_t(out.numel()), ctypes.byref(size)))
    return out[:size.value]


def codec_decompress(ctx: Context, packet):
    """CompressedCHBlockChunkReadBuffer over an LZ4 device packet -> the uncompressed V1 packet."""
    import torch
    size = ctypes.c_size_t()
    check(lib().tfg_codec_decompress(ctx.h, _p(packet), ctypes.c_size_t(packet.numel()), None, ctypes.c_size_t(0),
                                     ctypes.byref(size)))
    out = torch.empty(max(size.value, 1), dtype=torch.uint8, device=packet.device)
    check(lib().tfg_codec_decompress(ctx.h, _p(packet), ctypes.c_size_t(packet.numel()), _p(out),
                                     ctypes.c_size_t(out.numel()), ctypes.byref(size)))
    return out[:size.value]


def codec_decode(ctx: Context, packet, version: int = CODEC_V1):
    """CHBlockChunkCodec(V1)::decode of a device packet -> (rows, [column dicts]).

    Each column: {"name", "type_name", "type", "data", "offsets" (String), "nullmap" (Nullable)}."""
    import torch
    h = ctypes.c_void_p()
    check(lib().tfg_codec_decode(ctx.h, version, _p(packet), ctypes.c_size_t(packet.numel()), ctypes.byref(h)))
    try:
        nc, rows = ctypes.c_int(), ctypes.c_int64()
        check(lib().tfg_codec_packet_info(h, ctypes.byref(nc), ctypes.byref(rows)))
        n = rows.value
        cols = []
        name, tname = ctypes.create_string_buffer(256), ctypes.create_string_buffer(256)
        for i in range(nc.value):
            t, nl, cb = ctypes.c_int(), ctypes.c_int(), ctypes.c_uint64()
            check(lib().tfg_codec_column_info(h, i, name, 256, tname, 256, ctypes.byref(t), ctypes.byref(nl),
                                              ctypes.byref(cb)))
            dev = packet.device
            if t.value == STRING:
                data = torch.empty(max(cb.value, 1), dtype=torch.uint8, device=dev)
                offs = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
            else:
                dt = {INT8: torch.int8, INT16: torch.int16, INT32: torch.int32, INT64: torch.int64,
                      UINT8: torch.uint8, UINT16: torch.int16, UINT32: torch.int32, UINT64: torch.int64,
                      FLOAT32: torch.float32, FLOAT64: torch.float64, DECIMAL32: torch.int32,
                      DECIMAL64: torch.int64}.get(t.value, torch.int64)
                data = _alloc(max(n, 1), WIDTH[t.value], dev, dt)
                offs = None
            nm = torch.empty(max(n, 1), dtype=torch.uint8, device=dev) if nl.value else None
            check(lib().tfg_codec_column_read(h, i, _p(data), _p(offs), _p(nm)))
            cols.append({"name": name.value.decode(), "type_name": tname.value.decode(), "type": t.value,
                         "data": data[:cb.value] if t.value == STRING else data[:n],
                         "offsets": offs[:n] if offs is not None else None,
                         "nullmap": nm[:n] if nm is not None else None})
        torch.cuda.synchronize(packet.device)
        return n, cols
    finally:
        lib().tfg_codec_packet_destroy(h)
