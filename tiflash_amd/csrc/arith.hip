// arith.hip — binary arithmetic (a3): plus / minus / multiply on numbers and decimals.
//
// Reference: BinaryOperationImplBase::vectorVector / vectorConstant / constantVector
// (Functions/FunctionBinaryArithmetic.h:72-215) and DecimalBinaryOperation (:231-500): decimal
// operands of +/- are scaled to the result scale (applyScaled), * multiplies the raw scaled
// integers (result scale = sa + sb, MulDecimalInferer, Common/Decimal.h:109-163); Decimal64 x
// Decimal64 promotes to Int128.  Integer results wrap (two's complement), float results are IEEE.
// One thread per row, loads/stores coalesced; HBM-bound (bytes = inputs + output).
//
// Decimal256 results (and multiplies whose result scale is capped below sa + sb) run the wide
// kernel: operands sign-extended to 512 bits (PromoteType<Int256> = Int512, Common/Decimal.h:
// 402-425), +/- scale one side by 10^k, * multiplies and then divides by
// 10^(sa + sb - res_scale) truncating toward zero (DataTypeDecimal::getScales, DataTypes/
// DataTypeDecimal.h:96-123; applyScaledMul, FunctionBinaryArithmetic.h:574-598).  A Decimal256
// result computed from a Decimal256 operand (need_promote_type) that exceeds 10^65 - 1
// (DecimalMaxValue) raises DECIMAL_OVERFLOW, as does any value that does not fit Int256 (the
// reference's boost checked_int256_t, libs/libcommon/include/common/types.h:35): TFG_ERR_OVERFLOW.
#include "common.h"

namespace tfg {

struct ArithSide {
    int type;
    int is_const;
    const void *p;
    __int128 ci; // constant (integer / decimal) value
    double cf;   // constant (float) value
    __int128 mult; // decimal scale-up factor (+/-)
};

__device__ __forceinline__ __int128 load_i(const ArithSide &s, int64_t i) {
    if (s.is_const) return s.ci;
    switch (s.type) {
    case TFG_INT8: return ((const int8_t *)s.p)[i];
    case TFG_INT16: return ((const int16_t *)s.p)[i];
    case TFG_INT32: case TFG_DECIMAL32: return ((const int32_t *)s.p)[i];
    case TFG_INT64: case TFG_DECIMAL64: return ((const int64_t *)s.p)[i];
    case TFG_UINT8: return ((const uint8_t *)s.p)[i];
    case TFG_UINT16: return ((const uint16_t *)s.p)[i];
    case TFG_UINT32: return ((const uint32_t *)s.p)[i];
    case TFG_UINT64: return (__int128)((const uint64_t *)s.p)[i];
    case TFG_DECIMAL128: {
        const uint64_t *q = (const uint64_t *)s.p + 2 * i;
        return (__int128)(((unsigned __int128)q[1] << 64) | q[0]);
    }
    case TFG_FLOAT32: return (__int128)((const float *)s.p)[i];
    default: return (__int128)((const double *)s.p)[i];
    }
}

__device__ __forceinline__ double load_f(const ArithSide &s, int64_t i) {
    if (s.is_const) return s.cf;
    switch (s.type) {
    case TFG_FLOAT32: return ((const float *)s.p)[i];
    case TFG_FLOAT64: return ((const double *)s.p)[i];
    case TFG_UINT64: return (double)((const uint64_t *)s.p)[i];
    default: return (double)load_i(s, i);
    }
}

__global__ void arith_kernel(int op, ArithSide a, ArithSide b, int res_type, int64_t n, void *out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (res_type == TFG_FLOAT64 || res_type == TFG_FLOAT32) {
            const double x = load_f(a, i), y = load_f(b, i);
            const double r = op == TFG_PLUS ? x + y : op == TFG_MINUS ? x - y : x * y;
            if (res_type == TFG_FLOAT64) ((double *)out)[i] = r;
            else ((float *)out)[i] = (float)r;
            continue;
        }
        unsigned __int128 x = (unsigned __int128)(load_i(a, i) * a.mult);
        unsigned __int128 y = (unsigned __int128)(load_i(b, i) * b.mult);
        const unsigned __int128 r = op == TFG_PLUS ? x + y : op == TFG_MINUS ? x - y : x * y;
        switch (res_type) {
        case TFG_INT8: case TFG_UINT8: ((uint8_t *)out)[i] = (uint8_t)r; break;
        case TFG_INT16: case TFG_UINT16: ((uint16_t *)out)[i] = (uint16_t)r; break;
        case TFG_INT32: case TFG_UINT32: case TFG_DECIMAL32: ((uint32_t *)out)[i] = (uint32_t)r; break;
        case TFG_INT64: case TFG_UINT64: case TFG_DECIMAL64: ((uint64_t *)out)[i] = (uint64_t)r; break;
        default: {
            uint64_t *q = (uint64_t *)out + 2 * i;
            q[0] = (uint64_t)r;
            q[1] = (uint64_t)(r >> 64);
        }
        }
    }
}

// ---------------------------------------------------------------- 512-bit two's complement
struct W512 {
    uint64_t w[8];
};

__device__ __forceinline__ W512 w_from_i128(__int128 v) {
    W512 r;
    r.w[0] = (uint64_t)v;
    r.w[1] = (uint64_t)((unsigned __int128)v >> 64);
    const uint64_t ext = v < 0 ? ~0ull : 0ull;
    for (int k = 2; k < 8; ++k) r.w[k] = ext;
    return r;
}

__device__ __forceinline__ bool w_neg(const W512 &a) { return (int64_t)a.w[7] < 0; }

__device__ __forceinline__ W512 w_add(const W512 &a, const W512 &b) {
    W512 r;
    uint64_t c = 0;
    for (int k = 0; k < 8; ++k) {
        const uint64_t t = a.w[k] + c;
        const uint64_t c1 = t < c;
        r.w[k] = t + b.w[k];
        c = c1 + (r.w[k] < t);
    }
    return r;
}

__device__ __forceinline__ W512 w_negate(const W512 &a) {
    W512 r, one{};
    for (int k = 0; k < 8; ++k) r.w[k] = ~a.w[k];
    one.w[0] = 1;
    return w_add(r, one);
}

// a * m for an unsigned 64-bit m (mod 2^512)
__device__ __forceinline__ W512 w_mul_u64(const W512 &a, uint64_t m) {
    W512 r;
    unsigned __int128 c = 0;
    for (int k = 0; k < 8; ++k) {
        const unsigned __int128 t = (unsigned __int128)a.w[k] * m + c;
        r.w[k] = (uint64_t)t;
        c = t >> 64;
    }
    return r;
}

// magnitude product of two values that fit 256 bits (the result fits 512)
__device__ __forceinline__ W512 w_mul(const W512 &a, const W512 &b) {
    const bool neg = w_neg(a) != w_neg(b);
    const W512 x = w_neg(a) ? w_negate(a) : a, y = w_neg(b) ? w_negate(b) : b;
    W512 r{};
    for (int i = 0; i < 4; ++i) {
        unsigned __int128 c = 0;
        for (int j = 0; j < 8 - i; ++j) {
            const unsigned __int128 t = (unsigned __int128)x.w[i] * (j < 4 ? y.w[j] : 0ull) + r.w[i + j] + c;
            r.w[i + j] = (uint64_t)t;
            c = t >> 64;
        }
    }
    return neg ? w_negate(r) : r;
}

__device__ __forceinline__ uint64_t pow10_u64(int e) {
    uint64_t r = 1;
    while (e-- > 0) r *= 10;
    return r;
}

__device__ __forceinline__ W512 w_scale_up(W512 a, int e) {
    while (e > 0) {
        const int k = e > 19 ? 19 : e;
        a = w_mul_u64(a, pow10_u64(k));
        e -= k;
    }
    return a;
}

// trunc(a / 10^e): magnitude long division by 10^19 chunks (trunc(trunc(x / p) / q) = trunc(x / pq))
__device__ __forceinline__ W512 w_div_pow10(const W512 &a, int e) {
    const bool neg = w_neg(a);
    W512 x = neg ? w_negate(a) : a;
    while (e > 0) {
        const int k = e > 19 ? 19 : e;
        const uint64_t d = pow10_u64(k);
        uint64_t rem = 0;
        for (int j = 7; j >= 0; --j) {
            const unsigned __int128 cur = ((unsigned __int128)rem << 64) | x.w[j];
            x.w[j] = (uint64_t)(cur / d);
            rem = (uint64_t)(cur % d);
        }
        e -= k;
    }
    return neg ? w_negate(x) : x;
}

// a > b, signed
__device__ __forceinline__ bool w_gt(const W512 &a, const W512 &b) {
    if (w_neg(a) != w_neg(b)) return w_neg(b);
    for (int k = 7; k >= 0; --k)
        if (a.w[k] != b.w[k]) return a.w[k] > b.w[k];
    return false;
}

struct WideSide {
    int type;
    int is_const;
    const void *p;
    uint64_t c[4]; // constant, 256-bit two's complement
    int up;        // +/-: scale-up exponent
};

__device__ __forceinline__ W512 load_w(const WideSide &s, int64_t i) {
    const uint64_t *q = nullptr;
    if (s.is_const) q = s.c;
    else if (s.type == TFG_DECIMAL256) q = (const uint64_t *)s.p + 4 * i;
    if (q) {
        W512 r;
        for (int k = 0; k < 4; ++k) r.w[k] = q[k];
        const uint64_t ext = (int64_t)q[3] < 0 ? ~0ull : 0ull;
        for (int k = 4; k < 8; ++k) r.w[k] = ext;
        return r;
    }
    ArithSide a{};
    a.type = s.type;
    a.p = s.p;
    return w_from_i128(load_i(a, i));
}

// flags: bit 0 = promote (a Decimal256 operand and a Decimal256 result: the DecimalMaxValue check)
__global__ void arith_wide_kernel(int op, WideSide a, WideSide b, int res_type, int mul_div, int flags, int64_t n,
                                  void *out, unsigned *overflow) {
    W512 maxv{}; // 10^65 - 1
    maxv.w[0] = 1;
    maxv = w_scale_up(maxv, 65);
    {
        W512 m1;
        for (int k = 0; k < 8; ++k) m1.w[k] = ~0ull;
        maxv = w_add(maxv, m1);
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        W512 x = load_w(a, i), y = load_w(b, i), r;
        if (op == TFG_MULTIPLY) {
            r = w_mul(x, y);
            if (mul_div > 0) r = w_div_pow10(r, mul_div);
        } else {
            x = w_scale_up(x, a.up);
            y = w_scale_up(y, b.up);
            r = w_add(x, op == TFG_MINUS ? w_negate(y) : y);
        }
        if (res_type == TFG_DECIMAL256) {
            // fits Int256: bits 255..511 all equal
            bool fits = true;
            const uint64_t ext = (int64_t)r.w[3] < 0 ? ~0ull : 0ull;
            for (int k = 4; k < 8; ++k) fits = fits && r.w[k] == ext;
            if (!fits || ((flags & 1) && w_gt(r, maxv))) atomicOr(overflow, 1u);
            uint64_t *q = (uint64_t *)out + 4 * i;
            for (int k = 0; k < 4; ++k) q[k] = r.w[k];
        } else {
            switch (res_type) {
            case TFG_DECIMAL32: ((uint32_t *)out)[i] = (uint32_t)r.w[0]; break;
            case TFG_DECIMAL64: ((uint64_t *)out)[i] = r.w[0]; break;
            default: {
                uint64_t *q = (uint64_t *)out + 2 * i;
                q[0] = r.w[0];
                q[1] = r.w[1];
            }
            }
        }
    }
}

// any decimal type, Decimal256 included
static inline bool is_dec(int t) { return is_decimal_type(t) || t == TFG_DECIMAL256; }

static __int128 pow10_128(int e) {
    __int128 r = 1;
    while (e-- > 0) r *= 10;
    return r;
}

static int make_side(int type, const void *p, int is_const, int scale, int res_type, int res_scale, int op,
                     ArithSide &s) {
    TFG_CHECK(type_width(type) > 0 && type != TFG_DECIMAL256, TFG_ERR_ILLEGAL_TYPE, "unsupported operand type %d", type);
    TFG_CHECK(p, TFG_ERR_INVALID_ARG, "null operand");
    s.type = type;
    s.is_const = is_const;
    s.p = p;
    s.ci = 0;
    s.cf = 0;
    s.mult = 1;
    if (is_decimal_type(res_type) && op != TFG_MULTIPLY) {
        const int own = is_decimal_type(type) ? scale : 0;
        TFG_CHECK(res_scale >= own, TFG_ERR_INVALID_ARG, "result scale %d below operand scale %d", res_scale, own);
        s.mult = pow10_128(res_scale - own);
    }
    if (is_const) {
        if (type == TFG_DECIMAL128) {
            memcpy(&s.ci, p, 16);
        } else if (is_float_type(type)) {
            s.cf = type == TFG_FLOAT32 ? *(const float *)p : *(const double *)p;
            s.ci = (__int128)s.cf;
        } else {
            Num v = host_num(type, p);
            s.ci = v.cls == 1 ? (__int128)v.u : (__int128)v.s;
            s.cf = v.cls == 1 ? (double)v.u : (double)v.s;
        }
    }
    return TFG_OK;
}

// the wide path: Decimal256 results / operands, and multiplies with a capped result scale
static int arith_wide(Ctx *ctx, int op, int a_type, const void *a, int a_is_const, int a_scale, int b_type,
                      const void *b, int b_is_const, int b_scale, int res_type, int res_scale, int64_t n, void *out) {
    const int sa = is_dec(a_type) ? a_scale : 0, sb = is_dec(b_type) ? b_scale : 0;
    TFG_CHECK(!is_float_type(a_type) && !is_float_type(b_type), TFG_ERR_ILLEGAL_TYPE, "decimal result with a float operand");
    TFG_CHECK(a && b, TFG_ERR_INVALID_ARG, "null operand");
    WideSide ws[2];
    const int types[2] = {a_type, b_type}, consts[2] = {a_is_const, b_is_const}, scales[2] = {sa, sb};
    const void *ptrs[2] = {a, b};
    for (int j = 0; j < 2; ++j) {
        TFG_CHECK(type_width(types[j]) > 0, TFG_ERR_ILLEGAL_TYPE, "unsupported operand type %d", types[j]);
        WideSide &w = ws[j];
        w = WideSide{};
        w.type = types[j];
        w.is_const = consts[j];
        w.p = ptrs[j];
        if (op != TFG_MULTIPLY) {
            TFG_CHECK(res_scale >= scales[j], TFG_ERR_INVALID_ARG, "result scale %d below operand scale %d", res_scale,
                      scales[j]);
            w.up = res_scale - scales[j];
        }
        if (consts[j]) {
            if (types[j] == TFG_DECIMAL256) {
                memcpy(w.c, ptrs[j], 32);
            } else {
                __int128 v;
                if (types[j] == TFG_DECIMAL128) {
                    memcpy(&v, ptrs[j], 16);
                } else {
                    const Num x = host_num(types[j], ptrs[j]);
                    v = x.cls == 1 ? (__int128)x.u : (__int128)x.s;
                }
                w.c[0] = (uint64_t)v;
                w.c[1] = (uint64_t)((unsigned __int128)v >> 64);
                w.c[2] = w.c[3] = v < 0 ? ~0ull : 0ull;
            }
        }
    }
    int mul_div = 0;
    if (op == TFG_MULTIPLY) {
        mul_div = sa + sb - res_scale;
        TFG_CHECK(mul_div >= 0, TFG_ERR_INVALID_ARG, "multiply result scale %d above the operands' %d", res_scale, sa + sb);
    }
    const int flags = (res_type == TFG_DECIMAL256 && (a_type == TFG_DECIMAL256 || b_type == TFG_DECIMAL256)) ? 1 : 0;
    if (n <= 0) return TFG_OK;
    unsigned *flag = (unsigned *)(ctx->dev_counter + 62); // the context's own flag word (no allocation)
    TFG_HIP(hipMemsetAsync(flag, 0, sizeof(unsigned), ctx->stream));
    {
        ProfScope _ps(ctx, "arith.wide");
        hipLaunchKernelGGL(arith_wide_kernel, dim3(stream_grid(n, 256, 8192)), dim3(256), 0, ctx->stream, op, ws[0], ws[1],
                           res_type, mul_div, flags, n, out, flag);
    }
    TFG_LAUNCH_CHECK();
    uint64_t ov = 0;
    if (int rc = read_back_u64(ctx, ctx->dev_counter + 62, &ov, 1)) return rc;
    TFG_CHECK(!(unsigned)ov, TFG_ERR_OVERFLOW, "Decimal math overflow");
    return TFG_OK;
}

} // namespace tfg

using namespace tfg;

extern "C" int tfg_arith(tfg_ctx *ctx, int op, int a_type, const void *a, int a_is_const, int a_scale, int b_type,
                         const void *b, int b_is_const, int b_scale, int res_type, int res_scale, int64_t n, void *out) {
    TFG_CHECK(ctx && (n == 0 || out), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(op >= TFG_PLUS && op <= TFG_MULTIPLY, TFG_ERR_NOT_IMPLEMENTED, "arithmetic op %d", op);
    TFG_CHECK(type_width(res_type) > 0, TFG_ERR_NOT_IMPLEMENTED, "unsupported result type %d", res_type);
    TFG_CHECK(!(is_dec(res_type) && (is_float_type(a_type) || is_float_type(b_type))), TFG_ERR_ILLEGAL_TYPE,
              "decimal result with a float operand");
    TFG_CHECK(is_dec(res_type) || (a_type != TFG_DECIMAL256 && b_type != TFG_DECIMAL256), TFG_ERR_ILLEGAL_TYPE,
              "Decimal256 operand with a non-decimal result");
    const bool capped_mul = is_dec(res_type) && op == TFG_MULTIPLY &&
                            (is_dec(a_type) ? a_scale : 0) + (is_dec(b_type) ? b_scale : 0) != res_scale;
    if (res_type == TFG_DECIMAL256 || a_type == TFG_DECIMAL256 || b_type == TFG_DECIMAL256 || capped_mul) {
        if (int rc = set_device(ctx)) return rc;
        return arith_wide(ctx, op, a_type, a, a_is_const, a_scale, b_type, b, b_is_const, b_scale, res_type, res_scale, n,
                          out);
    }
    ArithSide sa, sb;
    if (int rc = make_side(a_type, a, a_is_const, a_scale, res_type, res_scale, op, sa)) return rc;
    if (int rc = make_side(b_type, b, b_is_const, b_scale, res_type, res_scale, op, sb)) return rc;
    if (n <= 0) return TFG_OK;
    { ProfScope _ps(ctx, "arith");
    hipLaunchKernelGGL(arith_kernel, dim3(stream_grid(n, 256, 8192)), dim3(256), 0, ctx->stream, op, sa, sb, res_type, n,
                       out);
    }
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}
