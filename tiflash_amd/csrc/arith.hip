// arith.hip — binary arithmetic (a3): plus / minus / multiply on numbers and decimals.
//
// Reference: BinaryOperationImplBase::vectorVector / vectorConstant / constantVector
// (Functions/FunctionBinaryArithmetic.h:72-215) and DecimalBinaryOperation (:231-500): decimal
// operands of +/- are scaled to the result scale (applyScaled), * multiplies the raw scaled
// integers (result scale = sa + sb, MulDecimalInferer, Common/Decimal.h:109-163); Decimal64 x
// Decimal64 promotes to Int128.  Integer results wrap (two's complement), float results are IEEE.
// One thread per row, loads/stores coalesced; HBM-bound (bytes = inputs + output).
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

} // namespace tfg

using namespace tfg;

extern "C" int tfg_arith(tfg_ctx *ctx, int op, int a_type, const void *a, int a_is_const, int a_scale, int b_type,
                         const void *b, int b_is_const, int b_scale, int res_type, int res_scale, int64_t n, void *out) {
    TFG_CHECK(ctx && (n == 0 || out), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(op >= TFG_PLUS && op <= TFG_MULTIPLY, TFG_ERR_NOT_IMPLEMENTED, "arithmetic op %d", op);
    TFG_CHECK(type_width(res_type) > 0 && res_type != TFG_DECIMAL256, TFG_ERR_NOT_IMPLEMENTED,
              "unsupported result type %d (Decimal256 arithmetic is not on the path)", res_type);
    TFG_CHECK(!(is_decimal_type(res_type) && (is_float_type(a_type) || is_float_type(b_type))), TFG_ERR_ILLEGAL_TYPE,
              "decimal result with a float operand");
    if (is_decimal_type(res_type) && op == TFG_MULTIPLY)
        TFG_CHECK((is_decimal_type(a_type) ? a_scale : 0) + (is_decimal_type(b_type) ? b_scale : 0) == res_scale,
                  TFG_ERR_INVALID_ARG, "multiply result scale must be the sum of operand scales");
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
