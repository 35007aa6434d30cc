// filter.hip — comparison (a1/a2), mask logic, countBytesInFilter (a6) and stable stream
// compaction (a5/a7/a8) for gfx950.
//
// Reference path: FilterTransformAction::transform (DataStreams/FilterTransformAction.cpp:72-173)
//   -> FunctionComparison -> NumComparisonImpl::vectorConstant (Functions/FunctionsComparison.h:101-114)
//   -> countBytesInFilter (Columns/countBytesInFilter.cpp:32-124)
//   -> ColumnVector<T>::filter -> filterImpl (Columns/ColumnVector.cpp:659-683, filterColumn.cpp:174-305).
//
// GPU design: a tile of 4096 rows per 256-thread workgroup.  Pass 1 computes the keep flags
// (from a mask or straight from the predicate column: the fused path never materialises the
// mask) and writes one count per tile; a device-wide scan turns counts into output offsets;
// pass 2 recomputes the keep flags into LDS, ranks them with a block scan (stable, so output
// order = input order as in filterImpl), then streams every column through 16-byte coalesced
// loads and writes kept values at offset + rank.  HBM-bound: bytes = predicate + columns + kept.
#include "common.h"
#include "tile.h"

namespace tfg {

constexpr int FT = 256;          // threads per tile
constexpr int FROWS = 4096;      // rows per tile (16 per thread)
constexpr int MAX_COLS = 8;

struct ColsArg {
    const void *in[MAX_COLS];
    void *out[MAX_COLS];
    int width[MAX_COLS];
    int aligned[MAX_COLS];
    int ncols;
};

// ---------------------------------------------------------------- predicates
struct MaskPred {
    const uint8_t *mask;
    const uint8_t *nullmap;
    bool aligned;
    // keep flags of tile rows into LDS keep[0..FROWS)
    __device__ __forceinline__ void tile_keep(int64_t base, int64_t n, uint8_t *keep) const {
        const int64_t c = base / 16 + threadIdx.x; // one 16-row chunk per thread
        uint8_t m[16], z[16];
        load_chunk<1>(mask, c, n, aligned && (nullmap == nullptr || is_al(nullmap)), m);
        if (nullmap) load_chunk<1>(nullmap, c, n, aligned, z);
#pragma unroll
        for (int e = 0; e < 16; ++e) keep[threadIdx.x * 16 + e] = (m[e] != 0) && !(nullmap && z[e]);
    }
    __device__ static bool is_al(const void *p) { return ((uintptr_t)p & 15) == 0; }
};

template <typename T> struct CmpPred {
    const T *col;
    const uint8_t *nullmap;
    Num b;
    int op;
    bool aligned;
    __device__ __forceinline__ void tile_keep(int64_t base, int64_t n, uint8_t *keep) const {
        constexpr int W = sizeof(T), PER = 16 / W, CHUNKS = FROWS / PER;
        using E = typename ElemOf<W>::T;
        for (int cc = threadIdx.x; cc < CHUNKS; cc += FT) {
            const int64_t c = base / PER + cc;
            E v[PER];
            load_chunk<W>(col, c, n, aligned, v);
#pragma unroll
            for (int e = 0; e < PER; ++e) {
                T x;
                memcpy(&x, &v[e], W);
                const int64_t r = c * PER + e;
                uint8_t k = cmp_value_num<T>(x, b, op);
                if (nullmap && r < n && nullmap[r]) k = 0;
                keep[cc * PER + e] = k;
            }
        }
    }
};

// ---------------------------------------------------------------- block helpers
__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t v, uint32_t *lds, uint32_t *total) {
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (unsigned)d) x += y;
    }
    if (lane == 63) lds[wave] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    const int nw = blockDim.x >> 6;
    for (int w = 0; w < nw; ++w) {
        uint32_t s = lds[w];
        if (w < (int)wave) off += s;
        tot += s;
    }
    __syncthreads();
    if (total) *total = tot;
    return off + x - v;
}

// ---------------------------------------------------------------- tile count / write kernels
template <typename P>
__global__ void __launch_bounds__(FT) filter_count_kernel(P pred, int64_t n, uint32_t *tile_counts) {
    __shared__ __attribute__((aligned(16))) uint8_t keep[FROWS];
    __shared__ uint32_t red[FT / 64];
    const int64_t base = (int64_t)blockIdx.x * FROWS;
    pred.tile_keep(base, n, keep);
    __syncthreads();
    uint32_t c = 0;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        int64_t r = base + threadIdx.x * 16 + e;
        c += (r < n) ? keep[threadIdx.x * 16 + e] : 0;
    }
    uint32_t tot;
    block_excl_scan_u32(c, red, &tot);
    if (threadIdx.x == 0) tile_counts[blockIdx.x] = tot;
}

template <int W>
__device__ __forceinline__ void copy_kept(const void *in, void *out, bool aligned, int64_t base, int64_t n,
                                          uint64_t tile_off, const uint16_t *rank) {
    using E = typename ElemOf<W>::T;
    constexpr int PER = 16 / W, CHUNKS = FROWS / PER;
    E *o = reinterpret_cast<E *>(out) + tile_off;
    for (int cc = threadIdx.x; cc < CHUNKS; cc += FT) {
        const int64_t c = base / PER + cc;
        E v[PER];
        load_chunk<W>(in, c, n, aligned, v);
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            uint16_t rk = rank[cc * PER + e];
            if (rk & 0x8000) o[rk & 0x7FFF] = v[e];
        }
    }
}

template <typename P>
__global__ void __launch_bounds__(FT) filter_write_kernel(P pred, int64_t n, const uint64_t *tile_offsets, ColsArg cols) {
    __shared__ __attribute__((aligned(16))) uint8_t keep[FROWS];
    __shared__ __attribute__((aligned(16))) uint16_t rank[FROWS];
    __shared__ uint32_t red[FT / 64];
    const int64_t base = (int64_t)blockIdx.x * FROWS;
    pred.tile_keep(base, n, keep);
    __syncthreads();
    uint8_t k[16];
    uint32_t c = 0;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        int64_t r = base + threadIdx.x * 16 + e;
        k[e] = (r < n) ? keep[threadIdx.x * 16 + e] : 0;
        c += k[e];
    }
    uint32_t off = block_excl_scan_u32(c, red, nullptr);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        rank[threadIdx.x * 16 + e] = k[e] ? (uint16_t)(0x8000 | off) : 0;
        off += k[e];
    }
    __syncthreads();
    const uint64_t tile_off = tile_offsets[blockIdx.x];
    for (int j = 0; j < cols.ncols; ++j) {
        switch (cols.width[j]) {
        case 1: copy_kept<1>(cols.in[j], cols.out[j], cols.aligned[j], base, n, tile_off, rank); break;
        case 2: copy_kept<2>(cols.in[j], cols.out[j], cols.aligned[j], base, n, tile_off, rank); break;
        case 4: copy_kept<4>(cols.in[j], cols.out[j], cols.aligned[j], base, n, tile_off, rank); break;
        case 8: copy_kept<8>(cols.in[j], cols.out[j], cols.aligned[j], base, n, tile_off, rank); break;
        default: copy_kept<16>(cols.in[j], cols.out[j], cols.aligned[j], base, n, tile_off, rank); break;
        }
    }
}

// ---------------------------------------------------------------- comparison kernels
template <typename A>
__global__ void cmp_const_kernel(const A *col, const uint8_t *nullmap, int64_t n, Num b, int op, bool aligned,
                                 uint8_t *out) {
    constexpr int W = sizeof(A), PER = 16 / W;
    using E = typename ElemOf<W>::T;
    const int64_t chunks = (n + PER - 1) / PER;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < chunks; c += (int64_t)gridDim.x * blockDim.x) {
        E v[PER];
        load_chunk<W>(col, c, n, aligned, v);
        uint8_t m[PER];
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            A x;
            memcpy(&x, &v[e], W);
            m[e] = cmp_value_num<A>(x, b, op);
            int64_t r = c * PER + e;
            if (nullmap && r < n && nullmap[r]) m[e] = 0;
        }
        const int64_t r0 = c * PER;
        if (r0 + PER <= n && ((uintptr_t)(out + r0) % PER) == 0) {
            if constexpr (PER == 16) *reinterpret_cast<uint4 *>(out + r0) = *reinterpret_cast<uint4 *>(m);
            else if constexpr (PER == 8) *reinterpret_cast<uint2 *>(out + r0) = *reinterpret_cast<uint2 *>(m);
            else if constexpr (PER == 4) *reinterpret_cast<uint32_t *>(out + r0) = *reinterpret_cast<uint32_t *>(m);
            else if constexpr (PER == 2) *reinterpret_cast<uint16_t *>(out + r0) = *reinterpret_cast<uint16_t *>(m);
            else out[r0] = m[0];
        } else {
            for (int e = 0; e < PER; ++e)
                if (r0 + e < n) out[r0 + e] = m[e];
        }
    }
}

template <typename A, typename B>
__global__ void cmp_vector_kernel(const A *a, const uint8_t *an, const B *b, const uint8_t *bn, int64_t n, int op,
                                  uint8_t *out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint8_t m = cmp_values<A, B>(a[i], b[i], op);
        if ((an && an[i]) || (bn && bn[i])) m = 0;
        out[i] = m;
    }
}

__global__ void mask_logic_kernel(int op, const uint8_t *a, const uint8_t *b, int64_t n, uint8_t *out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint8_t x = a[i] != 0;
        out[i] = op == TFG_AND ? (x && b[i]) : op == TFG_OR ? (x || b[i]) : !x;
    }
}

__global__ void count_mask_kernel(const uint8_t *mask, const uint8_t *nullmap, int64_t n, bool aligned,
                                  uint64_t *count) {
    const int64_t chunks = (n + 15) / 16;
    uint32_t c = 0;
    for (int64_t ch = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ch < chunks; ch += (int64_t)gridDim.x * blockDim.x) {
        uint8_t m[16], z[16];
        load_chunk<1>(mask, ch, n, aligned, m);
        if (nullmap) load_chunk<1>(nullmap, ch, n, aligned, z);
#pragma unroll
        for (int e = 0; e < 16; ++e) c += (m[e] != 0) && !(nullmap && z[e]);
    }
    // wave reduce then one atomic per wave
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd((unsigned long long *)count, (unsigned long long)c);
}

// ---------------------------------------------------------------- string filter helpers
__global__ void string_kept_lengths_kernel(const uint8_t *mask, const uint64_t *offsets, int64_t n, uint64_t *lens) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t prev = i ? offsets[i - 1] : 0;
        lens[i] = mask[i] ? offsets[i] - prev : 0;
    }
}

// one wave per row-group: lanes copy bytes of a row cooperatively
__global__ void string_copy_kernel(const uint8_t *mask, const uint8_t *chars, const uint64_t *offsets, int64_t n,
                                   const uint64_t *starts, uint8_t *out_chars, uint64_t *ends) {
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const unsigned lane = threadIdx.x & 63;
    for (int64_t i = wave; i < n; i += nwaves) {
        uint64_t prev = i ? offsets[i - 1] : 0;
        uint64_t len = offsets[i] - prev;
        uint64_t s = starts[i];
        if (lane == 0) ends[i] = s + len;
        if (!mask[i]) continue;
        for (uint64_t b = lane; b < len; b += 64) out_chars[s + b] = chars[prev + b];
    }
}

// String gather: row lengths through perm (0xFFFFFFFF -> the empty String, 1 byte '\0')
__global__ void string_gather_lengths_kernel(const uint32_t *perm, const uint64_t *offsets, int64_t n,
                                             uint64_t *lens) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t p = perm[i];
        lens[i] = p == 0xFFFFFFFFu ? 1 : offsets[p] - (p ? offsets[p - 1] : 0);
    }
}

__global__ void string_gather_offsets_kernel(const uint64_t *starts, const uint64_t *lens, int64_t n,
                                             uint64_t *out_offsets) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out_offsets[i] = starts[i] + lens[i];
}

// one wave per row: lanes copy the row's bytes
__global__ void string_gather_copy_kernel(const uint32_t *perm, const uint8_t *chars, const uint64_t *offsets,
                                          int64_t n, const uint64_t *starts, uint8_t *out_chars) {
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const unsigned lane = threadIdx.x & 63;
    for (int64_t i = wave; i < n; i += nwaves) {
        const uint32_t p = perm[i];
        const uint64_t s = starts[i];
        if (p == 0xFFFFFFFFu) {
            if (lane == 0) out_chars[s] = 0;
            continue;
        }
        const uint64_t prev = p ? offsets[p - 1] : 0, len = offsets[p] - prev;
        for (uint64_t b = lane; b < len; b += 64) out_chars[s + b] = chars[prev + b];
    }
}

// ---------------------------------------------------------------- host drivers
template <typename P>
static int run_filter(Ctx *ctx, const P &pred, int64_t n, const ColsArg &cols, uint64_t *out_count_dev,
                      uint64_t *out_count_host) {
    const int64_t tiles = (n + FROWS - 1) / FROWS;
    Carver cv;
    size_t o_counts = cv.take<uint32_t>(tiles > 0 ? tiles : 1);
    size_t o_offs = cv.take<uint64_t>(tiles + 1);
    size_t o_tmp = cv.take<uint8_t>(scan_tmp_bytes(tiles));
    void *s;
    if (int rc = scratch_get(ctx, cv.off, &s)) return rc;
    char *sb = (char *)s;
    uint32_t *counts = (uint32_t *)(sb + o_counts);
    uint64_t *offs = (uint64_t *)(sb + o_offs);
    if (tiles > 0) {
        { ProfScope _ps(ctx, "filter.count");
        hipLaunchKernelGGL(filter_count_kernel<P>, dim3((unsigned)tiles), dim3(FT), 0, ctx->stream, pred, n, counts);
        }
        TFG_LAUNCH_CHECK();
    }
    if (int rc = exclusive_scan_u32(ctx, counts, offs, tiles, sb + o_tmp)) return rc;
    if (tiles > 0 && cols.ncols > 0) {
        { ProfScope _ps(ctx, "filter.write");
        hipLaunchKernelGGL(filter_write_kernel<P>, dim3((unsigned)tiles), dim3(FT), 0, ctx->stream, pred, n, offs, cols);
        }
        TFG_LAUNCH_CHECK();
    }
    if (out_count_dev)
        TFG_HIP(hipMemcpyAsync(out_count_dev, offs + tiles, sizeof(uint64_t), hipMemcpyDeviceToDevice, ctx->stream));
    if (out_count_host) return read_back_u64(ctx, offs + tiles, out_count_host, 1);
    return TFG_OK;
}

static int make_cols(int ncols, const void *const *cols, const int *widths, void *const *outs, ColsArg &ca) {
    TFG_CHECK(ncols >= 0 && ncols <= MAX_COLS, TFG_ERR_INVALID_ARG, "ncols %d out of range [0,%d]", ncols, MAX_COLS);
    ca.ncols = ncols;
    for (int j = 0; j < ncols; ++j) {
        int w = widths[j];
        TFG_CHECK(w == 1 || w == 2 || w == 4 || w == 8 || w == 16, TFG_ERR_INVALID_ARG, "bad column width %d", w);
        TFG_CHECK(cols[j] && outs[j], TFG_ERR_INVALID_ARG, "null column pointer");
        ca.in[j] = cols[j];
        ca.out[j] = outs[j];
        ca.width[j] = w;
        ca.aligned[j] = is_aligned16(cols[j]);
    }
    return TFG_OK;
}

static int zero_count(Ctx *ctx, uint64_t *out_count_dev, uint64_t *out_count_host) {
    if (out_count_dev) TFG_HIP(hipMemsetAsync(out_count_dev, 0, sizeof(uint64_t), ctx->stream));
    if (out_count_host) *out_count_host = 0;
    return TFG_OK;
}

} // namespace tfg

using namespace tfg;

static inline int mirror_op(int op) {
    switch (op) {
    case TFG_LT: return TFG_GT;
    case TFG_GT: return TFG_LT;
    case TFG_LE: return TFG_GE;
    case TFG_GE: return TFG_LE;
    default: return op;
    }
}

extern "C" {

int tfg_cmp_const(tfg_ctx *ctx, int col_type, const void *col, const uint8_t *col_nullmap, int64_t n, int op,
                  int scalar_type, const void *scalar_host, uint8_t *out_mask) {
    TFG_CHECK(ctx && (n == 0 || (col && out_mask)) && scalar_host, TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(n >= 0, TFG_ERR_INVALID_ARG, "negative row count");
    TFG_CHECK(op >= TFG_EQ && op <= TFG_GE, TFG_ERR_INVALID_ARG, "bad comparison op %d", op);
    TFG_CHECK(is_fixed_numeric(scalar_type), TFG_ERR_ILLEGAL_TYPE, "unsupported constant type %d", scalar_type);
    if (failpoint("cmp_const")) return fail(TFG_ERR_FAULT_INJECTED, "failpoint cmp_const");
    if (n == 0) return TFG_OK;
    Num b = host_num(scalar_type, scalar_host);
    bool al = is_aligned16(col);
    TFG_DISPATCH_NUMERIC(col_type, A, {
        constexpr int PER = 16 / sizeof(A);
        unsigned grid = stream_grid((n + PER - 1) / PER, 256, 8192);
        { ProfScope _ps(ctx, "cmp.const");
        hipLaunchKernelGGL(cmp_const_kernel<A>, dim3(grid), dim3(256), 0, ctx->stream, (const A *)col, col_nullmap, n,
                           b, op, al, out_mask);
        }
    });
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_cmp_const_left(tfg_ctx *ctx, int scalar_type, const void *scalar_host, int op, int col_type, const void *col,
                       const uint8_t *col_nullmap, int64_t n, uint8_t *out_mask) {
    // Op(const, col) == mirror(Op)(col, const) — accurate:: comparisons are antisymmetric.
    return tfg_cmp_const(ctx, col_type, col, col_nullmap, n, mirror_op(op), scalar_type, scalar_host, out_mask);
}

int tfg_cmp_vector(tfg_ctx *ctx, int a_type, const void *a, const uint8_t *a_nullmap, int op, int b_type, const void *b,
                   const uint8_t *b_nullmap, int64_t n, uint8_t *out_mask) {
    TFG_CHECK(ctx && (n == 0 || (a && b && out_mask)), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(n >= 0, TFG_ERR_INVALID_ARG, "negative row count");
    TFG_CHECK(op >= TFG_EQ && op <= TFG_GE, TFG_ERR_INVALID_ARG, "bad comparison op %d", op);
    if (n == 0) return TFG_OK;
    unsigned grid = stream_grid(n, 256, 8192);
    TFG_DISPATCH_NUMERIC(a_type, A, {
        TFG_DISPATCH_NUMERIC(b_type, B, {
            hipLaunchKernelGGL((cmp_vector_kernel<A, B>), dim3(grid), dim3(256), 0, ctx->stream, (const A *)a,
                               a_nullmap, (const B *)b, b_nullmap, n, op, out_mask);
        });
    });
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_mask_logic(tfg_ctx *ctx, int op, const uint8_t *a, const uint8_t *b, int64_t n, uint8_t *out_mask) {
    TFG_CHECK(ctx && (n == 0 || (a && out_mask && (b || op == TFG_NOT))), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(op >= TFG_AND && op <= TFG_NOT, TFG_ERR_INVALID_ARG, "bad logic op %d", op);
    if (n <= 0) return TFG_OK;
    hipLaunchKernelGGL(mask_logic_kernel, dim3(stream_grid(n, 256, 8192)), dim3(256), 0, ctx->stream, op, a, b, n,
                       out_mask);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_count_mask(tfg_ctx *ctx, const uint8_t *mask, const uint8_t *nullmap, int64_t n, uint64_t *out_count_dev,
                   uint64_t *out_count_host) {
    TFG_CHECK(ctx && (n == 0 || mask), TFG_ERR_INVALID_ARG, "null argument");
    uint64_t *cnt = out_count_dev ? out_count_dev : ctx->dev_counter;
    TFG_HIP(hipMemsetAsync(cnt, 0, sizeof(uint64_t), ctx->stream));
    if (n > 0) {
        bool al = is_aligned16(mask) && (!nullmap || is_aligned16(nullmap));
        hipLaunchKernelGGL(count_mask_kernel, dim3(stream_grid((n + 15) / 16, 256, 4096)), dim3(256), 0, ctx->stream,
                           mask, nullmap, n, al, cnt);
        TFG_LAUNCH_CHECK();
    }
    if (out_count_host) return read_back_u64(ctx, cnt, out_count_host, 1);
    return TFG_OK;
}

int tfg_filter(tfg_ctx *ctx, const uint8_t *mask, int64_t n, int ncols, const void *const *cols, const int *widths,
               void *const *outs, uint64_t *out_count_dev, uint64_t *out_count_host) {
    TFG_CHECK(ctx && (n == 0 || mask), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(n >= 0, TFG_ERR_INVALID_ARG, "negative row count");
    if (failpoint("filter")) return fail(TFG_ERR_FAULT_INJECTED, "failpoint filter");
    if (n == 0) return zero_count(ctx, out_count_dev, out_count_host);
    ColsArg ca{};
    if (int rc = make_cols(ncols, cols, widths, outs, ca)) return rc;
    MaskPred p{mask, nullptr, is_aligned16(mask)};
    return run_filter(ctx, p, n, ca, out_count_dev, out_count_host);
}

int tfg_filter_cmp_const(tfg_ctx *ctx, int pred_type, const void *pred_col, const uint8_t *pred_nullmap, int op,
                         int scalar_type, const void *scalar_host, int64_t n, int ncols, const void *const *cols,
                         const int *widths, void *const *outs, uint64_t *out_count_dev, uint64_t *out_count_host) {
    TFG_CHECK(ctx && (n == 0 || pred_col) && scalar_host, TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(n >= 0, TFG_ERR_INVALID_ARG, "negative row count");
    TFG_CHECK(op >= TFG_EQ && op <= TFG_GE, TFG_ERR_INVALID_ARG, "bad comparison op %d", op);
    TFG_CHECK(is_fixed_numeric(scalar_type), TFG_ERR_ILLEGAL_TYPE, "unsupported constant type %d", scalar_type);
    if (n == 0) return zero_count(ctx, out_count_dev, out_count_host);
    ColsArg ca{};
    if (int rc = make_cols(ncols, cols, widths, outs, ca)) return rc;
    Num b = host_num(scalar_type, scalar_host);
    TFG_DISPATCH_NUMERIC(pred_type, A, {
        CmpPred<A> p{(const A *)pred_col, pred_nullmap, b, op, is_aligned16(pred_col)};
        return run_filter(ctx, p, n, ca, out_count_dev, out_count_host);
    });
    return TFG_OK;
}

int tfg_filter_string(tfg_ctx *ctx, const uint8_t *mask, int64_t n, const uint8_t *chars, const uint64_t *offsets,
                      uint8_t *out_chars, uint64_t *out_offsets, uint64_t *out_rows_host, uint64_t *out_bytes_host) {
    TFG_CHECK(ctx && (n == 0 || (mask && chars && offsets && out_chars && out_offsets)), TFG_ERR_INVALID_ARG,
              "null argument");
    if (n == 0) {
        if (out_rows_host) *out_rows_host = 0;
        if (out_bytes_host) *out_bytes_host = 0;
        return TFG_OK;
    }
    // scratch: lens (n), starts (n+1), ends (n), scan tmp; the row compaction below reuses
    // run_filter, whose own scratch lives after ours.
    Carver cv;
    size_t o_lens = cv.take<uint64_t>(n), o_starts = cv.take<uint64_t>(n + 1), o_ends = cv.take<uint64_t>(n);
    size_t o_tmp = cv.take<uint8_t>(scan_tmp_bytes(n));
    ArenaScope hold(ctx); // the call's buffers: reused by the next call on this stream, never freed here
    uint64_t *mine;
    if (int rc = set_device(ctx)) return rc;
    if (int rc = arena_alloc(ctx, cv.off, (void **)&mine)) return rc;
    char *sb = (char *)mine;
    uint64_t *lens = (uint64_t *)(sb + o_lens), *starts = (uint64_t *)(sb + o_starts), *ends = (uint64_t *)(sb + o_ends);
    unsigned grid = stream_grid(n, 256, 8192);
    hipLaunchKernelGGL(string_kept_lengths_kernel, dim3(grid), dim3(256), 0, ctx->stream, mask, offsets, n, lens);
    int rc = exclusive_scan_u64(ctx, lens, starts, n, sb + o_tmp);
    if (!rc) {
        hipLaunchKernelGGL(string_copy_kernel, dim3(stream_grid(n * 64, 256, 8192)), dim3(256), 0, ctx->stream, mask,
                           chars, offsets, n, starts, out_chars, ends);
        // compact the end offsets of kept rows
        const void *cin[1] = {ends};
        void *cout[1] = {out_offsets};
        int w[1] = {8};
        ColsArg ca{};
        rc = make_cols(1, cin, w, cout, ca);
        if (!rc) {
            MaskPred p{mask, nullptr, is_aligned16(mask)};
            uint64_t rows = 0;
            rc = run_filter(ctx, p, n, ca, nullptr, &rows);
            if (out_rows_host) *out_rows_host = rows;
            if (!rc && out_bytes_host) rc = read_back_u64(ctx, starts + n, out_bytes_host, 1);
        }
    }
    return rc;
}

int tfg_gather_string(tfg_ctx *ctx, const uint32_t *perm, int64_t n, const uint8_t *chars, const uint64_t *offsets,
                      uint64_t *out_offsets, uint8_t *out_chars, uint64_t chars_capacity, uint64_t *out_chars_host) {
    TFG_CHECK(ctx && (n == 0 || (perm && offsets && out_offsets)), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(!out_chars || chars, TFG_ERR_INVALID_ARG, "null chars");
    if (n <= 0) {
        if (out_chars_host) *out_chars_host = 0;
        return TFG_OK;
    }
    Carver cv;
    size_t o_lens = cv.take<uint64_t>(n), o_starts = cv.take<uint64_t>(n + 1);
    size_t o_tmp = cv.take<uint8_t>(scan_tmp_bytes(n));
    ArenaScope hold(ctx); // the call's buffers: reused by the next call on this stream, never freed here
    uint64_t *mine;
    if (int rc = set_device(ctx)) return rc;
    if (int rc = arena_alloc(ctx, cv.off, (void **)&mine)) return rc;
    char *sb = (char *)mine;
    uint64_t *lens = (uint64_t *)(sb + o_lens), *starts = (uint64_t *)(sb + o_starts);
    const unsigned grid = stream_grid(n, 256, 8192);
    hipLaunchKernelGGL(string_gather_lengths_kernel, dim3(grid), dim3(256), 0, ctx->stream, perm, offsets, n, lens);
    int rc = exclusive_scan_u64(ctx, lens, starts, n, sb + o_tmp);
    uint64_t total = 0;
    if (!rc) {
        hipLaunchKernelGGL(string_gather_offsets_kernel, dim3(grid), dim3(256), 0, ctx->stream, starts, lens, n,
                           out_offsets);
        rc = read_back_u64(ctx, starts + n, &total, 1);
    }
    if (!rc && out_chars_host) *out_chars_host = total;
    if (!rc && out_chars) {
        if (total > chars_capacity)
            rc = fail(TFG_ERR_CAPACITY, "String gather needs %llu chars bytes, capacity %llu",
                      (unsigned long long)total, (unsigned long long)chars_capacity);
        else
            hipLaunchKernelGGL(string_gather_copy_kernel, dim3(stream_grid(n * 64, 256, 8192)), dim3(256), 0,
                               ctx->stream, perm, chars, offsets, n, starts, out_chars);
    }
    return rc;
}

} // extern "C"
