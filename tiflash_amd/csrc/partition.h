// partition.h — stable counting partition (histogram -> scan -> scatter) shared by the
// exchange repartition (a23), the aggregation bucket pass (a11) and the join radix pass (a19/a21).
//
// Reference: IColumn::scatterImpl (Columns/IColumn.h:655-721) keeps row order inside every
// destination; fillSelector (Flash/Mpp/HashBaseWriterHelper.cpp:46-62) picks the destination.
//
// GPU design: G workgroups each own one contiguous row segment.  Pass 1 builds a per-segment
// histogram in LDS and writes it partition-major (counts[p * G + g]); an exclusive scan of that
// table gives every (partition, segment) its output base, so the output is partition-major and,
// inside a partition, segment order = row order.  Pass 2 re-reads the segment 256 rows at a time,
// ranks rows of equal partition inside each wave with ballot / mbcnt (a "match" loop over the
// distinct partitions present in the wave), combines the 4 waves through LDS in wave order and
// scatters every column to base + rank: the result is exactly the stable order.
#pragma once
#include "common.h"

namespace tfg {

constexpr int PT = 256;          // partition kernel threads (4 waves)
constexpr int PMAX = 4096;       // max partitions of the stable kernel
constexpr int PMAX_UNSTABLE = 16384; // max partitions of the LDS-atomic kernel
constexpr int PCOLS = 12;

struct PCols {
    const void *in[PCOLS];
    void *out[PCOLS];
    int width[PCOLS];
    int ncols;
};

// Key columns hashed with IColumn::updateWeakHash32 semantics.
struct KeyCols {
    const void *col[4];
    const uint8_t *nullmap[4];
    int type[4];
    int nkeys;
};

// value of key column j at row r converted to the UInt64 the reference feeds to crc32q
__device__ __forceinline__ uint32_t hash_key_row(const uint32_t (*t)[256], const KeyCols &k, int64_t r, uint32_t h) {
    for (int j = 0; j < k.nkeys; ++j) {
        if (k.nullmap[j] && k.nullmap[j][r]) continue;
        const void *c = k.col[j];
        switch (k.type[j]) {
        case TFG_INT8: h = crc32c_u64(t, h, (uint64_t)(int64_t)((const int8_t *)c)[r]); break;
        case TFG_INT16: h = crc32c_u64(t, h, (uint64_t)(int64_t)((const int16_t *)c)[r]); break;
        case TFG_INT32: case TFG_DECIMAL32: h = crc32c_u64(t, h, (uint64_t)(int64_t)((const int32_t *)c)[r]); break;
        case TFG_INT64: case TFG_DECIMAL64: case TFG_UINT64: h = crc32c_u64(t, h, ((const uint64_t *)c)[r]); break;
        case TFG_UINT8: h = crc32c_u64(t, h, (uint64_t)((const uint8_t *)c)[r]); break;
        case TFG_UINT16: h = crc32c_u64(t, h, (uint64_t)((const uint16_t *)c)[r]); break;
        case TFG_UINT32: h = crc32c_u64(t, h, (uint64_t)((const uint32_t *)c)[r]); break;
        case TFG_DECIMAL128: {
            const uint64_t *l = (const uint64_t *)c + 2 * r;
            h = crc32c_u64(t, h, l[0]);
            h = crc32c_u64(t, h, l[1]);
            break;
        }
        default: break;
        }
    }
    return h;
}

// ---------------------------------------------------------------- selectors
// sel(r) returns the partition of row r, or 0xFFFFFFFF to drop the row.
struct SelArray {
    const uint32_t *sel;
    static constexpr bool needs_crc = false;
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*)[256], int64_t r) const { return sel[r]; }
};

// fillSelector over the weak hash of key columns: part = (UInt64(h) * P) >> 32
struct SelHashMul {
    KeyCols k;
    uint32_t parts;
    static constexpr bool needs_crc = true;
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const {
        uint32_t h = hash_key_row(t, k, r, 0xFFFFFFFFu);
        return (uint32_t)(((uint64_t)h * parts) >> 32);
    }
};

// Per-row predicate: `pred_col Op scalar` (nullable -> drop), or a UInt8 mask, or none.
struct RowPred {
    int kind; // 0 none, 1 mask, 2 compare
    int type;
    const void *col;
    const uint8_t *nullmap;
    Num b;
    int op;
    __device__ __forceinline__ bool operator()(int64_t r) const {
        if (kind == 0) return true;
        if (kind == 1) return ((const uint8_t *)col)[r] != 0 && !(nullmap && nullmap[r]);
        if (nullmap && nullmap[r]) return false;
        switch (type) {
        case TFG_INT8: return cmp_value_num<int8_t>(((const int8_t *)col)[r], b, op);
        case TFG_INT16: return cmp_value_num<int16_t>(((const int16_t *)col)[r], b, op);
        case TFG_INT32: return cmp_value_num<int32_t>(((const int32_t *)col)[r], b, op);
        case TFG_INT64: return cmp_value_num<int64_t>(((const int64_t *)col)[r], b, op);
        case TFG_UINT8: return cmp_value_num<uint8_t>(((const uint8_t *)col)[r], b, op);
        case TFG_UINT16: return cmp_value_num<uint16_t>(((const uint16_t *)col)[r], b, op);
        case TFG_UINT32: return cmp_value_num<uint32_t>(((const uint32_t *)col)[r], b, op);
        case TFG_UINT64: return cmp_value_num<uint64_t>(((const uint64_t *)col)[r], b, op);
        case TFG_FLOAT32: return cmp_value_num<float>(((const float *)col)[r], b, op);
        default: return cmp_value_num<double>(((const double *)col)[r], b, op);
        }
    }
};

struct PartLayout {
    int64_t n;
    int64_t seg;   // rows per segment (multiple of PT)
    unsigned G;    // segments = workgroups
    uint32_t P;    // partitions
};

inline PartLayout make_layout(int64_t n, uint32_t P) {
    PartLayout L;
    L.n = n;
    L.P = P;
    // ~16K+ rows per segment, at most 2048 segments, and keep the P x G table <= 4M entries
    int64_t g = n / 16384;
    if (g < 1) g = 1;
    if (g > 2048) g = 2048;
    while (g > 1 && (int64_t)P * g > (int64_t)1 << 22) g >>= 1;
    int64_t seg = (n + g - 1) / g;
    seg = (seg + PT - 1) / PT * PT;
    if (seg < PT) seg = PT;
    g = (n + seg - 1) / seg;
    if (g < 1) g = 1;
    L.seg = seg;
    L.G = (unsigned)g;
    return L;
}

template <typename Sel>
__global__ void __launch_bounds__(PT) part_hist_kernel(Sel sel, RowPred pred, PartLayout L, uint32_t *counts) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[]; // P entries (+ crc tables)
    uint32_t(*crc)[256] = reinterpret_cast<uint32_t(*)[256]>(hist + ((L.P + 3) & ~3u));
    for (uint32_t p = threadIdx.x; p < L.P; p += PT) hist[p] = 0;
    if constexpr (Sel::needs_crc) load_crc_lds(crc);
    __syncthreads();
    const int64_t begin = (int64_t)blockIdx.x * L.seg;
    int64_t end = begin + L.seg;
    if (end > L.n) end = L.n;
    for (int64_t r = begin + threadIdx.x; r < end; r += PT) {
        if (!pred(r)) continue;
        uint32_t p = sel(crc, r);
        if (p < L.P) atomicAdd(&hist[p], 1u);
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < L.P; p += PT) counts[(int64_t)p * L.G + blockIdx.x] = hist[p];
}

__device__ __forceinline__ void scatter_row(const PCols &cols, int64_t r, uint64_t pos) {
    for (int j = 0; j < cols.ncols; ++j) {
        switch (cols.width[j]) {
        case 1: ((uint8_t *)cols.out[j])[pos] = ((const uint8_t *)cols.in[j])[r]; break;
        case 2: ((uint16_t *)cols.out[j])[pos] = ((const uint16_t *)cols.in[j])[r]; break;
        case 4: ((uint32_t *)cols.out[j])[pos] = ((const uint32_t *)cols.in[j])[r]; break;
        case 8: ((uint64_t *)cols.out[j])[pos] = ((const uint64_t *)cols.in[j])[r]; break;
        default: {
            const uint4 v = ((const uint4 *)cols.in[j])[r];
            ((uint4 *)cols.out[j])[pos] = v;
        }
        }
    }
}

// Writes perm (row ids), the partition ids and/or the columns at their partition-major position.
// STABLE: rank inside the wave by a ballot "match" loop and combine waves in order (exact
// IColumn::scatter order; cost grows with the distinct partitions per wave, so it is used for
// the exchange's small P).  !STABLE: one LDS atomic per row claims a slot inside the
// (partition, segment) range (order inside a range is unspecified; used by the aggregation
// bucket pass and the join radix pass, whose consumers are order-insensitive).
template <typename Sel, bool STABLE>
__global__ void __launch_bounds__(PT) part_scatter_kernel(Sel sel, RowPred pred, PartLayout L, const uint64_t *offs,
                                                          PCols cols, uint32_t *perm, uint32_t *part_out) {
    extern __shared__ __attribute__((aligned(16))) uint64_t run[]; // P running bases, then 4xP wave counts
    uint32_t *wcnt = reinterpret_cast<uint32_t *>(run + L.P);        // [4][P] (STABLE only)
    uint32_t(*crc)[256] = reinterpret_cast<uint32_t(*)[256]>(wcnt + (STABLE ? 4 * ((L.P + 3) & ~3u) : 0));
    for (uint32_t p = threadIdx.x; p < L.P; p += PT) {
        run[p] = offs[(int64_t)p * L.G + blockIdx.x];
        if constexpr (STABLE) wcnt[p] = wcnt[L.P + p] = wcnt[2 * L.P + p] = wcnt[3 * L.P + p] = 0;
    }
    if constexpr (Sel::needs_crc) load_crc_lds(crc);
    __syncthreads();
    const int64_t begin = (int64_t)blockIdx.x * L.seg;
    int64_t end = begin + L.seg;
    if (end > L.n) end = L.n;
    if constexpr (!STABLE) {
        for (int64_t r = begin + threadIdx.x; r < end; r += PT) {
            if (!pred(r)) continue;
            const uint32_t p = sel(crc, r);
            if (p >= L.P) continue;
            const uint64_t pos = atomicAdd((unsigned long long *)&run[p], 1ull);
            if (perm) perm[pos] = (uint32_t)r;
            if (part_out) part_out[pos] = p;
            scatter_row(cols, r, pos);
        }
        return;
    } else {
        const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        for (int64_t base = begin; base < end; base += PT) {
            const int64_t r = base + threadIdx.x;
            bool valid = r < end && pred(r);
            uint32_t p = valid ? sel(crc, r) : 0xFFFFFFFFu;
            valid = valid && p < L.P;
            uint64_t active = ballot(valid);
            uint32_t rank = 0, cnt = 0;
            bool leader = false;
            while (active) {
                const int lead = __ffsll((unsigned long long)active) - 1;
                const uint32_t lp = __shfl(p, lead, 64);
                const uint64_t m = ballot(valid && p == lp);
                if (valid && p == lp) {
                    rank = mbcnt(m);
                    cnt = (uint32_t)__popcll(m);
                    leader = (int)lane == lead;
                }
                active &= ~m;
            }
            if (leader) wcnt[wave * L.P + p] = cnt;
            __syncthreads();
            uint64_t pos = 0;
            if (valid) {
                pos = run[p] + rank;
                for (unsigned w = 0; w < wave; ++w) pos += wcnt[w * L.P + p];
            }
            __syncthreads();
            if (leader) {
                atomicAdd((unsigned long long *)&run[p], (unsigned long long)cnt);
                wcnt[wave * L.P + p] = 0;
            }
            if (valid) {
                if (perm) perm[pos] = (uint32_t)r;
                if (part_out) part_out[pos] = p;
                scatter_row(cols, r, pos);
            }
            __syncthreads();
        }
    }
}

inline size_t hist_lds_bytes(uint32_t P, bool crc) { return ((P + 3) & ~3u) * 4 + (crc ? 8192 : 0); }
inline size_t scatter_lds_bytes(uint32_t P, bool crc, bool stable) {
    return (size_t)P * 8 + (stable ? 4 * ((P + 3) & ~3u) * 4 : 0) + (crc ? 8192 : 0);
}

// Runs hist -> scan -> scatter.  offsets_out: device u64[P+1] partition offsets (optional).
// `tmp` must provide part_tmp_bytes(L) bytes.
inline size_t part_tmp_bytes(const PartLayout &L) {
    int64_t e = (int64_t)L.P * L.G;
    return ((size_t)e * 4 + 255) / 256 * 256 + ((size_t)(e + 1) * 8 + 255) / 256 * 256 + scan_tmp_bytes(e) + 256;
}

__global__ void gather_part_offsets_kernel(const uint64_t *offs, PartLayout L, uint64_t *out);

template <typename Sel, bool STABLE = true>
int run_partition(Ctx *ctx, const Sel &sel, const RowPred &pred, const PartLayout &L, const PCols &cols,
                  uint32_t *perm, uint32_t *part_out, uint64_t *offsets_out, void *tmp,
                  const char *hist_name = "part.hist", const char *scatter_name = "part.scatter") {
    TFG_CHECK(L.P >= 1 && L.P <= (STABLE ? PMAX : PMAX_UNSTABLE), TFG_ERR_INVALID_ARG, "partition count %u out of range", L.P);
    const int64_t e = (int64_t)L.P * L.G;
    char *t = (char *)tmp;
    uint32_t *counts = (uint32_t *)t;
    t += ((size_t)e * 4 + 255) / 256 * 256;
    uint64_t *offs = (uint64_t *)t;
    t += ((size_t)(e + 1) * 8 + 255) / 256 * 256;
    void *scan_tmp = t;
    if (L.n > 0) {
        { ProfScope _ps(ctx, hist_name);
        hipLaunchKernelGGL(part_hist_kernel<Sel>, dim3(L.G), dim3(PT), hist_lds_bytes(L.P, Sel::needs_crc), ctx->stream,
                           sel, pred, L, counts);
        }
        TFG_LAUNCH_CHECK();
    } else {
        TFG_HIP(hipMemsetAsync(counts, 0, (size_t)e * 4, ctx->stream));
    }
    if (int rc = exclusive_scan_u32(ctx, counts, offs, e, scan_tmp)) return rc;
    if (L.n > 0 && (perm || part_out || cols.ncols > 0)) {
        { ProfScope _ps(ctx, scatter_name);
        hipLaunchKernelGGL((part_scatter_kernel<Sel, STABLE>), dim3(L.G), dim3(PT),
                           scatter_lds_bytes(L.P, Sel::needs_crc, STABLE), ctx->stream, sel, pred, L, offs, cols, perm,
                           part_out);
        }
        TFG_LAUNCH_CHECK();
    }
    if (offsets_out) {
        hipLaunchKernelGGL(gather_part_offsets_kernel, dim3((L.P + 1 + 255) / 256), dim3(256), 0, ctx->stream, offs, L,
                           offsets_out);
        TFG_LAUNCH_CHECK();
    }
    return TFG_OK;
}

} // namespace tfg
