// hash.hip — WeakHash32 (a22), fillSelector (a23), stable scatter / gather and the fused
// HashBaseWriterHelper::scatterColumns (a23/a24) for the MPP hash exchange.
//
// Reference: IColumn::updateWeakHash32 (Columns/ColumnVector.cpp:499-535, ColumnNullable.cpp:131-173,
// ColumnString.cpp:1228-1327), intHashCRC32 (Common/HashTable/Hash.h:70-214), fillSelector
// (Flash/Mpp/HashBaseWriterHelper.cpp:46-84), scatterColumns (:144-172), IColumn::scatter
// (Columns/IColumn.h:655-721).  CRC32-C is computed in software (slicing-by-8 tables in LDS) and is
// bit-identical to the reference's _mm_crc32_u64, so partition row sets match exactly.
#include "collation.h"
#include "common.h"
#include "partition.h"

namespace tfg {

__global__ void gather_part_offsets_kernel(const uint64_t *offs, PartLayout L, uint64_t *out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < L.P) out[p] = offs[(int64_t)p * L.G];
    else if (p == L.P) out[p] = offs[(int64_t)L.P * L.G];
}

__global__ void weak_hash_init_kernel(uint32_t *h, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        h[i] = 0xFFFFFFFFu;
}

// sel (optional, BlockInfo::selective): h[i] hashes row sel[i] (ColumnVector.cpp:500-535)
__global__ void __launch_bounds__(256) weak_hash_update_kernel(KeyCols k, const uint64_t *sel, int64_t n, uint32_t *h) {
    __shared__ uint32_t crc[8][256];
    load_crc_lds(crc);
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        h[i] = hash_key_row(crc, k, sel ? (int64_t)sel[i] : i, h[i]);
}

// ::updateWeakHash32(bytes) (Hash.h:148-214): 8-byte words, then a length-tagged tail.
__device__ __forceinline__ uint64_t load_u64_unaligned(const uint8_t *p) {
    uint64_t v = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) v |= (uint64_t)p[b] << (8 * b);
    return v;
}

__device__ uint32_t weak_hash_bytes(const uint32_t (*t)[256], const uint8_t *pos, uint64_t size, uint32_t h) {
    if (size < 8) {
        uint64_t value = 0;
        for (uint64_t b = 0; b < size; ++b) value |= (uint64_t)pos[b] << (8 * b);
        value |= (uint64_t)size << 56;
        return crc32c_u64(t, h, value);
    }
    const uint8_t *end = pos + size;
    while (pos + 8 <= end) {
        h = crc32c_u64(t, h, load_u64_unaligned(pos));
        pos += 8;
    }
    if (pos < end) {
        const unsigned tail = (unsigned)(end - pos);
        uint64_t word = load_u64_unaligned(end - 8);
        word &= (~(uint64_t)0) << (8 * (8 - tail));
        word |= tail;
        h = crc32c_u64(t, h, word);
    }
    return h;
}

__global__ void __launch_bounds__(256) weak_hash_string_kernel(const uint8_t *chars, const uint64_t *offsets,
                                                              const uint8_t *nullmap, const uint64_t *sel, int64_t n,
                                                              int collator, int compact, uint32_t *h) {
    __shared__ uint32_t crc[8][256];
    load_crc_lds(crc);
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = sel ? (int64_t)sel[i] : i; // ColumnString.cpp:1256-1294 (selective rows)
        if (nullmap && nullmap[r]) continue;
        const int64_t rs = compact ? i : r; // a collated column holds row sel[i] at row i
        const uint64_t prev = rs ? offsets[rs - 1] : 0;
        uint64_t len = offsets[rs] - prev - 1; // size - 1: the trailing '\0' is excluded
        const uint8_t *s = chars + prev;
        if (collator == TFG_COLLATOR_BIN_PADDING)
            while (len > 0 && s[len - 1] == ' ') --len;
        h[i] = weak_hash_bytes(crc, s, len, h[i]);
    }
}

__global__ void fill_selector_kernel(const uint32_t *h, int64_t n, uint32_t parts, uint32_t fgs, uint32_t *sel) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t s = ((uint64_t)h[i] * parts) >> 32;
        if (fgs) s = s * fgs + h[i] % fgs;
        sel[i] = (uint32_t)s;
    }
}

// out[i] = selective[perm[i]] (perm null: selective[i]): the partition permutation of the
// selective rows mapped back to block rows (IColumn::scatter with a BlockSelective)
__global__ void selective_perm_kernel(const uint64_t *sel, const uint32_t *perm, int64_t n, uint32_t *out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)sel[perm ? perm[i] : i];
}

struct alignas(16) Bytes32 { // Decimal256 values
    uint4 a, b;
};
template <int W>
__global__ void gather_kernel(const uint32_t *perm, int64_t n, const void *in, void *out) {
    using E = typename std::conditional<W == 32, Bytes32, typename std::conditional<W == 16, uint4,
              typename std::conditional<W == 8, uint64_t,
              typename std::conditional<W == 4, uint32_t,
              typename std::conditional<W == 2, uint16_t, uint8_t>::type>::type>::type>::type>::type;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t r = perm[i];
        E v;
        if (r == 0xFFFFFFFFu) memset(&v, 0, sizeof(E));
        else v = ((const E *)in)[r];
        ((E *)out)[i] = v;
    }
}

static int make_keycols(int nkeys, const int *idx, const int *types, const void *const *cols,
                        const uint8_t *const *nullmaps, KeyCols &k) {
    TFG_CHECK(nkeys >= 1 && nkeys <= 4, TFG_ERR_INVALID_ARG, "nkeys %d out of range [1,4]", nkeys);
    k.nkeys = nkeys;
    for (int j = 0; j < nkeys; ++j) {
        int c = idx ? idx[j] : j;
        int t = types[c];
        TFG_CHECK(type_width(t) > 0 && type_width(t) <= 16, TFG_ERR_ILLEGAL_TYPE, "weak hash of type %d is not supported", t);
        k.col[j] = cols[c];
        k.nullmap[j] = nullmaps ? nullmaps[c] : nullptr;
        k.type[j] = t;
    }
    return TFG_OK;
}

} // namespace tfg

using namespace tfg;

extern "C" {

int tfg_weak_hash_init(tfg_ctx *ctx, uint32_t *h, int64_t n) {
    TFG_CHECK(ctx && (n == 0 || h), TFG_ERR_INVALID_ARG, "null argument");
    if (n <= 0) return TFG_OK;
    hipLaunchKernelGGL(weak_hash_init_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, ctx->stream, h, n);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_weak_hash_update(tfg_ctx *ctx, int type, const void *col, const uint8_t *nullmap, int64_t n, uint32_t *h) {
    return tfg_weak_hash_update_selective(ctx, type, col, nullmap, nullptr, n, h);
}

int tfg_weak_hash_update_selective(tfg_ctx *ctx, int type, const void *col, const uint8_t *nullmap,
                                   const uint64_t *selective, int64_t n, uint32_t *h) {
    TFG_CHECK(ctx && (n == 0 || (col && h)), TFG_ERR_INVALID_ARG, "null argument");
    KeyCols k{};
    const void *cols[1] = {col};
    const uint8_t *nms[1] = {nullmap};
    int types[1] = {type};
    if (int rc = make_keycols(1, nullptr, types, cols, nms, k)) return rc;
    if (n <= 0) return TFG_OK;
    { ProfScope _ps(ctx, "hash.weak");
    hipLaunchKernelGGL(weak_hash_update_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, ctx->stream, k, selective,
                       n, h);
    }
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_weak_hash_update_string(tfg_ctx *ctx, const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                                int64_t n, int collator, uint32_t *h) {
    return tfg_weak_hash_update_string_selective(ctx, chars, offsets, nullmap, nullptr, n, collator, h);
}

int tfg_weak_hash_update_string_selective(tfg_ctx *ctx, const uint8_t *chars, const uint64_t *offsets,
                                          const uint8_t *nullmap, const uint64_t *selective, int64_t n, int collator,
                                          uint32_t *h) {
    TFG_CHECK(ctx && (n == 0 || (chars && offsets && h)), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(collator_known(collator), TFG_ERR_NOT_IMPLEMENTED, "collator %d not supported", collator);
    if (n <= 0) return TFG_OK;
    if (collator_transforms(collator)) { // ColumnString.cpp:1244: the collator's sort key is hashed
        CollatedStrings cs;
        if (int rc = collate_strings(ctx, collator, chars, offsets, nullmap, nullptr, selective, n, cs)) return rc;
        hipLaunchKernelGGL(weak_hash_string_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, ctx->stream,
                           cs.chars, cs.offsets(), nullmap, selective, n, (int)TFG_COLLATOR_NONE, 1, h);
        TFG_LAUNCH_CHECK();
        return TFG_OK;
    }
    hipLaunchKernelGGL(weak_hash_string_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, ctx->stream, chars,
                       offsets, nullmap, selective, n, collator, 0, h);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_selective_perm(tfg_ctx *ctx, const uint64_t *selective, const uint32_t *perm, int64_t n, uint32_t *out_perm) {
    TFG_CHECK(ctx && (n == 0 || (selective && out_perm)), TFG_ERR_INVALID_ARG, "null argument");
    if (n <= 0) return TFG_OK;
    hipLaunchKernelGGL(selective_perm_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, ctx->stream, selective, perm,
                       n, out_perm);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_fill_selector(tfg_ctx *ctx, const uint32_t *h, int64_t n, uint32_t part_num, uint32_t fgs,
                      uint32_t *out_selector) {
    TFG_CHECK(ctx && (n == 0 || (h && out_selector)), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(part_num >= 1, TFG_ERR_INVALID_ARG, "part_num must be >= 1");
    if (n <= 0) return TFG_OK;
    hipLaunchKernelGGL(fill_selector_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, ctx->stream, h, n, part_num,
                       fgs, out_selector);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_partition(tfg_ctx *ctx, const uint32_t *selector, int64_t n, uint32_t num_parts, uint32_t *out_perm,
                  uint64_t *out_offsets, uint64_t *out_offsets_host) {
    TFG_CHECK(ctx && (n == 0 || selector) && out_offsets, TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(n >= 0 && n < (int64_t)0xFFFFFFFFll, TFG_ERR_INVALID_ARG, "row count out of range");
    TFG_CHECK(num_parts >= 1 && num_parts <= (uint32_t)PMAX, TFG_ERR_INVALID_ARG, "num_parts %u out of range", num_parts);
    if (failpoint("partition")) return fail(TFG_ERR_FAULT_INJECTED, "failpoint partition");
    PartLayout L = make_layout(n, num_parts);
    void *tmp;
    if (int rc = scratch_get(ctx, part_tmp_bytes(L), &tmp)) return rc;
    PCols cols{};
    RowPred pred{};
    if (int rc = run_partition(ctx, SelArray{selector}, pred, L, cols, out_perm, nullptr, out_offsets, tmp)) return rc;
    if (out_offsets_host) {
        TFG_HIP(hipMemcpyAsync(out_offsets_host, out_offsets, (num_parts + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                               ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
    }
    return TFG_OK;
}

int tfg_gather(tfg_ctx *ctx, const uint32_t *perm, int64_t n, int ncols, const void *const *cols, const int *widths,
               void *const *outs) {
    TFG_CHECK(ctx && (n == 0 || perm), TFG_ERR_INVALID_ARG, "null argument");
    if (n <= 0) return TFG_OK;
    unsigned grid = stream_grid(n, 256, 8192);
    for (int j = 0; j < ncols; ++j) {
        TFG_CHECK(cols[j] && outs[j], TFG_ERR_INVALID_ARG, "null column pointer");
        switch (widths[j]) {
        case 1: hipLaunchKernelGGL(gather_kernel<1>, dim3(grid), dim3(256), 0, ctx->stream, perm, n, cols[j], outs[j]); break;
        case 2: hipLaunchKernelGGL(gather_kernel<2>, dim3(grid), dim3(256), 0, ctx->stream, perm, n, cols[j], outs[j]); break;
        case 4: hipLaunchKernelGGL(gather_kernel<4>, dim3(grid), dim3(256), 0, ctx->stream, perm, n, cols[j], outs[j]); break;
        case 8: hipLaunchKernelGGL(gather_kernel<8>, dim3(grid), dim3(256), 0, ctx->stream, perm, n, cols[j], outs[j]); break;
        case 16: hipLaunchKernelGGL(gather_kernel<16>, dim3(grid), dim3(256), 0, ctx->stream, perm, n, cols[j], outs[j]); break;
        case 32: hipLaunchKernelGGL(gather_kernel<32>, dim3(grid), dim3(256), 0, ctx->stream, perm, n, cols[j], outs[j]); break;
        default: return fail(TFG_ERR_INVALID_ARG, "bad column width %d", widths[j]);
        }
    }
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_hash_partition(tfg_ctx *ctx, int64_t n, int nkeys, const int *key_col_idx, int ncols, const int *types,
                       const void *const *cols, const uint8_t *const *nullmaps, uint32_t part_num, void *const *outs,
                       uint64_t *out_offsets, uint64_t *out_offsets_host) {
    TFG_CHECK(ctx && types && cols && outs && out_offsets && key_col_idx, TFG_ERR_INVALID_ARG, "null argument");
    if (n == 0) { // every partition empty
        TFG_HIP(hipMemsetAsync(out_offsets, 0, (part_num + 1) * sizeof(uint64_t), ctx->stream));
        if (out_offsets_host) memset(out_offsets_host, 0, (part_num + 1) * sizeof(uint64_t));
        return TFG_OK;
    }
    TFG_CHECK(ncols >= 1 && ncols <= PCOLS, TFG_ERR_INVALID_ARG, "ncols %d out of range [1,%d]", ncols, PCOLS);
    TFG_CHECK(part_num >= 1 && part_num <= (uint32_t)PMAX, TFG_ERR_INVALID_ARG, "part_num %u out of range", part_num);
    TFG_CHECK(n >= 0 && n < (int64_t)0xFFFFFFFFll, TFG_ERR_INVALID_ARG, "row count out of range");
    for (int j = 0; j < nkeys; ++j)
        TFG_CHECK(key_col_idx[j] >= 0 && key_col_idx[j] < ncols, TFG_ERR_INVALID_ARG, "key column index out of range");
    if (failpoint("hash_partition")) return fail(TFG_ERR_FAULT_INJECTED, "failpoint hash_partition");
    SelHashMul sel{};
    if (int rc = make_keycols(nkeys, key_col_idx, types, cols, nullmaps, sel.k)) return rc;
    sel.parts = part_num;
    PCols pc{};
    pc.ncols = ncols;
    for (int j = 0; j < ncols; ++j) {
        size_t w = type_width(types[j]);
        TFG_CHECK(w > 0 && cols[j] && outs[j], TFG_ERR_INVALID_ARG, "bad column %d", j);
        pc.in[j] = cols[j];
        pc.out[j] = outs[j];
        pc.width[j] = (int)w;
    }
    PartLayout L = make_layout(n, part_num);
    void *tmp;
    if (int rc = scratch_get(ctx, part_tmp_bytes(L), &tmp)) return rc;
    RowPred pred{};
    if (int rc = run_partition(ctx, sel, pred, L, pc, nullptr, nullptr, out_offsets, tmp)) return rc;
    if (out_offsets_host) {
        TFG_HIP(hipMemcpyAsync(out_offsets_host, out_offsets, (part_num + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                               ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
    }
    return TFG_OK;
}

} // extern "C"
