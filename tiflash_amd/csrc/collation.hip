// collation.hip — utf8mb4_general_ci sort keys (see collation.h for the reference map).
#include "collation.h"
#include "collation_data.h"

namespace tfg {

namespace {

__constant__ uint32_t gci_runs_dev[TFG_GCI_RUNS][3] = {TFG_GCI_RUNS_INIT};

// weight of a code point: binary search of the runs (collation_data.h), else the code point
__device__ __forceinline__ uint32_t gci_weight(const uint32_t (*runs)[3], uint32_t c) {
    if (c > 0xFFFFu) return 0xFFFDu;
    int lo = 0, hi = TFG_GCI_RUNS - 1, hit = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (runs[mid][0] <= c) {
            hit = mid;
            lo = mid + 1;
        } else {
            hi = mid - 1;
        }
    }
    if (hit < 0 || c > runs[hit][1]) return c;
    const uint32_t v = runs[hit][2];
    return (v >> 16) ? (v & 0xFFFFu) : ((c + (uint32_t)(int32_t)(int16_t)(v & 0xFFFFu)) & 0xFFFFu);
}

struct RowSpan {
    const uint8_t *s;
    uint64_t len; // after the right-trim
    const uint8_t *limit; // one past the row's '\0'
};

__device__ __forceinline__ RowSpan row_span(const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                                            int64_t r) {
    RowSpan sp{chars, 0, chars};
    if (nullmap && nullmap[r]) return sp;
    const uint64_t b = r ? offsets[r - 1] : 0, e = offsets[r];
    sp.s = chars + b;
    sp.limit = chars + e;
    uint64_t len = e - b - 1; // ColumnString rows end with '\0'
    while (len > 0 && sp.s[len - 1] == ' ') --len;
    sp.len = len;
    return sp;
}

// decodeUtf8Char: the lead byte decides the length; continuation bytes are not validated.  A
// sequence truncated by the row's end reads the row's '\0' and then zeros (the reference reads
// on into the next row's bytes there: malformed UTF-8 only)
__device__ __forceinline__ uint32_t decode_utf8(const RowSpan &sp, uint64_t &off) {
    auto at = [&](uint64_t k) -> uint32_t { return sp.s + k < sp.limit ? sp.s[k] : 0u; };
    const uint32_t b0 = at(off);
    if (b0 < 0x80) {
        off += 1;
        return b0;
    }
    if (b0 < 0xE0) {
        const uint32_t c = (b0 & 0x1Fu) << 6 | (at(off + 1) & 0x3Fu);
        off += 2;
        return c;
    }
    if (b0 < 0xF0) {
        const uint32_t c = (b0 & 0x0Fu) << 12 | (at(off + 1) & 0x3Fu) << 6 | (at(off + 2) & 0x3Fu);
        off += 3;
        return c;
    }
    const uint32_t c = (b0 & 0x07u) << 18 | (at(off + 1) & 0x3Fu) << 12 | (at(off + 2) & 0x3Fu) << 6 | (at(off + 3) & 0x3Fu);
    off += 4;
    return c;
}

__device__ __forceinline__ int64_t pick(const uint32_t *s32, const uint64_t *s64, int64_t i) {
    return s32 ? (int64_t)s32[i] : s64 ? (int64_t)s64[i] : i;
}

__global__ void gci_len_kernel(const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                               const uint32_t *s32, const uint64_t *s64, int64_t n, uint64_t *len_out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const RowSpan sp = row_span(chars, offsets, nullmap, pick(s32, s64, i));
        uint64_t off = 0, nc = 0;
        while (off < sp.len) {
            (void)decode_utf8(sp, off);
            ++nc;
        }
        len_out[i] = 2 * nc + 1; // two weight bytes a character, then '\0'
    }
}

__global__ void gci_write_kernel(const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                                 const uint32_t *s32, const uint64_t *s64, int64_t n, const uint64_t *start,
                                 uint8_t *out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const RowSpan sp = row_span(chars, offsets, nullmap, pick(s32, s64, i));
        uint8_t *o = out + start[i];
        uint64_t off = 0;
        while (off < sp.len) {
            const uint32_t w = gci_weight(gci_runs_dev, decode_utf8(sp, off));
            *o++ = (uint8_t)(w >> 8);
            *o++ = (uint8_t)w;
        }
        *o = 0;
    }
}

} // namespace

CollatedStrings::~CollatedStrings() {
    if (!ctx) return;
    if (chars) (void)hipFreeAsync(chars, ctx->stream);
    if (scan) (void)hipFreeAsync(scan, ctx->stream);
}

int collate_strings(Ctx *ctx, int collator, const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                    const uint32_t *sel32, const uint64_t *sel64, int64_t n, CollatedStrings &out) {
    TFG_CHECK(collator == TFG_COLLATOR_GENERAL_CI, TFG_ERR_NOT_IMPLEMENTED, "collator %d has no sort-key transform",
              collator);
    TFG_CHECK(n >= 0 && n <= ((int64_t)1 << 26), TFG_ERR_INVALID_ARG, "collated column of %lld rows", (long long)n);
    out.ctx = ctx;
    out.rows = n;
    TFG_HIP(hipMallocAsync((void **)&out.scan, (size_t)(n + 1) * 8, ctx->stream));
    if (n == 0) {
        TFG_HIP(hipMemsetAsync(out.scan, 0, 8, ctx->stream));
        TFG_HIP(hipMallocAsync((void **)&out.chars, 16, ctx->stream));
        return TFG_OK;
    }
    TFG_CHECK(chars && offsets, TFG_ERR_INVALID_ARG, "String column needs its chars and offsets");
    uint64_t *len = nullptr;
    TFG_HIP(hipMallocAsync((void **)&len, (size_t)n * 8, ctx->stream));
    const unsigned grid = stream_grid(n, 256, 4096);
    hipLaunchKernelGGL(gci_len_kernel, dim3(grid), dim3(256), 0, ctx->stream, chars, offsets, nullmap, sel32, sel64, n,
                       len);
    TFG_LAUNCH_CHECK();
    void *tmp = nullptr;
    TFG_HIP(hipMallocAsync(&tmp, scan_tmp_bytes(n) + 256, ctx->stream));
    if (int rc = exclusive_scan_u64(ctx, len, out.scan, n, tmp)) return rc;
    uint64_t total = 0;
    if (int rc = read_back_u64(ctx, out.scan + n, &total, 1)) return rc;
    TFG_HIP(hipMallocAsync((void **)&out.chars, total + 16, ctx->stream));
    hipLaunchKernelGGL(gci_write_kernel, dim3(grid), dim3(256), 0, ctx->stream, chars, offsets, nullmap, sel32, sel64, n,
                       out.scan, out.chars);
    TFG_LAUNCH_CHECK();
    TFG_HIP(hipFreeAsync(len, ctx->stream));
    TFG_HIP(hipFreeAsync(tmp, ctx->stream));
    return TFG_OK;
}

} // namespace tfg
