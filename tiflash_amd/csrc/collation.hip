// collation.hip — sort keys of the case-insensitive collators (see collation.h for the reference map).
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "collation.h"
#include "collation_data.h"
#include "uca_data.h"

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

// whole: the row with its terminating '\0' and no trim (the bytes SingleValueDataString compares,
// getDataAtWithTerminatingZero: a padding collator's right-trim stops at the '\0')
__device__ __forceinline__ RowSpan row_span(const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                                            int64_t r, bool whole) {
    RowSpan sp{chars, 0, chars};
    if (nullmap && nullmap[r]) return sp;
    const uint64_t b = r ? offsets[r - 1] : 0, e = offsets[r];
    sp.s = chars + b;
    sp.limit = chars + e;
    if (whole) {
        sp.len = e - b;
        return sp;
    }
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
                               const uint32_t *s32, const uint64_t *s64, int64_t n, bool whole, uint64_t *len_out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const RowSpan sp = row_span(chars, offsets, nullmap, pick(s32, s64, i), whole);
        uint64_t off = 0, nc = 0;
        while (off < sp.len) {
            (void)decode_utf8(sp, off);
            ++nc;
        }
        len_out[i] = 2 * nc + 1; // two weight bytes a character, then '\0'
    }
}

// every row writes inside its slot [start[i], start[i + 1]) of the `total` bytes (the lengths
// pass computed the slots): a scan that disagrees can never write outside the buffer
__device__ __forceinline__ void put_byte(uint8_t *&o, const uint8_t *lim, uint8_t v) {
    if (o < lim) *o = v;
    ++o;
}

__global__ void gci_write_kernel(const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                                 const uint32_t *s32, const uint64_t *s64, int64_t n, bool whole, const uint64_t *start,
                                 uint64_t total, uint8_t *out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const RowSpan sp = row_span(chars, offsets, nullmap, pick(s32, s64, i), whole);
        const uint64_t b = start[i], e = start[i + 1];
        if (b > e || e > total) continue;
        uint8_t *o = out + b;
        const uint8_t *lim = out + e;
        uint64_t off = 0;
        while (off < sp.len) {
            const uint32_t w = gci_weight(gci_runs_dev, decode_utf8(sp, off));
            put_byte(o, lim, (uint8_t)(w >> 8));
            put_byte(o, lim, (uint8_t)w);
        }
        put_byte(o, lim, 0);
    }
}

// ---------------------------------------------------------------- UCA (unicode_ci, 0900_ai_ci)
// The weight LUTs live expanded in device memory (0.5 MB + 1.4 MB, one per device), filled once
// from their runs (uca_data.h); long weights are searched in a 22 / 27-entry table.
struct UcaRun {
    uint32_t start, count;
    uint64_t base, delta;
};
struct UcaLong {
    uint32_t cp;
    uint64_t first, second;
};
__device__ const UcaRun uca0400_runs_dev[TFG_UCA0400_NRUNS] = {TFG_UCA0400_RUNS_INIT};
__device__ const UcaRun uca0900_runs_dev[TFG_UCA0900_NRUNS] = {TFG_UCA0900_RUNS_INIT};
__constant__ UcaLong uca0400_long_dev[TFG_UCA0400_NLONG] = {TFG_UCA0400_LONG_INIT};
__constant__ UcaLong uca0900_long_dev[TFG_UCA0900_NLONG] = {TFG_UCA0900_LONG_INIT};
__device__ uint64_t uca0400_lut_dev[TFG_UCA0400_SIZE];
__device__ uint64_t uca0900_lut_dev[TFG_UCA0900_SIZE];

// one workgroup per run
__global__ void uca_expand_kernel(int v0900) {
    const UcaRun r = v0900 ? uca0900_runs_dev[blockIdx.x] : uca0400_runs_dev[blockIdx.x];
    uint64_t *lut = v0900 ? uca0900_lut_dev : uca0400_lut_dev;
    for (uint32_t k = threadIdx.x; k < r.count; k += blockDim.x) lut[r.start + k] = r.base + (uint64_t)k * r.delta;
}

// Unicode0400::weight / Unicode0900::weight (Collator.cpp:703-727, 791-816): false = a
// zero-weight character (skipped)
template <bool V0900>
__device__ __forceinline__ bool uca_weight(uint32_t r, uint64_t &first, uint64_t &second) {
    second = 0;
    if (!V0900 && r > 0xFFFFu) {
        first = 0xFFFDu;
        return true;
    }
    if (V0900 && r >= (uint32_t)TFG_UCA0900_SIZE) { // implicit weight (the reference reads one past its LUT at 0x2CEA1)
        first = (uint64_t)(r >> 15) + 0xFBC0u + ((uint64_t)((r & 0x7FFFu) | 0x8000u) << 16);
        return true;
    }
    const uint64_t w = V0900 ? uca0900_lut_dev[r] : uca0400_lut_dev[r];
    if (w == 0) return false;
    if (w != 0xFFFDu) {
        first = w;
        return true;
    }
    first = 0; // weightLutLongMap's default entry {0, 0}
    const int nl = V0900 ? TFG_UCA0900_NLONG : TFG_UCA0400_NLONG;
    for (int i = 0; i < nl; ++i) {
        const UcaLong &e = V0900 ? uca0900_long_dev[i] : uca0400_long_dev[i];
        if (e.cp == r) {
            first = e.first;
            second = e.second;
        }
    }
    return true;
}

// bytes writeResult (Collator.h:336-344) emits for a weight word: two per non-zero 16-bit chunk
// from the low end
__device__ __forceinline__ uint32_t uca_chunk_bytes(uint64_t w) { return w ? 2u * ((64u - __clzll(w) + 15u) / 16u) : 0u; }

// 0400 pads (right-trims ' '); 0900 keeps trailing spaces
template <bool V0900>
__device__ __forceinline__ RowSpan uca_span(const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap, int64_t r,
                                            bool whole) {
    RowSpan sp = row_span(chars, offsets, nullmap, r, whole);
    if (V0900 && !whole && !(nullmap && nullmap[r])) sp.len = (uint64_t)(sp.limit - sp.s) - 1;
    return sp;
}

template <bool V0900>
__global__ void uca_len_kernel(const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                               const uint32_t *s32, const uint64_t *s64, int64_t n, bool whole, uint64_t *len_out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const RowSpan sp = uca_span<V0900>(chars, offsets, nullmap, pick(s32, s64, i), whole);
        uint64_t off = 0, bytes = 0;
        while (off < sp.len) {
            uint64_t f, s;
            if (uca_weight<V0900>(decode_utf8(sp, off), f, s)) bytes += uca_chunk_bytes(f) + uca_chunk_bytes(s);
        }
        len_out[i] = bytes + 1; // then '\0'
    }
}

template <bool V0900>
__global__ void uca_write_kernel(const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                                 const uint32_t *s32, const uint64_t *s64, int64_t n, bool whole, const uint64_t *start,
                                 uint64_t total, uint8_t *out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const RowSpan sp = uca_span<V0900>(chars, offsets, nullmap, pick(s32, s64, i), whole);
        const uint64_t b = start[i], e = start[i + 1];
        if (b > e || e > total) continue;
        uint8_t *o = out + b;
        const uint8_t *lim = out + e;
        uint64_t off = 0;
        while (off < sp.len) {
            uint64_t w[2];
            if (!uca_weight<V0900>(decode_utf8(sp, off), w[0], w[1])) continue;
            for (int h = 0; h < 2; ++h)
                for (uint64_t x = w[h]; x != 0; x >>= 16) {
                    put_byte(o, lim, (uint8_t)(x >> 8));
                    put_byte(o, lim, (uint8_t)x);
                }
        }
        put_byte(o, lim, 0);
    }
}

// the expanded LUTs of device `dev` (filled on its first UCA collation)
int uca_ready(Ctx *ctx) {
    static std::mutex mu;
    static bool ready[64];
    std::lock_guard<std::mutex> lk(mu);
    TFG_CHECK(ctx->device >= 0 && ctx->device < 64, TFG_ERR_INVALID_ARG, "device %d", ctx->device);
    if (ready[ctx->device]) return TFG_OK;
    hipLaunchKernelGGL(uca_expand_kernel, dim3(TFG_UCA0400_NRUNS), dim3(256), 0, ctx->stream, 0);
    hipLaunchKernelGGL(uca_expand_kernel, dim3(TFG_UCA0900_NRUNS), dim3(256), 0, ctx->stream, 1);
    TFG_LAUNCH_CHECK();
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    ready[ctx->device] = true;
    return TFG_OK;
}

} // namespace

// The sort keys and their scan live in the context's call arena (DevArena): no allocation in
// steady state, and nothing to free — the arena is reused by the next call on the same stream.
// TFG_EXP_POOL (experiment builds only): the stream-ordered pool of round 5 instead, with an
// allocation log (TFG_POOLDBG=1) for the fault analysis of DESIGN §4.3.
#ifdef TFG_EXP_POOL
static bool pool_dbg() {
    static const bool on = getenv("TFG_POOLDBG") != nullptr;
    return on;
}
// Non-faulting form of the experiment: the pool never returns memory to the system (release
// threshold = max), so a read after a free sees the poison written at the free (0xFF: offsets far
// past every buffer, caught by ref_cmp's bounds) instead of an unmapped page; every block carries
// 4 KB of canary after its bytes, checked at the free (an overrun by its own writer or a
// neighbour's wild write)
constexpr size_t CANARY = 4096;
struct PoolBlock {
    void *p;
    size_t bytes;
};
static std::vector<PoolBlock> &pool_blocks() {
    static std::vector<PoolBlock> v;
    return v;
}
static bool pool_env(const char *name, bool dflt) {
    const char *v = getenv(name);
    return v && *v ? *v == '1' : dflt;
}
static int coll_alloc(Ctx *ctx, void **p, size_t bytes, const char *what) {
    static bool once = [] {
        if (!pool_env("TFG_POOL_KEEP", true)) return true; // the default threshold (0: trim at syncs)
        hipMemPool_t pool;
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
            uint64_t thr = ~0ull;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
        }
        return true;
    }();
    (void)once;
    TFG_HIP(hipMallocAsync(p, bytes + CANARY, ctx->stream));
    TFG_HIP(hipMemsetAsync((char *)*p + bytes, 0xA5, CANARY, ctx->stream));
    pool_blocks().push_back({*p, bytes});
    if (pool_dbg()) fprintf(stderr, "POOL alloc %s %p +%zu (stream %p)\n", what, *p, bytes, (void *)ctx->stream);
    return TFG_OK;
}
static void coll_free(Ctx *ctx, void *p, const char *what) {
    if (!p) return;
    size_t bytes = 0;
    auto &v = pool_blocks();
    for (size_t i = 0; i < v.size(); ++i)
        if (v[i].p == p) {
            bytes = v[i].bytes;
            v.erase(v.begin() + (long)i);
            break;
        }
    static const bool sync_check = pool_env("TFG_POOL_SYNCFREE", false); // the canary read-back syncs
    std::vector<uint8_t> c(CANARY);
    if (sync_check && hipMemcpyAsync(c.data(), (char *)p + bytes, CANARY, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess &&
        hipStreamSynchronize(ctx->stream) == hipSuccess) {
        size_t bad = 0, first = CANARY;
        for (size_t i = 0; i < CANARY; ++i)
            if (c[i] != 0xA5) bad++, first = std::min(first, i);
        if (bad) fprintf(stderr, "POOL CANARY %s %p +%zu: %zu bytes overwritten from +%zu\n", what, p, bytes, bad, first);
    }
    if (pool_dbg()) fprintf(stderr, "POOL free %s %p\n", what, p);
    (void)hipMemsetAsync(p, 0xFF, bytes, ctx->stream); // poison: a later reader sees offsets past everything
    (void)hipFreeAsync(p, ctx->stream);
}
#else
static int coll_alloc(Ctx *ctx, void **p, size_t bytes, const char *) { return arena_alloc(ctx, bytes, p); }
static void coll_free(Ctx *, void *, const char *) {}
#endif

CollatedStrings::~CollatedStrings() {
    if (!ctx) return;
    coll_free(ctx, chars, "chars");
    coll_free(ctx, scan, "scan");
    arena_drop(ctx);
}

int collate_strings(Ctx *ctx, int collator, const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                    const uint32_t *sel32, const uint64_t *sel64, int64_t n, CollatedStrings &out, bool whole) {
    TFG_CHECK(collator_transforms(collator), TFG_ERR_NOT_IMPLEMENTED, "collator %d has no sort-key transform",
              collator);
    TFG_CHECK(!out.ctx, TFG_ERR_LOGICAL, "collated column reused");
    const bool uca = collator != TFG_COLLATOR_GENERAL_CI, v0900 = collator == TFG_COLLATOR_UCA0900_AI_CI;
    if (uca)
        if (int rc = uca_ready(ctx)) return rc;
    TFG_CHECK(n >= 0 && n <= ((int64_t)1 << 26), TFG_ERR_INVALID_ARG, "collated column of %lld rows", (long long)n);
    arena_hold(ctx); // dropped by out's destructor
    out.ctx = ctx;
    out.rows = n;
    if (int rc = coll_alloc(ctx, (void **)&out.scan, (size_t)(n + 1) * 8, "scan")) return rc;
    if (n == 0) {
        TFG_HIP(hipMemsetAsync(out.scan, 0, 8, ctx->stream));
        return coll_alloc(ctx, (void **)&out.chars, 16, "chars");
    }
    TFG_CHECK(chars && offsets, TFG_ERR_INVALID_ARG, "String column needs its chars and offsets");
    // the lengths and the scan's work space (dead after the total's read-back)
    uint64_t *len = nullptr;
    void *tmp = nullptr;
    if (int rc = coll_alloc(ctx, (void **)&len, (size_t)n * 8, "len")) return rc;
    const unsigned grid = stream_grid(n, 256, 4096);
    if (!uca)
        hipLaunchKernelGGL(gci_len_kernel, dim3(grid), dim3(256), 0, ctx->stream, chars, offsets, nullmap, sel32, sel64,
                           n, whole, len);
    else if (v0900)
        hipLaunchKernelGGL(uca_len_kernel<true>, dim3(grid), dim3(256), 0, ctx->stream, chars, offsets, nullmap, sel32,
                           sel64, n, whole, len);
    else
        hipLaunchKernelGGL(uca_len_kernel<false>, dim3(grid), dim3(256), 0, ctx->stream, chars, offsets, nullmap, sel32,
                           sel64, n, whole, len);
    TFG_LAUNCH_CHECK();
    if (int rc = coll_alloc(ctx, &tmp, scan_tmp_bytes(n) + 256, "tmp")) return rc;
    if (int rc = exclusive_scan_u64(ctx, len, out.scan, n, tmp)) return rc;
    uint64_t total = 0;
    if (int rc = read_back_u64(ctx, out.scan + n, &total, 1)) return rc; // synchronizes the stream
    coll_free(ctx, len, "len");
    coll_free(ctx, tmp, "tmp");
    if (int rc = coll_alloc(ctx, (void **)&out.chars, total + 16, "chars")) return rc;
    out.bytes = total;
    if (!uca)
        hipLaunchKernelGGL(gci_write_kernel, dim3(grid), dim3(256), 0, ctx->stream, chars, offsets, nullmap, sel32, sel64,
                           n, whole, out.scan, total, out.chars);
    else if (v0900)
        hipLaunchKernelGGL(uca_write_kernel<true>, dim3(grid), dim3(256), 0, ctx->stream, chars, offsets, nullmap, sel32,
                           sel64, n, whole, out.scan, total, out.chars);
    else
        hipLaunchKernelGGL(uca_write_kernel<false>, dim3(grid), dim3(256), 0, ctx->stream, chars, offsets, nullmap, sel32,
                           sel64, n, whole, out.scan, total, out.chars);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

} // namespace tfg
