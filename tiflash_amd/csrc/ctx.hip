// ctx.hip — context, memory, error state, and the device-wide scan used by every
// count -> scan -> write pipeline (filter, partition, aggregation, join).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

#include "common.h"

namespace tfg {



static thread_local std::string g_last_error;

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

int fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    set_error("HIP error %d (%s) in %s", (int)e, hipGetErrorString(e), what);
    return e == hipErrorOutOfMemory ? TFG_ERR_OOM : TFG_ERR_HIP;
}

bool sync_check() {
    static const bool on = [] {
        const char *v = getenv("TFG_SYNC_CHECK");
        return v && *v && strcmp(v, "0") != 0;
    }();
    return on;
}

bool failpoint(const char *name) {
    const char *fp = getenv("TFG_FAILPOINT");
    return fp && strcmp(fp, name) == 0;
}

size_t type_width(int t) {
    switch (t) {
    case TFG_INT8: case TFG_UINT8: return 1;
    case TFG_INT16: case TFG_UINT16: return 2;
    case TFG_INT32: case TFG_UINT32: case TFG_FLOAT32: case TFG_DECIMAL32: return 4;
    case TFG_INT64: case TFG_UINT64: case TFG_FLOAT64: case TFG_DECIMAL64: return 8;
    case TFG_DECIMAL128: return 16;
    case TFG_DECIMAL256: return 32;
    default: return 0;
    }
}

Num host_num(int type, const void *p) {
    Num r{0, 0, 0, 0.0};
    switch (type) {
    case TFG_INT8: r.s = *(const int8_t *)p; break;
    case TFG_INT16: r.s = *(const int16_t *)p; break;
    case TFG_INT32: case TFG_DECIMAL32: r.s = *(const int32_t *)p; break;
    case TFG_INT64: case TFG_DECIMAL64: r.s = *(const int64_t *)p; break;
    case TFG_UINT8: r.cls = 1; r.u = *(const uint8_t *)p; break;
    case TFG_UINT16: r.cls = 1; r.u = *(const uint16_t *)p; break;
    case TFG_UINT32: r.cls = 1; r.u = *(const uint32_t *)p; break;
    case TFG_UINT64: r.cls = 1; r.u = *(const uint64_t *)p; break;
    case TFG_FLOAT32: r.cls = 2; r.d = *(const float *)p; break;
    case TFG_FLOAT64: r.cls = 2; r.d = *(const double *)p; break;
    default: break;
    }
    return r;
}

int scratch_get(Ctx *ctx, size_t bytes, void **out) {
    if (bytes == 0) bytes = 256;
    if (bytes > ctx->scratch_bytes) {
        if (ctx->scratch) {
            TFG_HIP(hipStreamSynchronize(ctx->stream));
            TFG_HIP(hipFree(ctx->scratch));
            ctx->scratch = nullptr;
            ctx->scratch_bytes = 0;
        }
        size_t sz = bytes + bytes / 4 + (1 << 20);
        TFG_HIP(hipMalloc(&ctx->scratch, sz));
        ctx->scratch_bytes = sz;
    }
    *out = ctx->scratch;
    return TFG_OK;
}

void arena_hold(Ctx *ctx) { ++ctx->arena.holds; }

void arena_free_all(Ctx *ctx) {
    for (auto &c : ctx->arena.chunks) (void)hipFree(c.p);
    ctx->arena = DevArena{};
}

void arena_drop(Ctx *ctx) {
    DevArena &A = ctx->arena;
    if (--A.holds > 0) return;
    A.holds = 0;
    A.cur = A.off = 0;
    if (A.chunks.size() > 1) { // outgrown during the call: one chunk of the high-water size
        size_t total = 0;
        for (auto &c : A.chunks) total += c.cap;
        (void)hipStreamSynchronize(ctx->stream);
        arena_free_all(ctx);
        void *p = nullptr;
        if (hipMalloc(&p, total) == hipSuccess) A.chunks.push_back({(char *)p, total});
    }
}

int arena_alloc(Ctx *ctx, size_t bytes, void **out) {
    DevArena &A = ctx->arena;
    TFG_CHECK(A.holds > 0, TFG_ERR_LOGICAL, "arena_alloc without a hold");
    bytes = (std::max<size_t>(bytes, 1) + 255) & ~size_t(255);
    while (A.cur < A.chunks.size()) {
        DevArena::Chunk &c = A.chunks[A.cur];
        if (A.off + bytes <= c.cap) {
            *out = c.p + A.off;
            A.off += bytes;
            return TFG_OK;
        }
        ++A.cur;
        A.off = 0;
    }
    size_t cap = std::max<size_t>(bytes, (size_t)4 << 20);
    for (auto &c : A.chunks) cap = std::max(cap, c.cap); // at least double the arena
    void *p = nullptr;
    TFG_HIP(hipMalloc(&p, cap));
    A.chunks.push_back({(char *)p, cap});
    A.cur = A.chunks.size() - 1;
    A.off = bytes;
    *out = p;
    return TFG_OK;
}

static hipEvent_t prof_take(Ctx *ctx) {
    if (!ctx->prof_pool.empty()) {
        hipEvent_t e = ctx->prof_pool.back();
        ctx->prof_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

ProfScope::ProfScope(Ctx *c, const char *name) : ctx(c) {
    if (!ctx->prof_on) return;
    ev.name = name;
    ev.start = prof_take(ctx);
    ev.stop = prof_take(ctx);
    if (ev.start) (void)hipEventRecord(ev.start, ctx->stream);
}

ProfScope::~ProfScope() {
    if (!ctx->prof_on || !ev.start || !ev.stop) return;
    (void)hipEventRecord(ev.stop, ctx->stream);
    ctx->prof_pending.push_back(ev);
}

int prof_resolve(Ctx *ctx) {
    if (ctx->prof_pending.empty()) return TFG_OK;
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    for (auto &e : ctx->prof_pending) {
        float ms = 0;
        TFG_HIP(hipEventElapsedTime(&ms, e.start, e.stop));
        ProfTotal *t = nullptr;
        for (auto &x : ctx->prof_totals)
            if (x.name == e.name) t = &x;
        if (!t) {
            ctx->prof_totals.push_back(ProfTotal{e.name, 0, 0});
            t = &ctx->prof_totals.back();
        }
        t->ms += ms;
        t->count++;
        ctx->prof_pool.push_back(e.start);
        ctx->prof_pool.push_back(e.stop);
    }
    ctx->prof_pending.clear();
    return TFG_OK;
}

int read_back_u64(Ctx *ctx, const uint64_t *dev, uint64_t *host, size_t count) {
    TFG_CHECK(count <= 64, TFG_ERR_LOGICAL, "read_back_u64: count %zu > 64", count);
    TFG_HIP(hipMemcpyAsync(ctx->host_pinned, dev, count * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    memcpy(host, ctx->host_pinned, count * sizeof(uint64_t));
    return TFG_OK;
}

// ------------------------------------------------------------------------------------------
// exclusive scan: 1024 threads x 8 items per block (8192 entries), block sums scanned by one
// block (<= 8192 blocks), then a fix-up pass.
constexpr int SCAN_T = 1024, SCAN_I = 8, SCAN_TILE = SCAN_T * SCAN_I;

template <typename T> __device__ __forceinline__ uint64_t block_scan_excl(uint64_t v, uint64_t *lds, uint64_t *total) {
    // wave inclusive scan via shuffles, then wave totals in LDS
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d, 64);
        if (lane >= (unsigned)d) x += y;
    }
    if (lane == 63) lds[wave] = x;
    __syncthreads();
    if (wave == 0) {
        const int nw = blockDim.x >> 6;
        uint64_t w = lane < (unsigned)nw ? lds[lane] : 0;
        uint64_t s = w;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint64_t y = __shfl_up(s, d, 64);
            if (lane >= (unsigned)d) s += y;
        }
        if (lane < (unsigned)nw) lds[32 + lane] = s - w; // exclusive wave offsets
        if (lane == (unsigned)nw - 1) lds[31] = s;
    }
    __syncthreads();
    uint64_t r = x - v + lds[32 + wave];
    if (total) *total = lds[31];
    __syncthreads();
    return r;
}

template <typename TIn>
__global__ void __launch_bounds__(SCAN_T) scan_reduce_kernel(const TIn *in, int64_t n, uint64_t *block_sums) {
    __shared__ uint64_t lds[64];
    int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_I; ++i) {
        int64_t idx = base + (int64_t)i * SCAN_T + threadIdx.x;
        if (idx < n) s += (uint64_t)in[idx];
    }
    uint64_t tot;
    block_scan_excl<uint64_t>(s, lds, &tot);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(SCAN_T) scan_block_sums_kernel(uint64_t *block_sums, int64_t nb, uint64_t *total_out) {
    __shared__ uint64_t lds[64];
    // nb <= SCAN_TILE; each thread owns SCAN_I consecutive entries
    uint64_t v[SCAN_I];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_I; ++i) {
        int64_t idx = (int64_t)threadIdx.x * SCAN_I + i;
        v[i] = idx < nb ? block_sums[idx] : 0;
        s += v[i];
    }
    uint64_t tot;
    uint64_t off = block_scan_excl<uint64_t>(s, lds, &tot);
#pragma unroll
    for (int i = 0; i < SCAN_I; ++i) {
        int64_t idx = (int64_t)threadIdx.x * SCAN_I + i;
        if (idx < nb) block_sums[idx] = off;
        off += v[i];
    }
    if (threadIdx.x == 0 && total_out) *total_out = tot;
}

template <typename TIn>
__global__ void __launch_bounds__(SCAN_T) scan_apply_kernel(const TIn *in, uint64_t *out, int64_t n, const uint64_t *block_offsets) {
    __shared__ uint64_t lds[64];
    int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    uint64_t v[SCAN_I];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_I; ++i) {
        int64_t idx = base + i;
        v[i] = idx < n ? (uint64_t)in[idx] : 0;
        s += v[i];
    }
    uint64_t off = block_scan_excl<uint64_t>(s, lds, nullptr) + block_offsets[blockIdx.x];
#pragma unroll
    for (int i = 0; i < SCAN_I; ++i) {
        int64_t idx = base + i;
        if (idx < n) out[idx] = off;
        off += v[i];
    }
}

// n <= SCAN_T * SMALL_I: one workgroup scans everything (one launch instead of three)
constexpr int SMALL_I = 16;
template <typename TIn>
__global__ void __launch_bounds__(SCAN_T) scan_small_kernel(const TIn *in, uint64_t *out, int64_t n) {
    __shared__ uint64_t lds[64];
    const int64_t base = (int64_t)threadIdx.x * SMALL_I;
    uint64_t v[SMALL_I];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < SMALL_I; ++i) {
        v[i] = base + i < n ? (uint64_t)in[base + i] : 0;
        s += v[i];
    }
    uint64_t tot;
    uint64_t off = block_scan_excl<uint64_t>(s, lds, &tot);
#pragma unroll
    for (int i = 0; i < SMALL_I; ++i) {
        if (base + i < n) out[base + i] = off;
        off += v[i];
    }
    if (threadIdx.x == 0) out[n] = tot;
}

size_t scan_tmp_bytes(int64_t n) {
    int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    return (size_t)(nb + 1) * sizeof(uint64_t) + 256;
}

template <typename TIn> static int scan_impl(Ctx *ctx, const TIn *in, uint64_t *out, int64_t n, void *tmp) {
    TFG_CHECK(n >= 0 && n <= (int64_t)SCAN_TILE * SCAN_TILE, TFG_ERR_INVALID_ARG, "scan size %lld out of range",
              (long long)n);
    int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (nb == 0) {
        TFG_HIP(hipMemsetAsync(out, 0, sizeof(uint64_t), ctx->stream));
        return TFG_OK;
    }
    if (n <= (int64_t)SCAN_T * SMALL_I) {
        ProfScope _ps(ctx, "scan");
        hipLaunchKernelGGL(scan_small_kernel<TIn>, dim3(1), dim3(SCAN_T), 0, ctx->stream, in, out, n);
        TFG_LAUNCH_CHECK();
        return TFG_OK;
    }
    uint64_t *bs = (uint64_t *)tmp;
    // NB: the reduce pass reads the same elements as the apply pass; with the scan operating
    // on the block sum layout (blocked vs striped) the sum per block is identical.
    { ProfScope _ps(ctx, "scan");
    hipLaunchKernelGGL(scan_reduce_kernel<TIn>, dim3((unsigned)nb), dim3(SCAN_T), 0, ctx->stream, in, n, bs);
    hipLaunchKernelGGL(scan_block_sums_kernel, dim3(1), dim3(SCAN_T), 0, ctx->stream, bs, nb, out + n);
    hipLaunchKernelGGL(scan_apply_kernel<TIn>, dim3((unsigned)nb), dim3(SCAN_T), 0, ctx->stream, in, out, n, bs);
    }
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int exclusive_scan_u32(Ctx *ctx, const uint32_t *in, uint64_t *out, int64_t n, void *tmp) {
    return scan_impl<uint32_t>(ctx, in, out, n, tmp);
}
int exclusive_scan_u64(Ctx *ctx, const uint64_t *in, uint64_t *out, int64_t n, void *tmp) {
    return scan_impl<uint64_t>(ctx, in, out, n, tmp);
}

} // namespace tfg

using namespace tfg;

extern "C" {

const char *tfg_last_error(void) { return g_last_error.c_str(); }
extern "C" const char tfg_build_stamp[]; // build/stamp.cpp, written by the Makefile
const char *tfg_version(void) {
    static char v[512];
    if (!v[0]) snprintf(v, sizeof v, "tiflash_amd 0.2 (%s)", tfg_build_stamp);
    return v;
}
size_t tfg_type_width(int type) { return type_width(type); }

int tfg_device_count(int *out) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *out = 0;
        return fail(TFG_ERR_NO_DEVICE, "hipGetDeviceCount failed: %s", hipGetErrorString(e));
    }
    *out = n;
    return TFG_OK;
}

int tfg_ctx_create(int device, void *stream, tfg_ctx **out) {
    TFG_CHECK(out, TFG_ERR_INVALID_ARG, "out is null");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(TFG_ERR_NO_DEVICE, "no HIP device visible");
    TFG_CHECK(device >= 0 && device < n, TFG_ERR_INVALID_ARG, "device %d out of range (%d devices)", device, n);
    TFG_HIP(hipSetDevice(device));
    tfg_ctx *c = new tfg_ctx();
    c->device = device;
    c->stream = (hipStream_t)stream;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->cu_count = prop.multiProcessorCount;
    if (hipMalloc(&c->dev_counter, 64 * sizeof(uint64_t)) != hipSuccess ||
        hipHostMalloc(&c->host_pinned, 64 * sizeof(uint64_t), 0) != hipSuccess) {
        delete c;
        return fail(TFG_ERR_OOM, "context allocation failed");
    }
    *out = c;
    return TFG_OK;
}

int tfg_ctx_destroy(tfg_ctx *ctx) {
    if (!ctx) return TFG_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    else (void)hipDeviceSynchronize();
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    arena_free_all(ctx);
    for (auto &e : ctx->prof_pending) {
        (void)hipEventDestroy(e.start);
        (void)hipEventDestroy(e.stop);
    }
    for (auto e : ctx->prof_pool) (void)hipEventDestroy(e);
    if (ctx->dev_counter) (void)hipFree(ctx->dev_counter);
    if (ctx->host_pinned) (void)hipHostFree(ctx->host_pinned);
    delete ctx;
    return TFG_OK;
}

int tfg_ctx_set_stream(tfg_ctx *ctx, void *stream) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    // the scratch and the call arena are reused in stream order: the old stream's last readers
    // finish before the new stream's first writers start
    if ((hipStream_t)stream != ctx->stream) TFG_HIP(hipStreamSynchronize(ctx->stream));
    ctx->stream = (hipStream_t)stream;
    return TFG_OK;
}

int tfg_ctx_sync(tfg_ctx *ctx) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    return TFG_OK;
}

int tfg_ctx_reserve(tfg_ctx *ctx, size_t bytes) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    void *p;
    return scratch_get(ctx, bytes, &p);
}

int tfg_profile_enable(tfg_ctx *ctx, int on) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    if (int rc = prof_resolve(ctx)) return rc;
    ctx->prof_on = on != 0;
    return TFG_OK;
}

int tfg_profile_reset(tfg_ctx *ctx) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    if (int rc = prof_resolve(ctx)) return rc;
    ctx->prof_totals.clear();
    return TFG_OK;
}

int tfg_profile_read(tfg_ctx *ctx, int index, char *name, size_t name_len, double *total_ms, uint64_t *count) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    if (int rc = prof_resolve(ctx)) return rc;
    if (index < 0 || index >= (int)ctx->prof_totals.size()) return TFG_ERR_INVALID_ARG;
    const ProfTotal &t = ctx->prof_totals[index];
    if (name && name_len) {
        strncpy(name, t.name.c_str(), name_len - 1);
        name[name_len - 1] = 0;
    }
    if (total_ms) *total_ms = t.ms;
    if (count) *count = t.count;
    return TFG_OK;
}

int tfg_buf_alloc(tfg_ctx *ctx, size_t bytes, void **out_dev) {
    TFG_CHECK(ctx && out_dev, TFG_ERR_INVALID_ARG, "null argument");
    if (set_device(ctx)) return TFG_ERR_HIP;
    TFG_HIP(hipMalloc(out_dev, bytes ? bytes : 1));
    return TFG_OK;
}

int tfg_buf_free(tfg_ctx *ctx, void *dev) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    if (!dev) return TFG_OK;
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    TFG_HIP(hipFree(dev));
    return TFG_OK;
}

int tfg_upload(tfg_ctx *ctx, void *dst_dev, const void *src_host, size_t bytes) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    if (!bytes) return TFG_OK;
    TFG_HIP(hipMemcpyAsync(dst_dev, src_host, bytes, hipMemcpyHostToDevice, ctx->stream));
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    return TFG_OK;
}

int tfg_copy(tfg_ctx *ctx, void *dst_dev, const void *src_dev, size_t bytes) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    if (!bytes) return TFG_OK;
    TFG_CHECK(dst_dev && src_dev, TFG_ERR_INVALID_ARG, "null buffer");
    TFG_HIP(hipMemcpyAsync(dst_dev, src_dev, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return TFG_OK;
}

int tfg_memset(tfg_ctx *ctx, void *dst_dev, int value, size_t bytes) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    if (!bytes) return TFG_OK;
    TFG_CHECK(dst_dev, TFG_ERR_INVALID_ARG, "null buffer");
    TFG_HIP(hipMemsetAsync(dst_dev, value, bytes, ctx->stream));
    return TFG_OK;
}

int tfg_download(tfg_ctx *ctx, void *dst_host, const void *src_dev, size_t bytes) {
    TFG_CHECK(ctx, TFG_ERR_INVALID_ARG, "ctx is null");
    if (!bytes) return TFG_OK;
    TFG_HIP(hipMemcpyAsync(dst_host, src_dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    return TFG_OK;
}

} // extern "C"
