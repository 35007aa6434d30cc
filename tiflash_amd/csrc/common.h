// common.h — shared device/host utilities of the gfx950 execution layer.
//
// Wave64 helpers, the software CRC32-C (the reference hashes with the SSE4.2 crc32q instruction,
// dbms/src/Common/HashTable/Hash.h:70-95; the GPU has none, so we use slicing-by-8 tables staged
// in LDS), exact mixed-type comparison (dbms/src/Core/AccurateComparison.h:33-159), the context
// with its scratch arena, and error plumbing for the C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tiflash_amd.h"

namespace tfg {

// ------------------------------------------------------------------------------------------
// errors (thread-local message behind tfg_last_error)
void set_error(const char *fmt, ...);
int fail(int code, const char *fmt, ...);
int hip_fail(hipError_t e, const char *what);
bool failpoint(const char *name); // TFG_FAILPOINT=<name> injects TFG_ERR_FAULT_INJECTED

#define TFG_HIP(expr)                                      \
    do {                                                   \
        hipError_t _e = (expr);                            \
        if (_e != hipSuccess) return ::tfg::hip_fail(_e, #expr); \
    } while (0)
#define TFG_CHECK(cond, code, ...)                         \
    do {                                                   \
        if (!(cond)) return ::tfg::fail((code), __VA_ARGS__); \
    } while (0)
// TFG_SYNC_CHECK=1 in the environment: every checked launch also waits for the device, so a kernel
// fault is reported at the launch site that follows it (file:line) instead of at a later sync
bool sync_check();
#define TFG_STR2(x) #x
#define TFG_STR(x) TFG_STR2(x)
#define TFG_LAUNCH_CHECK()                                                                          \
    do {                                                                                            \
        TFG_HIP(hipGetLastError());                                                                 \
        if (::tfg::sync_check()) {                                                                  \
            hipError_t _s = hipDeviceSynchronize();                                                 \
            if (_s != hipSuccess) return ::tfg::hip_fail(_s, "a kernel launched before " __FILE__ ":" TFG_STR(__LINE__)); \
        }                                                                                           \
    } while (0)

// ------------------------------------------------------------------------------------------
// context + scratch arena
struct ProfEvent {
    const char *name;
    hipEvent_t start, stop;
};
struct ProfTotal {
    std::string name;
    double ms = 0;
    uint64_t count = 0;
};

// Device buffers that live for one call but whose sizes are known only inside it (collated sort
// keys, their scans): carved from chunks the context keeps, so steady-state calls never allocate.
// Every buffer of a call holds the arena (ArenaHold); when the last hold is dropped the arena is
// empty again — its chunks are reused by the next call, whose kernels run after this call's on the
// same stream.  The first call that outgrows the chunks adds one; at the next reset the chunks
// are merged into one (a sync + free then, never in steady state).
struct DevArena {
    struct Chunk {
        char *p;
        size_t cap;
    };
    std::vector<Chunk> chunks;
    size_t cur = 0, off = 0; // bump position: chunk `cur`, byte `off`
    int holds = 0;
};

struct Ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    DevArena arena;
    uint64_t *dev_counter = nullptr; // small device scratch for counts (64 x u64)
    uint64_t *host_pinned = nullptr; // pinned host words for count read-back
    int cu_count = 256;
    // kernel profiler: HIP events recorded on `stream` around each launch (tfg_profile_*)
    bool prof_on = false;
    std::vector<ProfEvent> prof_pending;
    std::vector<hipEvent_t> prof_pool;
    std::vector<ProfTotal> prof_totals;
};

// RAII: brackets the kernel launches of one named phase with events on the context stream.
struct ProfScope {
    Ctx *ctx;
    ProfEvent ev{};
    ProfScope(Ctx *c, const char *name);
    ~ProfScope();
};
int prof_resolve(Ctx *ctx);

// Returns a device pointer to at least `bytes` of scratch (grows the arena; growth syncs the
// stream).  The region is reused by the next call: callers carve it, never keep it.
int scratch_get(Ctx *ctx, size_t bytes, void **out);

// The call arena (DevArena): arena_alloc needs a hold; arena_hold / arena_drop count the holds.
int arena_alloc(Ctx *ctx, size_t bytes, void **out);
void arena_hold(Ctx *ctx);
void arena_drop(Ctx *ctx);
void arena_free_all(Ctx *ctx); // context teardown (the stream synchronized)
struct ArenaScope {
    Ctx *c;
    explicit ArenaScope(Ctx *ctx) : c(ctx) { arena_hold(c); }
    ~ArenaScope() { arena_drop(c); }
    ArenaScope(const ArenaScope &) = delete;
    ArenaScope &operator=(const ArenaScope &) = delete;
};

struct Carver {
    size_t off = 0;
    template <typename T> size_t take(size_t count) {
        size_t o = off;
        off += (count * sizeof(T) + 255) & ~size_t(255);
        return o;
    }
};

inline int set_device(Ctx *ctx) {
    TFG_HIP(hipSetDevice(ctx->device));
    return TFG_OK;
}

// Reads `count` device u64 words into host memory (syncs the stream).
int read_back_u64(Ctx *ctx, const uint64_t *dev, uint64_t *host, size_t count);

size_t type_width(int t);
inline bool is_float_type(int t) { return t == TFG_FLOAT32 || t == TFG_FLOAT64; }
inline bool is_unsigned_type(int t) {
    return t == TFG_UINT8 || t == TFG_UINT16 || t == TFG_UINT32 || t == TFG_UINT64;
}
inline bool is_decimal_type(int t) { return t == TFG_DECIMAL32 || t == TFG_DECIMAL64 || t == TFG_DECIMAL128; }
inline bool is_fixed_numeric(int t) { return t >= TFG_INT8 && t <= TFG_FLOAT64; }

// Grid size for streaming kernels: enough workgroups to fill 256 CUs several times over.
inline unsigned stream_grid(int64_t items, int items_per_block, unsigned cap = 4096) {
    int64_t g = (items + items_per_block - 1) / items_per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// ------------------------------------------------------------------------------------------
// wave64 helpers
__device__ __forceinline__ unsigned lane_id() { return __lane_id(); }
__device__ __forceinline__ unsigned mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// ------------------------------------------------------------------------------------------
// CRC32-C (reflected 0x82F63B78), slicing-by-8.  crc32c_u64(crc, x) == _mm_crc32_u64(crc, x).
struct CrcTables {
    uint32_t t[8][256];
};
constexpr CrcTables make_crc_tables() {
    CrcTables r{};
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int b = 0; b < 8; ++b) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
        r.t[0][i] = c;
    }
    for (int k = 1; k < 8; ++k)
        for (uint32_t i = 0; i < 256; ++i) r.t[k][i] = (r.t[k - 1][i] >> 8) ^ r.t[0][r.t[k - 1][i] & 0xFF];
    return r;
}
static __constant__ CrcTables g_crc = make_crc_tables(); // per-TU copy (no -fgpu-rdc)

// Stage the 8 KB tables in LDS (call with all threads, then __syncthreads()).
__device__ __forceinline__ void load_crc_lds(uint32_t (*lds)[256]) {
    const uint32_t *src = &g_crc.t[0][0];
    uint32_t *dst = &lds[0][0];
    for (int i = threadIdx.x; i < 8 * 256; i += blockDim.x) dst[i] = src[i];
}

__device__ __forceinline__ uint32_t crc32c_u64(const uint32_t (*t)[256], uint32_t crc, uint64_t x) {
    uint32_t lo = (uint32_t)x ^ crc;
    uint32_t hi = (uint32_t)(x >> 32);
    return t[7][lo & 0xFF] ^ t[6][(lo >> 8) & 0xFF] ^ t[5][(lo >> 16) & 0xFF] ^ t[4][lo >> 24] ^
           t[3][hi & 0xFF] ^ t[2][(hi >> 8) & 0xFF] ^ t[1][(hi >> 16) & 0xFF] ^ t[0][hi >> 24];
}

// intHashCRC32(x) with the reference's seed (Hash.h:70-80).
__device__ __forceinline__ uint32_t int_hash_crc32(const uint32_t (*t)[256], uint64_t x) {
    return crc32c_u64(t, 0xFFFFFFFFu, x);
}

// ------------------------------------------------------------------------------------------
// exact number comparison (accurate:: semantics)
struct Num {
    int cls; // 0 signed, 1 unsigned, 2 float
    int64_t s;
    uint64_t u;
    double d;
};
Num host_num(int type, const void *p); // host: load one value

template <typename T> struct NumCls {
    static constexpr int value = std::is_floating_point<T>::value ? 2 : (std::is_unsigned<T>::value ? 1 : 0);
};

__device__ __forceinline__ int cmp_s_d(int64_t a, double d) {
    if (d >= 9223372036854775808.0) return -1;
    if (d < -9223372036854775808.0) return 1;
    int64_t t = (int64_t)d;
    if (a < t) return -1;
    if (a > t) return 1;
    double frac = d - (double)t;
    return frac > 0 ? -1 : (frac < 0 ? 1 : 0);
}
__device__ __forceinline__ int cmp_u_d(uint64_t a, double d) {
    if (d >= 18446744073709551616.0) return -1;
    if (d < 0) return 1;
    uint64_t t = (uint64_t)d;
    if (a < t) return -1;
    if (a > t) return 1;
    double frac = d - (double)t;
    return frac > 0 ? -1 : 0;
}
// returns -1/0/1, or 2 when unordered (NaN)
template <int CA, int CB>
__device__ __forceinline__ int cmp_cls(int64_t as, uint64_t au, double ad, int64_t bs, uint64_t bu, double bd) {
    if constexpr (CA == 2 && CB == 2) {
        if (ad != ad || bd != bd) return 2;
        return ad < bd ? -1 : (ad > bd ? 1 : 0);
    } else if constexpr (CA == 0 && CB == 0) {
        return as < bs ? -1 : (as > bs ? 1 : 0);
    } else if constexpr (CA == 1 && CB == 1) {
        return au < bu ? -1 : (au > bu ? 1 : 0);
    } else if constexpr (CA == 0 && CB == 1) {
        return as < 0 ? -1 : ((uint64_t)as < bu ? -1 : ((uint64_t)as > bu ? 1 : 0));
    } else if constexpr (CA == 1 && CB == 0) {
        return bs < 0 ? 1 : (au < (uint64_t)bs ? -1 : (au > (uint64_t)bs ? 1 : 0));
    } else if constexpr (CA == 0 && CB == 2) {
        if (bd != bd) return 2;
        return cmp_s_d(as, bd);
    } else if constexpr (CA == 1 && CB == 2) {
        if (bd != bd) return 2;
        return cmp_u_d(au, bd);
    } else if constexpr (CA == 2 && CB == 0) {
        if (ad != ad) return 2;
        return -cmp_s_d(bs, ad);
    } else {
        if (ad != ad) return 2;
        return -cmp_u_d(bu, ad);
    }
}

__device__ __forceinline__ uint8_t apply_cmp(int op, int c) {
    if (c == 2) return op == TFG_NE;
    switch (op) {
    case TFG_EQ: return c == 0;
    case TFG_NE: return c != 0;
    case TFG_LT: return c < 0;
    case TFG_LE: return c <= 0;
    case TFG_GT: return c > 0;
    default: return c >= 0;
    }
}

// Compare a column value of native type A with a constant Num of runtime class.
template <typename A> __device__ __forceinline__ uint8_t cmp_value_num(A a, const Num &b, int op) {
    constexpr int CA = NumCls<A>::value;
    int64_t as = 0;
    uint64_t au = 0;
    double ad = 0;
    if constexpr (CA == 0) as = (int64_t)a;
    else if constexpr (CA == 1) au = (uint64_t)a;
    else ad = (double)a;
    int c;
    if (b.cls == 0) c = cmp_cls<CA, 0>(as, au, ad, b.s, b.u, b.d);
    else if (b.cls == 1) c = cmp_cls<CA, 1>(as, au, ad, b.s, b.u, b.d);
    else c = cmp_cls<CA, 2>(as, au, ad, b.s, b.u, b.d);
    return apply_cmp(op, c);
}

template <typename A, typename B> __device__ __forceinline__ uint8_t cmp_values(A a, B b, int op) {
    constexpr int CA = NumCls<A>::value, CB = NumCls<B>::value;
    int64_t as = 0, bs = 0;
    uint64_t au = 0, bu = 0;
    double ad = 0, bd = 0;
    if constexpr (CA == 0) as = (int64_t)a;
    else if constexpr (CA == 1) au = (uint64_t)a;
    else ad = (double)a;
    if constexpr (CB == 0) bs = (int64_t)b;
    else if constexpr (CB == 1) bu = (uint64_t)b;
    else bd = (double)b;
    return apply_cmp(op, cmp_cls<CA, CB>(as, au, ad, bs, bu, bd));
}

// Host-side type dispatch over the 10 fixed numeric types.
#define TFG_DISPATCH_NUMERIC(TYPE, T, ...)                 \
    switch (TYPE) {                                        \
    case TFG_INT8: { using T = int8_t; __VA_ARGS__; break; }     \
    case TFG_INT16: { using T = int16_t; __VA_ARGS__; break; }   \
    case TFG_INT32: { using T = int32_t; __VA_ARGS__; break; }   \
    case TFG_INT64: { using T = int64_t; __VA_ARGS__; break; }   \
    case TFG_UINT8: { using T = uint8_t; __VA_ARGS__; break; }   \
    case TFG_UINT16: { using T = uint16_t; __VA_ARGS__; break; } \
    case TFG_UINT32: { using T = uint32_t; __VA_ARGS__; break; } \
    case TFG_UINT64: { using T = uint64_t; __VA_ARGS__; break; } \
    case TFG_FLOAT32: { using T = float; __VA_ARGS__; break; }   \
    case TFG_FLOAT64: { using T = double; __VA_ARGS__; break; }  \
    default: return ::tfg::fail(TFG_ERR_ILLEGAL_TYPE, "unsupported column type %d", (int)(TYPE)); \
    }

// Device-wide exclusive scan of u32 counts into u64 offsets; out[n] = total (out holds n+1).
// `tmp` must hold scan_tmp_bytes(n) bytes of device memory.  n <= 2^26.
int exclusive_scan_u32(Ctx *ctx, const uint32_t *in, uint64_t *out, int64_t n, void *tmp);
int exclusive_scan_u64(Ctx *ctx, const uint64_t *in, uint64_t *out, int64_t n, void *tmp);
size_t scan_tmp_bytes(int64_t n);

} // namespace tfg

struct tfg_ctx : public tfg::Ctx {};
