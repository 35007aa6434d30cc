// join.hip — hash join build + probe (a18-a21) for gfx950.
//
// Reference: Join::insertFromBlock -> JoinPartition::insertBlockIntoMaps -> insertBlockIntoMapsTypeCase
// (Interpreters/Join.cpp:532-735, JoinPartition.cpp:584-728; MapsAll = HashMap<UInt64, RowRefList,
// HashCRC32>, JoinHashMap.h:175-188) and Join::joinBlock -> probeBlockImplTypeCase + Adder<KIND, All>
// (Join.cpp:1153-1358, 1977; JoinPartition.cpp:1290-1378, 1465-1644).
//
// GPU design (radix-partitioned, LDS-bucketed open addressing):
//   finalize: the build keys are partitioned into P = 2^k partitions by the Fibonacci radix of
//             the key bits (fib_part; internal, so not the CRC), P sized so a partition fits the
//             LDS table;
//   probe:    probe keys are partitioned by the same function, then one workgroup per partition
//             loads the build partition into an LDS open-addressing table (u64 keys, 64-bit CAS,
//             per-key chains of build rows = RowRefList), streams the probe partition, and emits
//             (probe row, build row) pairs through an LDS output buffer flushed with one global
//             atomic per 2K pairs.  Build partitions larger than one LDS chunk (duplicate-heavy
//             keys) are processed chunk by chunk with a per-probe-row "found" flag, so LEFT / SEMI /
//             ANTI stay exact.  Rows with a NULL key never match (not inserted / not probed).
#include <algorithm>

#include "common.h"
#include "partition.h"

namespace tfg {

constexpr int JT = 512;
constexpr int JCAP = 4096;   // LDS table cells
constexpr int JCHUNK = 2048; // build rows per LDS pass
constexpr int JBUF = 2048;   // buffered output pairs

__device__ __forceinline__ uint64_t jmix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__device__ __forceinline__ uint64_t jload_bits(const void *p, int width, int64_t i) {
    switch (width) {
    case 1: return ((const uint8_t *)p)[i];
    case 2: return ((const uint16_t *)p)[i];
    case 4: return ((const uint32_t *)p)[i];
    default: return ((const uint64_t *)p)[i];
    }
}

struct SelJoin {
    const void *key;
    const uint8_t *key_null;
    int width;
    uint32_t shift;
    static constexpr bool needs_crc = false;
    __device__ __forceinline__ Loaded load(int64_t r) const {
        return Loaded{jload_bits(key, width, r), key_null ? (uint32_t)key_null[r] : 0u};
    }
    __device__ __forceinline__ uint32_t part(const uint32_t (*t)[256], const Loaded &l, int64_t) const {
        return l.null ? 0xFFFFFFFFu : fib_part(l.bits, shift); // NULL keys never join
    }
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const { return part(t, load(r), r); }
};

struct JoinArgs {
    const uint64_t *bkeys;   // build keys (u64 bits), partition-major
    const uint32_t *brows;   // build row ids
    const uint64_t *boff;    // P+1
    const void *pkeys;       // probe keys (raw width), partition-major
    const uint32_t *prows;   // probe row ids
    const uint64_t *poff;    // P+1
    int pwidth;
    int kind;
    uint8_t *found;          // per staged probe row (multi-chunk partitions), zeroed
    uint32_t *out_probe;
    uint32_t *out_build;
    uint64_t capacity;
    unsigned long long *cursor;
};

struct JLds {
    uint64_t keys[JCAP];
    uint32_t head[JCAP];
    uint32_t next[JCHUNK];
    uint32_t brow[JCHUNK];
    uint32_t buf_p[JBUF];
    uint32_t buf_b[JBUF];
    uint32_t red[JT / 64];
    unsigned buf_n;
    unsigned long long base;
};

__device__ __forceinline__ void emit_pair(const JoinArgs &A, uint64_t pos, uint32_t p, uint32_t b) {
    if (pos < A.capacity) {
        A.out_probe[pos] = p;
        if (A.out_build) A.out_build[pos] = b;
    }
}

__device__ void flush_buf(const JoinArgs &A, JLds &L) {
    // caller: all threads, after a barrier
    const unsigned n = L.buf_n;
    if (n == 0) return;
    if (threadIdx.x == 0) L.base = atomicAdd(A.cursor, (unsigned long long)n);
    __syncthreads();
    const uint64_t base = L.base;
    for (unsigned i = threadIdx.x; i < n; i += JT) emit_pair(A, base + i, L.buf_p[i], L.buf_b[i]);
    __syncthreads();
    if (threadIdx.x == 0) L.buf_n = 0;
    __syncthreads();
}

__device__ __forceinline__ uint32_t jblock_scan(uint32_t v, uint32_t *red, uint32_t &total) {
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (unsigned)d) x += y;
    }
    if (lane == 63) red[wave] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < JT / 64; ++w) {
        const uint32_t s = red[w];
        if (w < (int)wave) off += s;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return off + x - v;
}

__global__ void __launch_bounds__(JT) join_probe_kernel(JoinArgs A) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    JLds &L = *reinterpret_cast<JLds *>(lds_raw);
    const int b = blockIdx.x;
    const int64_t bs = (int64_t)A.boff[b], be = (int64_t)A.boff[b + 1];
    const int64_t ps = (int64_t)A.poff[b], pe = (int64_t)A.poff[b + 1];
    if (pe == ps) return; // no probe rows in this partition
    const int64_t nb = be - bs;
    const int chunks = nb == 0 ? 1 : (int)((nb + JCHUNK - 1) / JCHUNK);
    if (threadIdx.x == 0) L.buf_n = 0;
    for (int c = 0; c < chunks; ++c) {
        for (int i = threadIdx.x; i < JCAP; i += JT) {
            L.keys[i] = 0;
            L.head[i] = 0xFFFFFFFFu;
        }
        __syncthreads();
        // ---- build the LDS table from this chunk (key 0 lives in cell JCAP-1's twin: use a sentinel
        // remap — key 0 is stored as ~0 with an exact-compare guard below)
        const int64_t c0 = bs + (int64_t)c * JCHUNK;
        const int cn = (int)std::min<int64_t>(JCHUNK, be - c0);
        for (int j = threadIdx.x; j < cn; j += JT) {
            const uint64_t key = A.bkeys[c0 + j];
            L.brow[j] = A.brows[c0 + j];
            const uint64_t tag = key == 0 ? 0xFFFFFFFFFFFFFFFFull : key; // 0 is the empty marker
            unsigned pos = (unsigned)jmix(key) & (JCAP - 1);
            for (;;) {
                const uint64_t old = atomicCAS((unsigned long long *)&L.keys[pos], 0ull, (unsigned long long)tag);
                if (old == 0 || old == tag) break;
                pos = (pos + 1) & (JCAP - 1);
            }
            // keys ~0 (real) and 0 (remapped) share a tag: keep them apart by the exact key in bkeys
            L.next[j] = atomicExch(&L.head[pos], (uint32_t)j);
        }
        __syncthreads();
        const bool last = c == chunks - 1;
        // ---- stream the probe partition
        for (int64_t step = ps; step < pe; step += JT) {
            const int64_t r = step + threadIdx.x;
            const bool valid = r < pe;
            uint64_t key = 0;
            uint32_t prow = 0;
            unsigned head = 0xFFFFFFFFu;
            uint32_t cnt = 0;
            if (valid) {
                key = jload_bits(A.pkeys, A.pwidth, r);
                prow = A.prows[r];
                const uint64_t tag = key == 0 ? 0xFFFFFFFFFFFFFFFFull : key;
                unsigned pos = (unsigned)jmix(key) & (JCAP - 1);
                for (;;) {
                    const uint64_t k = L.keys[pos];
                    if (k == tag) {
                        head = L.head[pos];
                        break;
                    }
                    if (k == 0) break;
                    pos = (pos + 1) & (JCAP - 1);
                }
                for (unsigned j = head; j != 0xFFFFFFFFu; j = L.next[j]) cnt += (key + 1 > 1) || A.bkeys[c0 + j] == key; // exact check only for the shared tag of keys 0 and ~0
            }
            bool prev_found = false;
            if (valid && chunks > 1) {
                prev_found = A.found[r] != 0;
                if (cnt && !last) A.found[r] = 1;
            }
            uint32_t e = 0;
            if (valid) {
                switch (A.kind) {
                case TFG_JOIN_INNER: e = cnt; break;
                case TFG_JOIN_LEFT: e = cnt + ((last && cnt == 0 && !prev_found) ? 1 : 0); break;
                case TFG_JOIN_SEMI: e = (last && (cnt || prev_found)) ? 1 : 0; break;
                default: e = (last && !cnt && !prev_found) ? 1 : 0; break;
                }
            }
            uint32_t total;
            const uint32_t off = jblock_scan(e, L.red, total);
            if (total == 0) continue;
            if (L.buf_n + total > (unsigned)JBUF) flush_buf(A, L);
            if (total > (unsigned)JBUF) {
                // too many pairs for the buffer: reserve and write straight to HBM
                if (threadIdx.x == 0) L.base = atomicAdd(A.cursor, (unsigned long long)total);
                __syncthreads();
                uint64_t pos = L.base + off;
                if (A.kind == TFG_JOIN_INNER || A.kind == TFG_JOIN_LEFT) {
                    for (unsigned j = head; j != 0xFFFFFFFFu; j = L.next[j])
                        if ((key + 1 > 1) || A.bkeys[c0 + j] == key) emit_pair(A, pos++, prow, L.brow[j]);
                    if (e > cnt) emit_pair(A, pos, prow, 0xFFFFFFFFu);
                } else if (e) {
                    emit_pair(A, pos, prow, 0xFFFFFFFFu);
                }
                __syncthreads();
                continue;
            }
            unsigned pos = L.buf_n + off;
            if (A.kind == TFG_JOIN_INNER || A.kind == TFG_JOIN_LEFT) {
                for (unsigned j = head; j != 0xFFFFFFFFu && cnt; j = L.next[j])
                    if ((key + 1 > 1) || A.bkeys[c0 + j] == key) {
                        L.buf_p[pos] = prow;
                        L.buf_b[pos++] = L.brow[j];
                    }
                if (e > cnt) {
                    L.buf_p[pos] = prow;
                    L.buf_b[pos] = 0xFFFFFFFFu;
                }
            } else if (e) {
                L.buf_p[pos] = prow;
                L.buf_b[pos] = 0xFFFFFFFFu;
            }
            __syncthreads();
            if (threadIdx.x == 0) L.buf_n += total;
            __syncthreads();
        }
        __syncthreads();
    }
    flush_buf(A, L);
}

// LEFT / ANTI: probe rows with a NULL key are unmatched rows
__global__ void join_null_rows_kernel(const uint8_t *key_null, int64_t n, uint32_t *out_probe, uint32_t *out_build,
                                      uint64_t capacity, unsigned long long *cursor) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        if (!key_null[r]) continue;
        const uint64_t pos = atomicAdd(cursor, 1ull);
        if (pos < capacity) {
            out_probe[pos] = (uint32_t)r;
            if (out_build) out_build[pos] = 0xFFFFFFFFu;
        }
    }
}

__global__ void widen_keys_kernel(const void *in, int width, const uint8_t *key_null, int64_t n, uint64_t *out,
                                  uint8_t *out_null, int64_t row0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        out[row0 + i] = jload_bits(in, width, i);
        out_null[row0 + i] = key_null ? (key_null[i] != 0) : 0;
    }
}

} // namespace tfg

using namespace tfg;

struct tfg_join {
    Ctx *ctx = nullptr;
    int key_type = 0;
    int width = 8;
    // accumulated build keys (u64 bits) + null flags
    uint64_t *keys = nullptr;
    uint8_t *nulls = nullptr;
    int64_t n_rows = 0, cap_rows = 0;
    // finalized partitioned build
    bool finalized = false;
    uint32_t P = 1;
    uint64_t *bkeys = nullptr;
    uint32_t *brows = nullptr;
    uint64_t *boff = nullptr;
    int64_t n_inserted = 0;
};

namespace {

int join_grow(tfg_join *j, int64_t need) {
    if (need <= j->cap_rows) return TFG_OK;
    int64_t nc = std::max<int64_t>(need, j->cap_rows * 2);
    nc = std::max<int64_t>(nc, 1 << 16);
    uint64_t *k;
    uint8_t *z;
    TFG_HIP(hipMalloc(&k, nc * 8));
    TFG_HIP(hipMalloc(&z, nc));
    if (j->n_rows) {
        TFG_HIP(hipMemcpyAsync(k, j->keys, j->n_rows * 8, hipMemcpyDeviceToDevice, j->ctx->stream));
        TFG_HIP(hipMemcpyAsync(z, j->nulls, j->n_rows, hipMemcpyDeviceToDevice, j->ctx->stream));
    }
    TFG_HIP(hipStreamSynchronize(j->ctx->stream));
    if (j->keys) TFG_HIP(hipFree(j->keys));
    if (j->nulls) TFG_HIP(hipFree(j->nulls));
    j->keys = k;
    j->nulls = z;
    j->cap_rows = nc;
    return TFG_OK;
}

void free_build(tfg_join *j) {
    if (j->bkeys) (void)hipFree(j->bkeys);
    if (j->brows) (void)hipFree(j->brows);
    if (j->boff) (void)hipFree(j->boff);
    j->bkeys = nullptr;
    j->brows = nullptr;
    j->boff = nullptr;
}

} // namespace

extern "C" {

int tfg_join_create(tfg_ctx *ctx, int key_type, int64_t expected_build_rows, tfg_join **out) {
    TFG_CHECK(ctx && out, TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(type_width(key_type) > 0 && type_width(key_type) <= 8, TFG_ERR_ILLEGAL_TYPE,
              "unsupported join key type %d", key_type);
    if (int rc = set_device(ctx)) return rc;
    tfg_join *j = new tfg_join();
    j->ctx = ctx;
    j->key_type = key_type;
    j->width = (int)type_width(key_type);
    if (expected_build_rows > 0) {
        if (int rc = join_grow(j, expected_build_rows)) {
            delete j;
            return rc;
        }
    }
    *out = j;
    return TFG_OK;
}

int tfg_join_destroy(tfg_join *j) {
    if (!j) return TFG_OK;
    (void)hipSetDevice(j->ctx->device);
    (void)hipStreamSynchronize(j->ctx->stream);
    if (j->keys) (void)hipFree(j->keys);
    if (j->nulls) (void)hipFree(j->nulls);
    free_build(j);
    delete j;
    return TFG_OK;
}

int tfg_join_build(tfg_join *j, const void *keys, const uint8_t *key_nullmap, int64_t n) {
    TFG_CHECK(j && (n == 0 || keys), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(!j->finalized, TFG_ERR_LOGICAL, "build after finalize");
    TFG_CHECK(n >= 0 && j->n_rows + n < (int64_t)0xFFFFFFFFll, TFG_ERR_INVALID_ARG, "build row count out of range");
    if (failpoint("join_build")) return fail(TFG_ERR_FAULT_INJECTED, "failpoint join_build");
    if (n == 0) return TFG_OK;
    if (int rc = set_device(j->ctx)) return rc;
    if (int rc = join_grow(j, j->n_rows + n)) return rc;
    hipLaunchKernelGGL(widen_keys_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, j->ctx->stream, keys, j->width,
                       key_nullmap, n, j->keys, j->nulls, j->n_rows);
    TFG_LAUNCH_CHECK();
    j->n_rows += n;
    return TFG_OK;
}

int tfg_join_finalize(tfg_join *j) {
    TFG_CHECK(j, TFG_ERR_INVALID_ARG, "join is null");
    if (j->finalized) return TFG_OK;
    if (int rc = set_device(j->ctx)) return rc;
    Ctx *ctx = j->ctx;
    // partitions: keep the average build partition well under one LDS chunk
    int64_t want = j->n_rows / (JCHUNK * 5 / 8);
    uint32_t P = 1;
    while ((int64_t)P < want && P < (uint32_t)PMAX_UNSTABLE) P <<= 1;
    j->P = P;
    const int64_t n = j->n_rows;
    TFG_HIP(hipMalloc(&j->bkeys, std::max<int64_t>(n, 1) * 8));
    TFG_HIP(hipMalloc(&j->brows, std::max<int64_t>(n, 1) * 4));
    TFG_HIP(hipMalloc(&j->boff, (P + 1) * 8));
    PartLayout L = make_layout(n, P);
    void *tmp;
    if (int rc = scratch_get(ctx, part_tmp_bytes(L), &tmp)) return rc;
    PCols pc{};
    pc.ncols = 1;
    pc.in[0] = j->keys;
    pc.out[0] = j->bkeys;
    pc.width[0] = 8;
    pc.key0 = 1;
    SelJoin sel{j->keys, j->nulls, 8, fib_shift(P)};
    RowPred pred{};
    if (int rc = run_partition<SelJoin, false>(ctx, sel, pred, L, pc, j->brows, nullptr, j->boff, tmp, "join.build.hist",
                                               "join.build.scatter"))
        return rc;
    uint64_t ins = 0;
    if (int rc = read_back_u64(ctx, j->boff + P, &ins, 1)) return rc;
    j->n_inserted = (int64_t)ins;
    j->finalized = true;
    return TFG_OK;
}

int tfg_join_stats(tfg_join *j, uint64_t *rows, uint64_t *partitions) {
    TFG_CHECK(j, TFG_ERR_INVALID_ARG, "join is null");
    if (rows) *rows = (uint64_t)j->n_inserted;
    if (partitions) *partitions = j->P;
    return TFG_OK;
}

int tfg_join_probe(tfg_join *j, int kind, const void *keys, const uint8_t *key_nullmap, int64_t n,
                   uint32_t *out_probe_idx, uint32_t *out_build_idx, uint64_t capacity, uint64_t *out_count_dev,
                   uint64_t *out_count_host) {
    TFG_CHECK(j && (n == 0 || keys) && (capacity == 0 || out_probe_idx), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(kind >= TFG_JOIN_INNER && kind <= TFG_JOIN_ANTI, TFG_ERR_NOT_IMPLEMENTED, "join kind %d", kind);
    TFG_CHECK(n >= 0 && n < (int64_t)0xFFFFFFFFll, TFG_ERR_INVALID_ARG, "probe row count out of range");
    if (failpoint("join_probe")) return fail(TFG_ERR_FAULT_INJECTED, "failpoint join_probe");
    if (!j->finalized)
        if (int rc = tfg_join_finalize(j)) return rc;
    if (int rc = set_device(j->ctx)) return rc;
    Ctx *ctx = j->ctx;
    const uint32_t P = j->P;
    PartLayout L = make_layout(n, P);
    Carver cv;
    const size_t o_pk = cv.take<uint64_t>(n), o_pr = cv.take<uint32_t>(n), o_poff = cv.take<uint64_t>(P + 1);
    const size_t o_found = cv.take<uint8_t>(n), o_cur = cv.take<uint64_t>(1);
    const size_t o_tmp = cv.take<uint8_t>(part_tmp_bytes(L));
    void *sp;
    if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
    char *sb = (char *)sp;
    unsigned long long *cursor = (unsigned long long *)(sb + o_cur);
    TFG_HIP(hipMemsetAsync(cursor, 0, 8, ctx->stream));
    if (n > 0) {
        PCols pc{};
        pc.ncols = 1;
        pc.in[0] = keys;
        pc.out[0] = sb + o_pk;
        pc.width[0] = j->width;
        pc.key0 = j->width == 8;
        SelJoin sel{keys, key_nullmap, j->width, fib_shift(P)};
        RowPred pred{};
        uint64_t *poff = (uint64_t *)(sb + o_poff);
        if (int rc = run_partition<SelJoin, false>(ctx, sel, pred, L, pc, (uint32_t *)(sb + o_pr), nullptr, poff, sb + o_tmp,
                                                   "join.part.hist", "join.part.scatter"))
            return rc;
        TFG_HIP(hipMemsetAsync(sb + o_found, 0, n, ctx->stream));
        JoinArgs A{};
        A.bkeys = j->bkeys;
        A.brows = j->brows;
        A.boff = j->boff;
        A.pkeys = sb + o_pk;
        A.prows = (const uint32_t *)(sb + o_pr);
        A.poff = poff;
        A.pwidth = j->width;
        A.kind = kind;
        A.found = (uint8_t *)(sb + o_found);
        A.out_probe = out_probe_idx;
        A.out_build = out_build_idx;
        A.capacity = capacity;
        A.cursor = cursor;
        { ProfScope _ps(ctx, "join.probe");
        hipLaunchKernelGGL(join_probe_kernel, dim3(P), dim3(JT), sizeof(JLds), ctx->stream, A);
        }
        TFG_LAUNCH_CHECK();
        if (key_nullmap && (kind == TFG_JOIN_LEFT || kind == TFG_JOIN_ANTI)) {
            hipLaunchKernelGGL(join_null_rows_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, ctx->stream,
                               key_nullmap, n, out_probe_idx, out_build_idx, capacity, cursor);
            TFG_LAUNCH_CHECK();
        }
    }
    if (out_count_dev) TFG_HIP(hipMemcpyAsync(out_count_dev, cursor, 8, hipMemcpyDeviceToDevice, ctx->stream));
    uint64_t total = 0;
    if (int rc = read_back_u64(ctx, (const uint64_t *)cursor, &total, 1)) return rc;
    if (out_count_host) *out_count_host = total;
    if (total > capacity)
        return fail(TFG_ERR_CAPACITY, "join result needs %llu pairs, capacity %llu", (unsigned long long)total,
                    (unsigned long long)capacity);
    return TFG_OK;
}

} // extern "C"
