// join.hip — hash join build + probe (a18-a21) for gfx950.
//
// Reference: Join::insertFromBlock -> JoinPartition::insertBlockIntoMaps -> insertBlockIntoMapsTypeCase
// (Interpreters/Join.cpp:532-735, JoinPartition.cpp:584-728; MapsAll = HashMap<UInt64, RowRefList,
// HashCRC32>, JoinHashMap.h:175-188) and Join::joinBlock -> probeBlockImplTypeCase + Adder<KIND, All>
// (Join.cpp:1153-1358, 1977; JoinPartition.cpp:1290-1378, 1465-1644), replicateRange
// (Columns/ColumnVector.cpp:706-738).
//
// GPU design (radix-partitioned, LDS-bucketed open addressing, materialising):
//   finalize: build rows (key widened to u64, up to 2 payload words) are radix-partitioned by the
//             Fibonacci radix of the key into P <= 4096 partitions of ~2.5K rows with the
//             LDS-staged scatter, as interleaved records {key, payload...};
//   probe:    probe rows are partitioned the same way (records {key, payload...}); one workgroup
//             per partition loads the build partition into an LDS table (u64 keys, grouped
//             probing of 4 cells per 32-byte read, 64-bit CAS; per key a chain of build rows and
//             its length) and streams the probe records JT * JRPT at a time: a block scan of the
//             rows' output counts, one global atomic for the step's output range, and every
//             thread writes its rows at its scanned offset — probe payload words from the record
//             in registers, build payload words from the build record — so the joined block
//             needs no gathers.
//             The index-pair API (tfg_join_probe) is the same kernel with row ids as the payload.
//   Build partitions larger than one LDS chunk (duplicate-heavy keys) are processed chunk by
//   chunk with a per-probe-row found flag so LEFT / SEMI / ANTI stay exact.  Rows with a NULL key
//   never match (not inserted / not probed); LEFT and ANTI emit them as unmatched rows.
#include <algorithm>
#include <vector>

#include "collation.h"
#include "common.h"
#include "partition.h"

namespace tfg {

constexpr int JT = 512;      // probe workgroup (1024 measured slower: join.probe 0.954 vs 0.892 ms)
constexpr uint32_t JBIG = 65535u / JT; // per-row output count that still packs into a 16-bit field
constexpr int JCAP = 4096;   // LDS table cells (power of two)
constexpr int JGS = 4;       // cells per probe group (one 32-byte read)
constexpr int JCHUNK = 4096; // build rows per LDS pass (row index fits 16 bits)
constexpr int JRPT = 4;      // probe rows per thread per step
constexpr int JFILL = 2560;  // target build rows per partition (table load ~0.63)
constexpr int JMAXW = 2;     // payload words per side
// probe records and output rows stream past the partition's build records, which the probe's
// matches re-read at random: nontemporal loads / stores keep them from evicting those lines
#ifdef TFG_EXP_JOIN_TEMPORAL
constexpr bool JOIN_NT = false;
#else
constexpr bool JOIN_NT = true;
#endif
template <typename T> __device__ __forceinline__ void jstore(T *p, T v) {
    if constexpr (JOIN_NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__device__ __forceinline__ uint64_t jload_bits(const void *p, int width, int64_t i) {
    switch (width) {
    case 1: return ((const uint8_t *)p)[i];
    case 2: return ((const uint16_t *)p)[i];
    case 4: return ((const uint32_t *)p)[i];
    default: return ((const uint64_t *)p)[i];
    }
}

// partition of a key: the Fibonacci radix (internal; NULL keys are dropped)
struct SelJoin {
    const void *key;
    const uint8_t *key_null;
    int width;
    uint32_t shift;
    static constexpr bool needs_crc = false;
    static constexpr bool fib_radix = true;
    __device__ __forceinline__ Loaded load(int64_t r) const {
        return Loaded{jload_bits(key, width, r), key_null ? (uint32_t)key_null[r] : 0u};
    }
    __device__ __forceinline__ uint32_t part(const uint32_t (*t)[256], const Loaded &l, int64_t) const {
        return l.null ? 0xFFFFFFFFu : fib_part(l.bits, shift); // NULL keys never join
    }
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const { return part(t, load(r), r); }
};

// in-partition group of a key: the product bits below the partition radix
__device__ __forceinline__ unsigned join_group(uint64_t key, int slot_shift) {
    return (unsigned)((key * 0x9E3779B97F4A7C15ull) >> slot_shift) & (JCAP / JGS - 1);
}

struct JoinArgs {
    const uint64_t *brec;  // build records (key + bw words), partition-major
    const uint32_t *brows; // build row ids (partition-major)
    const uint64_t *boff;  // P+1
    int bw;                // build payload words in a record
    const uint64_t *prec;  // probe records (key + payload words), partition-major
    const uint32_t *prows; // probe row ids (null when pw > 0)
    const uint64_t *poff;  // P+1
    int pw;                // probe payload words output
    int prw;               // probe record words
    int pw0;               // record word of payload 0 (0 when payload 0 is the key column itself)
    int kind;
    int slot_shift;
    uint8_t *found; // per staged probe row (multi-chunk partitions), zeroed
    // outputs: out_p[w] (pw > 0: u64 payload words; pw == 0: u32 probe row ids in out_p[0]),
    // out_b[w] likewise for the build side; out_bnull: 1 for LEFT rows without a match
    void *out_p[JMAXW];
    void *out_b[JMAXW];
    uint8_t *out_bnull;
    uint64_t capacity;
    unsigned long long *cursor;
};

struct JLds {
    uint64_t keys[JCAP];
    uint32_t head[JCAP + 1]; // [JCAP] = chain of key 0 (ZeroValueStorage)
    uint32_t cnt[JCAP + 1];
    uint16_t next[JCHUNK];
    uint32_t red[JT / 64 + 2];
    uint64_t red64[JT / 64];
    uint32_t redbig[JT / 64];
    unsigned long long base;
};

static_assert(2 * sizeof(JLds) <= 160 * 1024, "two probe workgroups per CU");

__device__ __forceinline__ uint32_t jblock_scan(uint32_t v, uint32_t *red, uint32_t &total) {
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
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

// Block scan of the four 16-bit output counts of a thread's rows (fields u = 0..3 of v, each
// count <= JBIG so no field overflows over JT threads): off = the exclusive prefix of every
// field, total = the block totals; any_big = some thread flagged a row with > JBIG outputs.
__device__ __forceinline__ uint64_t jblock_scan4(uint64_t v, bool big, JLds &L, uint64_t &total, bool &any_big) {
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= (unsigned)d) x += y;
    }
    const bool wbig = __ballot(big) != 0;
    if (lane == 63) {
        L.red64[wave] = x;
        L.redbig[wave] = wbig;
    }
    __syncthreads();
    uint64_t off = 0, tot = 0;
    bool ab = false;
#pragma unroll
    for (int w = 0; w < JT / 64; ++w) {
        const uint64_t sw = L.red64[w];
        if (w < (int)wave) off += sw;
        tot += sw;
        ab |= L.redbig[w] != 0;
    }
    __syncthreads();
    total = tot;
    any_big = ab;
    return off + x - v;
}

__device__ __forceinline__ int jfind(const JLds &L, uint64_t key, int slot_shift) {
    if (key == 0) return JCAP;
    unsigned g = join_group(key, slot_shift);
    for (int step = 0; step < JCAP / JGS; ++step) {
        const uint4 a = *reinterpret_cast<const uint4 *>(&L.keys[g * JGS]);
        const uint4 c = *reinterpret_cast<const uint4 *>(&L.keys[g * JGS + 2]);
        const uint64_t k[JGS] = {((uint64_t)a.y << 32) | a.x, ((uint64_t)a.w << 32) | a.z, ((uint64_t)c.y << 32) | c.x,
                                 ((uint64_t)c.w << 32) | c.z};
#pragma unroll
        for (int s = 0; s < JGS; ++s) {
            if (k[s] == key) return (int)(g * JGS + s);
            if (k[s] == 0) return -1;
        }
        g = (g + 1) & (JCAP / JGS - 1);
    }
    return -1;
}

__device__ __forceinline__ int jinsert(JLds &L, uint64_t key, int slot_shift) {
    if (key == 0) return JCAP;
    unsigned g = join_group(key, slot_shift);
    for (;;) {
        for (int s = 0; s < JGS; ++s) {
            const int cell = (int)(g * JGS + s);
            const uint64_t cur = L.keys[cell];
            if (cur == key) return cell;
            if (cur != 0) continue;
            const uint64_t old = atomicCAS((unsigned long long *)&L.keys[cell], 0ull, (unsigned long long)key);
            if (old == 0 || old == key) return cell;
        }
        g = (g + 1) & (JCAP / JGS - 1);
    }
}

// PRW probe record words, BW build payload words: compile-time, so the pipelined registers
// (two steps' records + the first match's build payload) stay within 4 waves per SIMD
template <int PRW, int BW>
__global__ void __launch_bounds__(JT) join_probe_kernel(JoinArgs A) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    JLds &L = *reinterpret_cast<JLds *>(lds_raw);
    const int b = blockIdx.x;
    const int64_t bs = (int64_t)A.boff[b], be = (int64_t)A.boff[b + 1];
    const int64_t ps = (int64_t)A.poff[b], pe = (int64_t)A.poff[b + 1];
    if (pe == ps) return; // no probe rows in this partition
    const int64_t nb = be - bs;
    const int chunks = nb == 0 ? 1 : (int)((nb + JCHUNK - 1) / JCHUNK);
    constexpr int brw = 1 + BW;
    for (int c = 0; c < chunks; ++c) {
        for (int i = threadIdx.x; i < JCAP + 1; i += JT) {
            if (i < JCAP) L.keys[i] = 0;
            L.head[i] = 0xFFFFFFFFu;
            L.cnt[i] = 0;
        }
        __syncthreads();
        // ---- build the LDS table from this chunk: per key a chain (RowRefList) and its length
        const int64_t c0 = bs + (int64_t)c * JCHUNK;
        const int cn = (int)std::min<int64_t>(JCHUNK, be - c0);
        for (int jr = threadIdx.x; jr < cn; jr += JT) {
            const uint64_t key = A.brec[(c0 + jr) * brw];
            const int cell = jinsert(L, key, A.slot_shift);
            L.next[jr] = (uint16_t)atomicExch(&L.head[cell], (uint32_t)jr);
            atomicAdd(&L.cnt[cell], 1u);
        }
        __syncthreads();
        const bool last = c == chunks - 1;
        // ---- stream the probe partition, JRPT rows per thread per step (their record loads in
        // flight together; one block scan and one barrier pair per JT * JRPT rows)
        const bool pairs = A.kind <= TFG_JOIN_LEFT; // SEMI / ANTI emit the probe row alone
        const bool bpay = pairs && BW > 0 && A.out_b[0];
        constexpr int64_t STEP = (int64_t)JT * JRPT;
        // software pipelined: the next step's record loads are issued before this step's output
        // range is claimed, so their latency overlaps the global atomic and the stores
        auto load_step = [&](int64_t st, uint64_t (&dst)[JRPT][PRW]) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < JRPT; ++u) {
                const int64_t r = st + u * JT + threadIdx.x;
                if (r < pe) load_rec<PRW, JOIN_NT>(A.prec, (size_t)r, dst[u]);
            }
        };
        uint64_t rw[JRPT][PRW]; // the probe records (key + payload words)
        load_step(ps, rw);
        // the first step's records complete here, so no use of rw inside the loop (the output
        // stores) has to assume a load of the loop's entry may still be pending: those waits
        // drained the next step's prefetch with it (s_waitcnt vmcnt(0) at every store)
        __builtin_amdgcn_s_waitcnt(0);
        for (int64_t step = ps; step < pe; step += STEP) {
            unsigned head[JRPT];
            uint32_t cnt[JRPT], e[JRPT];
            uint64_t bp[JRPT][BW > 0 ? BW : 1]; // the first match's build payload words, loaded early
            uint32_t esum = 0;
#pragma unroll
            for (int u = 0; u < JRPT; ++u) {
                const int64_t r = step + u * JT + threadIdx.x;
                const bool valid = r < pe;
                head[u] = 0xFFFFFFFFu;
                cnt[u] = 0;
                e[u] = 0;
                if (!valid) continue;
                const int cell = jfind(L, rw[u][0], A.slot_shift);
                if (cell >= 0) {
                    head[u] = L.head[cell];
                    cnt[u] = L.cnt[cell];
                }
                if (bpay && cnt[u]) {
                    const uint64_t *rec = A.brec + (c0 + head[u]) * brw;
#pragma unroll
                    for (int w = 0; w < BW; ++w) bp[u][w] = rec[1 + w];
                }
                bool prev_found = false;
                if (chunks > 1) {
                    prev_found = A.found[r] != 0;
                    if (cnt[u] && !last) A.found[r] = 1;
                }
                switch (A.kind) {
                case TFG_JOIN_INNER: e[u] = cnt[u]; break;
                case TFG_JOIN_LEFT: e[u] = cnt[u] + ((last && cnt[u] == 0 && !prev_found) ? 1 : 0); break;
                case TFG_JOIN_SEMI: e[u] = (last && (cnt[u] || prev_found)) ? 1 : 0; break;
                default: e[u] = (last && !cnt[u] && !prev_found) ? 1 : 0; break;
                }
                esum += e[u];
            }
            // one output range per workgroup step (one global atomic).  Rows are placed u-major
            // (all threads' row u = 0, then u = 1, ...), so the lanes of a store instruction write
            // consecutive output rows; a step holding a row with > JBIG outputs (duplicate-heavy
            // keys) places them thread-major from a plain scan of the per-thread sums instead.
            static_assert(JRPT == 4, "four 16-bit count fields");
            uint64_t packed = 0;
            bool big = false;
#pragma unroll
            for (int u = 0; u < JRPT; ++u) {
                big |= e[u] > JBIG;
                packed |= (uint64_t)(e[u] > JBIG ? 0 : e[u]) << (16 * u);
            }
            uint64_t ptotal;
            bool any_big;
            const uint64_t poff = jblock_scan4(packed, big, L, ptotal, any_big);
            uint32_t total = 0, toff = 0;
            if (any_big) toff = jblock_scan(esum, L.red, total);
            else
#pragma unroll
                for (int u = 0; u < JRPT; ++u) total += (uint32_t)(ptotal >> (16 * u)) & 0xFFFFu;
            // the output range is claimed BEFORE the next step's loads are issued: the wait for the
            // atomic's result then leaves those loads in flight (vmcnt counts in issue order;
            // claimed after them, the wait drained the prefetch with it)
            unsigned long long claimed = 0;
            if (total && threadIdx.x == 0) claimed = atomicAdd(A.cursor, (unsigned long long)total);
            uint64_t nx[JRPT][PRW];
            if (step + STEP < pe) load_step(step + STEP, nx);
            if (total) {
                if (threadIdx.x == 0) L.base = claimed;
                __syncthreads();
                const uint64_t base = L.base;
                uint64_t pos = base + toff; // thread-major cursor (any_big)
                uint32_t ubase = 0;         // u-major: rows of the earlier u
#pragma unroll
                for (int u = 0; u < JRPT; ++u) {
                    const int64_t r = step + u * JT + threadIdx.x;
                    if (!any_big) pos = base + ubase + ((poff >> (16 * u)) & 0xFFFFu);
                    ubase += (uint32_t)(ptotal >> (16 * u)) & 0xFFFFu;
                    unsigned jb = head[u];
                    for (uint32_t q = 0; q < e[u]; ++q, ++pos) {
                        const bool pair = pairs && q < cnt[u];
                        if (pos < A.capacity) {
                            if (A.pw == 0) {
                                jstore((uint32_t *)A.out_p[0] + pos, A.prows[r]);
                            } else {
#pragma unroll
                                for (int w = 0; w < PRW; ++w)
                                    if (w < A.pw)
                                        jstore((uint64_t *)A.out_p[w] + pos, A.pw0 ? rw[u][w + 1 < PRW ? w + 1 : w] : rw[u][w]);
                            }
                            if (A.out_bnull) A.out_bnull[pos] = !pair;
                            if (A.out_b[0]) {
                                if constexpr (BW == 0) {
                                    jstore((uint32_t *)A.out_b[0] + pos, pair ? A.brows[c0 + jb] : 0xFFFFFFFFu);
                                } else if (pair && q == 0) {
#pragma unroll
                                    for (int w = 0; w < BW; ++w) jstore((uint64_t *)A.out_b[w] + pos, bp[u][w]);
                                } else {
                                    const uint64_t *rec = A.brec + (c0 + (pair ? jb : 0)) * brw;
#pragma unroll
                                    for (int w = 0; w < BW; ++w) jstore((uint64_t *)A.out_b[w] + pos, pair ? rec[1 + w] : (uint64_t)0);
                                }
                            }
                        }
                        if (pair) jb = L.next[jb];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < JRPT; ++u)
#pragma unroll
                for (int w = 0; w < PRW; ++w) rw[u][w] = nx[u][w];
        }
        __syncthreads();
    }
}

// LEFT / ANTI: probe rows with a NULL key are unmatched rows
__global__ void join_null_rows_kernel(const uint8_t *key_null, int64_t n, JoinArgs A, const void *const *ppay_in,
                                      int pw) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        if (!key_null[r]) continue;
        const uint64_t pos = atomicAdd(A.cursor, 1ull);
        if (pos >= A.capacity) continue;
        if (pw == 0) ((uint32_t *)A.out_p[0])[pos] = (uint32_t)r;
        for (int w = 0; w < pw; ++w) ((uint64_t *)A.out_p[w])[pos] = ((const uint64_t *)ppay_in[w])[r];
        if (A.out_bnull) A.out_bnull[pos] = 1;
        if (A.bw == 0) {
            if (A.out_b[0]) ((uint32_t *)A.out_b[0])[pos] = 0xFFFFFFFFu;
        } else if (A.out_b[0]) {
            for (int w = 0; w < A.bw; ++w) ((uint64_t *)A.out_b[w])[pos] = 0;
        }
    }
}

__global__ void widen_keys_kernel(const void *in, int width, const uint8_t *key_null, int64_t n, uint64_t *out,
                                  uint8_t *out_null, int64_t row0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        out[row0 + i] = jload_bits(in, width, i);
        if (out_null) out_null[row0 + i] = key_null ? (key_null[i] != 0) : 0;
    }
}

// other conditions (Join::handleOtherConditions, Interpreters/Join.cpp:798-1150): a probe row
// is matched when at least one of its key-equal pairs passes the condition
__global__ void join_mark_kernel(const uint32_t *probe_idx, const uint8_t *pass, int64_t n, uint8_t *flags) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (!pass || pass[i]) flags[probe_idx[i]] = 1; // benign race: every writer stores 1
}

// ---------------------------------------------------------------- JoinV2 pointer table (§8 f3)
// HashJoinPointerTable (Interpreters/JoinV2/HashJoinPointerTable.{h,cpp}): one table of 2^d
// heads, d from pointerTableCapacity(rows) = max(pow2ceil(2 * rows), 1024); bucket = the top d
// bits of the row's 64-bit hash; rows are pushed onto their bucket's chain by an exchange of the
// head (the row keeps the old head as its next link).  A tagged head carries in its top 16 bits
// the OR of (hash & 0xFFFF) of every row on the chain, so a probe whose 16 hash bits are not all
// present skips the chain without touching it.  Here a head is (tag << 48) | (row + 1) and the
// links are a row-indexed array; probing needs no partitioning pass.
constexpr int V2_TAG_SHIFT = 48;
constexpr uint64_t V2_ROW_MASK = (1ull << V2_TAG_SHIFT) - 1;

__device__ __forceinline__ uint64_t v2_hash(uint64_t k) { // splitmix64 finaliser
    k ^= k >> 30;
    k *= 0xBF58476D1CE4E5B9ull;
    k ^= k >> 27;
    k *= 0x94D049BB133111EBull;
    return k ^ (k >> 31);
}

// a chain link: the row's key and the next row (+ 1; 0 = end) in one 16-byte record, so every
// step of a chain walk is a single load
__global__ void join_v2_build_kernel(const uint64_t *keys, const uint8_t *nulls, int64_t n, uint64_t *heads,
                                     uint32_t shift, int tagged, uint4 *link) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = keys[r];
        if (nulls && nulls[r]) {
            link[r] = make_uint4((unsigned)key, (unsigned)(key >> 32), 0u, 0u);
            continue; // NULL keys never join (never on a chain)
        }
        const uint64_t h = v2_hash(key);
        uint64_t *slot = heads + (h >> shift);
        uint64_t old = atomicExch((unsigned long long *)slot, (unsigned long long)(r + 1));
        if (tagged) { // insertRowToList + tag: the chain's tag bits, ours included, on the head
            const uint64_t tag = (h & 0xFFFFull) | (old >> V2_TAG_SHIFT);
            atomicOr((unsigned long long *)slot, (unsigned long long)(tag << V2_TAG_SHIFT));
        }
        link[r] = make_uint4((unsigned)key, (unsigned)(key >> 32), (unsigned)(old & V2_ROW_MASK), 0u);
    }
}

struct V2Probe {
    const uint4 *link; // {key, next} per build row
    const uint64_t *heads;
    uint32_t shift;
    int tagged;
    const void *pkeys;
    int pwidth;
    const uint8_t *pnull;
    int64_t n;
    int kind;
    int pw, bw;                  // payload words out (0: row ids)
    const uint64_t *ppay[JMAXW]; // probe payload columns (pw > 0)
    const uint64_t *bpay[JMAXW]; // build payload columns (bw > 0)
    void *out_p[JMAXW];
    void *out_b[JMAXW];
    uint8_t *out_bnull;
    uint64_t capacity;
    unsigned long long *cursor;
};

// the first build row of r's chain whose key equals `key` at or after link `row` (row + 1; 0 = end)
// (returns the row + 1, and the link after it in *after)
__device__ __forceinline__ uint32_t v2_next_match(const V2Probe &A, uint32_t row, uint64_t key, uint32_t &after) {
    while (row) {
        const uint4 l = A.link[row - 1];
        if ((((uint64_t)l.y << 32) | l.x) == key) {
            after = l.z;
            return row;
        }
        row = l.z;
    }
    after = 0;
    return 0;
}

// Each probe row counts its output rows (INNER: matches, LEFT: max(matches, 1), SEMI: matched,
// ANTI: !matched), the wave reserves its slots with one atomic, then the rows walk their chains
// again (now cache hits) writing probe row / build row outputs.
__global__ void __launch_bounds__(256) join_v2_probe_kernel(V2Probe A) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < A.n; base += stride) {
        const int64_t r = base + threadIdx.x;
        const bool valid = r < A.n;
        const bool isnull = valid && A.pnull && A.pnull[r];
        uint64_t key = 0;
        uint32_t head = 0;
        if (valid && !isnull) {
            key = jload_bits(A.pkeys, A.pwidth, r);
            const uint64_t h = v2_hash(key);
            const uint64_t e = A.heads[h >> A.shift];
            const uint64_t t = h & 0xFFFFull;
            if (!A.tagged || ((e >> V2_TAG_SHIFT) & t) == t) head = (uint32_t)(e & V2_ROW_MASK);
        }
        uint32_t m = 0, first = 0, after = 0;
        for (uint32_t row = v2_next_match(A, head, key, after); row; row = v2_next_match(A, after, key, after)) {
            if (!m) first = row;
            ++m;
            if (A.kind >= TFG_JOIN_SEMI) break; // SEMI / ANTI only need "any"
        }
        uint32_t e = 0;
        if (valid) {
            switch (A.kind) {
            case TFG_JOIN_INNER: e = m; break;
            case TFG_JOIN_LEFT: e = m ? m : 1; break;
            case TFG_JOIN_SEMI: e = m ? 1 : 0; break;
            default: e = m ? 0 : 1; break;
            }
        }
        uint32_t inc = e; // wave-inclusive scan of the output counts
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d, 64);
            if (lane >= d) inc += y;
        }
        unsigned long long wbase = 0;
        if (lane == 63) wbase = atomicAdd(A.cursor, (unsigned long long)inc);
        wbase = __shfl(wbase, 63, 64);
        if (!e) continue;
        uint64_t pos = wbase + inc - e;
        auto emit = [&](uint32_t brow) __attribute__((always_inline)) { // brow: build row + 1, 0 = none
            if (pos < A.capacity) {
                if (A.pw == 0) {
                    ((uint32_t *)A.out_p[0])[pos] = (uint32_t)r;
                } else {
                    for (int w = 0; w < A.pw; ++w) ((uint64_t *)A.out_p[w])[pos] = A.ppay[w][r];
                }
                if (A.out_bnull) A.out_bnull[pos] = brow == 0;
                if (A.bw == 0) {
                    if (A.out_b[0]) ((uint32_t *)A.out_b[0])[pos] = brow ? brow - 1 : 0xFFFFFFFFu;
                } else if (A.out_b[0]) {
                    for (int w = 0; w < A.bw; ++w) ((uint64_t *)A.out_b[w])[pos] = brow ? A.bpay[w][brow - 1] : 0ull;
                }
            }
            ++pos;
        };
        if (m == 1 && A.kind <= TFG_JOIN_LEFT) {
            emit(first); // one match (unique build keys): no second walk
        } else if (A.kind == TFG_JOIN_INNER || (A.kind == TFG_JOIN_LEFT && m)) {
            for (uint32_t row = v2_next_match(A, head, key, after); row; row = v2_next_match(A, after, key, after))
                emit(row);
        } else {
            emit(0); // LEFT without a match / SEMI / ANTI: the probe row alone
        }
    }
}

} // namespace tfg

using namespace tfg;

struct tfg_join {
    Ctx *ctx = nullptr;
    int key_type = 0;
    int width = 8;
    // accumulated build side: keys widened to u64, null flags, payload words
    uint64_t *keys = nullptr;
    uint8_t *nulls = nullptr;
    uint64_t *pay[JMAXW] = {};
    int bw = -1; // payload words per build row (-1: not fixed yet)
    int64_t n_rows = 0, cap_rows = 0;
    // finalized partitioned build
    bool finalized = false;
    uint32_t P = 1;
    int slot_shift = 0;
    uint64_t *brec = nullptr;
    uint32_t *brows = nullptr;
    uint64_t *boff = nullptr;
    int64_t n_inserted = 0;
    uint64_t max_part = 0; // build rows of the largest partition (> JCHUNK: chunked probes need found flags)
    // JoinV2 pointer table (tfg_join_create_v2)
    bool v2 = false;
    bool tagged = false;
    uint64_t *heads = nullptr;
    void *next = nullptr; // uint4 {key, next} links
    uint32_t v2_shift = 64;
    uint64_t v2_size = 0;
};

namespace {

int join_grow(tfg_join *j, int64_t need) {
    if (need <= j->cap_rows) return TFG_OK;
    int64_t nc = std::max<int64_t>(need, j->cap_rows * 2);
    nc = std::max<int64_t>(nc, 1 << 16);
    const int words = std::max(j->bw, 0);
    uint64_t *k;
    uint8_t *z;
    uint64_t *p[JMAXW] = {};
    TFG_HIP(hipMalloc(&k, nc * 8));
    TFG_HIP(hipMalloc(&z, nc));
    for (int w = 0; w < words; ++w) TFG_HIP(hipMalloc(&p[w], nc * 8));
    if (j->n_rows) {
        TFG_HIP(hipMemcpyAsync(k, j->keys, j->n_rows * 8, hipMemcpyDeviceToDevice, j->ctx->stream));
        TFG_HIP(hipMemcpyAsync(z, j->nulls, j->n_rows, hipMemcpyDeviceToDevice, j->ctx->stream));
        for (int w = 0; w < words; ++w)
            TFG_HIP(hipMemcpyAsync(p[w], j->pay[w], j->n_rows * 8, hipMemcpyDeviceToDevice, j->ctx->stream));
    }
    TFG_HIP(hipStreamSynchronize(j->ctx->stream));
    if (j->keys) TFG_HIP(hipFree(j->keys));
    if (j->nulls) TFG_HIP(hipFree(j->nulls));
    for (int w = 0; w < JMAXW; ++w)
        if (j->pay[w]) TFG_HIP(hipFree(j->pay[w]));
    j->keys = k;
    j->nulls = z;
    for (int w = 0; w < JMAXW; ++w) j->pay[w] = p[w];
    j->cap_rows = nc;
    return TFG_OK;
}

void free_build(tfg_join *j) {
    if (j->heads) (void)hipFree(j->heads);
    if (j->next) (void)hipFree(j->next);
    j->heads = nullptr;
    j->next = nullptr;
    if (j->brec) (void)hipFree(j->brec);
    if (j->brows) (void)hipFree(j->brows);
    if (j->boff) (void)hipFree(j->boff);
    j->brec = nullptr;
    j->brows = nullptr;
    j->boff = nullptr;
}

uint32_t bits_of(uint32_t P) {
    uint32_t b = 0;
    while ((1u << b) < P) ++b;
    return b;
}

int build_rows(tfg_join *j, const void *keys, const uint8_t *key_nullmap, int64_t n, int npay, const void *const *pay) {
    TFG_CHECK(j && (n == 0 || keys), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(!j->finalized, TFG_ERR_LOGICAL, "build after finalize");
    TFG_CHECK(npay >= 0 && npay <= JMAXW && (npay == 0 || pay), TFG_ERR_INVALID_ARG, "build payload words %d", npay);
    TFG_CHECK(j->bw < 0 || j->bw == npay, TFG_ERR_LOGICAL, "every build block must carry the same payload columns");
    TFG_CHECK(n >= 0 && j->n_rows + n < (int64_t)0xFFFFFFFFll, TFG_ERR_INVALID_ARG, "build row count out of range");
    if (failpoint("join_build")) return fail(TFG_ERR_FAULT_INJECTED, "failpoint join_build");
    if (int rc = set_device(j->ctx)) return rc;
    if (j->bw < 0) {
        j->bw = npay;
        if (npay && j->cap_rows) { // capacity reserved at create: allocate the payload planes too
            const int64_t cap = j->cap_rows;
            if (j->keys) TFG_HIP(hipFree(j->keys));
            if (j->nulls) TFG_HIP(hipFree(j->nulls));
            j->keys = nullptr;
            j->nulls = nullptr;
            j->cap_rows = 0;
            if (int rc = join_grow(j, cap)) return rc;
        }
    }
    if (n == 0) return TFG_OK;
    if (int rc = join_grow(j, j->n_rows + n)) return rc;
    hipLaunchKernelGGL(widen_keys_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, j->ctx->stream, keys, j->width,
                       key_nullmap, n, j->keys, j->nulls, j->n_rows);
    TFG_LAUNCH_CHECK();
    for (int w = 0; w < npay; ++w)
        TFG_HIP(hipMemcpyAsync(j->pay[w] + j->n_rows, pay[w], n * 8, hipMemcpyDeviceToDevice, j->ctx->stream));
    j->n_rows += n;
    return TFG_OK;
}

int probe_common(tfg_join *j, int kind, const void *keys, const uint8_t *key_nullmap, int64_t n, int npay,
                 const void *const *ppay, void *const *out_p, void *const *out_b, uint8_t *out_bnull, uint64_t capacity,
                 uint64_t *out_count_dev, uint64_t *out_count_host) {
    TFG_CHECK(kind >= TFG_JOIN_INNER && kind <= TFG_JOIN_ANTI, TFG_ERR_NOT_IMPLEMENTED, "join kind %d", kind);
    TFG_CHECK(n >= 0 && n < (int64_t)0xFFFFFFFFll, TFG_ERR_INVALID_ARG, "probe row count out of range");
    TFG_CHECK(npay >= 0 && npay <= JMAXW && (npay == 0 || ppay), TFG_ERR_INVALID_ARG, "probe payload words %d", npay);
    if (failpoint("join_probe")) return fail(TFG_ERR_FAULT_INJECTED, "failpoint join_probe");
    if (!j->finalized)
        if (int rc = tfg_join_finalize(j)) return rc;
    if (int rc = set_device(j->ctx)) return rc;
    Ctx *ctx = j->ctx;
    if (j->v2) { // pointer table: no partitioning, one probe pass
        void *sp;
        if (int rc = scratch_get(ctx, 64, &sp)) return rc;
        unsigned long long *cursor = (unsigned long long *)sp;
        TFG_HIP(hipMemsetAsync(cursor, 0, 8, ctx->stream));
        V2Probe A{};
        A.link = (const uint4 *)j->next;
        A.heads = j->heads;
        A.shift = j->v2_shift;
        A.tagged = j->tagged;
        A.pkeys = keys;
        A.pwidth = j->width;
        A.pnull = key_nullmap;
        A.n = n;
        A.kind = kind;
        A.pw = npay;
        A.bw = j->bw < 0 ? 0 : j->bw;
        for (int w = 0; w < JMAXW; ++w) {
            A.ppay[w] = w < npay ? (const uint64_t *)ppay[w] : nullptr;
            A.bpay[w] = w < A.bw ? j->pay[w] : nullptr;
            A.out_p[w] = out_p ? out_p[w] : nullptr;
            A.out_b[w] = out_b ? out_b[w] : nullptr;
        }
        A.out_bnull = out_bnull;
        A.capacity = capacity;
        A.cursor = cursor;
        if (n > 0) {
            ProfScope _ps(ctx, "join.v2.probe");
            hipLaunchKernelGGL(join_v2_probe_kernel, dim3(stream_grid(n, 256, 16384)), dim3(256), 0, ctx->stream, A);
            TFG_LAUNCH_CHECK();
        }
        if (out_count_dev) TFG_HIP(hipMemcpyAsync(out_count_dev, cursor, 8, hipMemcpyDeviceToDevice, ctx->stream));
        uint64_t total = 0;
        if (int rc = read_back_u64(ctx, (const uint64_t *)cursor, &total, 1)) return rc;
        if (out_count_host) *out_count_host = total;
        if (total > capacity)
            return fail(TFG_ERR_CAPACITY, "join result needs %llu rows, capacity %llu", (unsigned long long)total,
                        (unsigned long long)capacity);
        return TFG_OK;
    }
    const uint32_t P = j->P;
    PartLayout L = make_layout(n, P);
    // payload 0 may be the key column itself (the joined block's key): the record's key word
    // then serves it instead of a second copy
    const bool key_pay0 = npay >= 1 && ppay[0] == keys && j->width == 8;
    const int prw = key_pay0 ? npay : 1 + npay;
    // P > 1024 with payload records: the two-level tiled partition (no histogram passes, no host
    // round trip); the index-pair form (row ids) keeps the histogram + scatter passes
    TiledGeom tg{};
    bool two_level = false;
    if (npay > 0 && n > 0 && P > TWO_PASS_MIN) {
        PCols probe_cols{};
        probe_cols.ncols = prw;
        for (int c = 0; c < prw; ++c) probe_cols.width[c] = 8;
        two_level = make_two_level_geom(ctx, n, P, probe_cols, tg);
    }
    Carver cv;
    const size_t o_wide = cv.take<uint64_t>(j->width == 8 ? 0 : n);
    const size_t o_prec = cv.take<uint64_t>(n * prw), o_pr = cv.take<uint32_t>(npay == 0 ? n : 0);
    const size_t o_poff = cv.take<uint64_t>(P + 1), o_found = cv.take<uint8_t>(n), o_cur = cv.take<uint64_t>(1);
    const size_t o_pin = cv.take<uint64_t>(JMAXW);
    const size_t o_tmp = cv.take<uint8_t>(two_level ? two_level_tmp_bytes(tg, P, prw)
                                                    : part_tmp_bytes(L, (size_t)prw * 8, npay == 0));
    void *sp;
    if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
    char *sb = (char *)sp;
    unsigned long long *cursor = (unsigned long long *)(sb + o_cur);
    TFG_HIP(hipMemsetAsync(cursor, 0, 8, ctx->stream));
    JoinArgs A{};
    A.brec = j->brec;
    A.brows = j->brows;
    A.boff = j->boff;
    A.bw = j->bw < 0 ? 0 : j->bw;
    A.pw = npay;
    A.prw = prw;
    A.pw0 = key_pay0 ? 0 : 1;
    A.kind = kind;
    A.slot_shift = j->slot_shift;
    for (int w = 0; w < JMAXW; ++w) {
        A.out_p[w] = out_p ? out_p[w] : nullptr;
        A.out_b[w] = out_b ? out_b[w] : nullptr;
    }
    A.out_bnull = out_bnull;
    A.capacity = capacity;
    A.cursor = cursor;
    if (n > 0) {
        // probe keys as u64 (narrower key types widened like the build side)
        const void *pk = keys;
        if (j->width != 8) {
            hipLaunchKernelGGL(widen_keys_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, ctx->stream, keys,
                               j->width, nullptr, n, (uint64_t *)(sb + o_wide), nullptr, (int64_t)0);
            TFG_LAUNCH_CHECK();
            pk = sb + o_wide;
        }
        PCols pc{};
        pc.ncols = prw;
        pc.in[0] = pk;
        pc.out[0] = sb + o_prec;
        pc.width[0] = 8;
        for (int w = key_pay0 ? 1 : 0; w < npay; ++w) {
            pc.in[pc.ncols - npay + w] = ppay[w];
            pc.width[pc.ncols - npay + w] = 8;
        }
        pc.key0 = 1;
        pc.aos = prw >= 2;
        pc.two_pass = 1;
        SelJoin sel{pk, key_nullmap, 8, fib_shift(P)};
        RowPred pred{};
        uint64_t *poff = (uint64_t *)(sb + o_poff);
        uint32_t *prows = npay == 0 ? (uint32_t *)(sb + o_pr) : nullptr;
        if (two_level) {
            pc.aos = 1;
            if (int rc = run_partition_two_level(ctx, sel, pred, tg, P, pc, poff, sb + o_tmp, "join.part.tiled",
                                                 "join.part.regroup"))
                return rc;
        } else if (int rc = run_partition<SelJoin, false>(ctx, sel, pred, L, pc, prows, nullptr, poff, sb + o_tmp,
                                                          "join.part.hist", "join.part.scatter")) {
            return rc;
        }
        if (j->max_part > (uint64_t)JCHUNK) // only chunked partitions read / write the found flags
            TFG_HIP(hipMemsetAsync(sb + o_found, 0, n, ctx->stream));
        A.prec = (const uint64_t *)(sb + o_prec);
        A.prows = prows;
        A.poff = poff;
        A.found = (uint8_t *)(sb + o_found);
        {
            ProfScope _ps(ctx, "join.probe");
            TFG_CHECK(prw >= 1 && prw <= 3 && A.bw >= 0 && A.bw <= 2, TFG_ERR_INVALID_ARG, "join record words");
            void (*kern)(JoinArgs);
            switch (prw * 3 + A.bw) {
            case 3: kern = join_probe_kernel<1, 0>; break;
            case 4: kern = join_probe_kernel<1, 1>; break;
            case 5: kern = join_probe_kernel<1, 2>; break;
            case 6: kern = join_probe_kernel<2, 0>; break;
            case 7: kern = join_probe_kernel<2, 1>; break;
            case 8: kern = join_probe_kernel<2, 2>; break;
            case 9: kern = join_probe_kernel<3, 0>; break;
            case 10: kern = join_probe_kernel<3, 1>; break;
            default: kern = join_probe_kernel<3, 2>; break;
            }
            hipLaunchKernelGGL(kern, dim3(P), dim3(JT), sizeof(JLds), ctx->stream, A);
        }
        TFG_LAUNCH_CHECK();
        if (key_nullmap && (kind == TFG_JOIN_LEFT || kind == TFG_JOIN_ANTI)) {
            const void **pin = nullptr;
            if (npay) {
                pin = (const void **)(sb + o_pin); // device array of the payload pointers
                TFG_HIP(hipMemcpyAsync(pin, ppay, npay * sizeof(void *), hipMemcpyHostToDevice, ctx->stream));
            }
            hipLaunchKernelGGL(join_null_rows_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, ctx->stream,
                               key_nullmap, n, A, (const void *const *)pin, npay);
            TFG_LAUNCH_CHECK();
        }
    }
    if (out_count_dev) TFG_HIP(hipMemcpyAsync(out_count_dev, cursor, 8, hipMemcpyDeviceToDevice, ctx->stream));
    uint64_t total = 0;
    if (int rc = read_back_u64(ctx, (const uint64_t *)cursor, &total, 1)) return rc;
    if (out_count_host) *out_count_host = total;
    if (total > capacity)
        return fail(TFG_ERR_CAPACITY, "join result needs %llu rows, capacity %llu", (unsigned long long)total,
                    (unsigned long long)capacity);
    return TFG_OK;
}

// ---------------------------------------------------------------- general join keys (§8 f2)
// chooseJoinMapMethod (Interpreters/JoinHashMap.cpp:33-116) picks keys128 / keys256 for several
// fixed keys, key_strbin / key_strbinpadding for one String key (by collator) and serialized
// otherwise.  Here every such key set joins through the one fixed-width table: each row's key
// tuple is folded into a 64-bit fingerprint (tfg_join_key_hash), the u64 join produces the
// candidate pairs, and tfg_join_keys_equal keeps the pairs whose full key tuples are equal, so
// a fingerprint collision costs a rejected pair, never a wrong one.  A row with a NULL in any
// key column is a NULL key (extractNestedColumnsAndNullMap ORs the key null maps).
constexpr int JKMAX = 8;
struct JoinKeyCols {
    int nkeys;
    int width[JKMAX]; // bytes; 0 = String
    int collator[JKMAX];
    const void *col[JKMAX];
    const uint64_t *offsets[JKMAX];
    const uint8_t *nullmap[JKMAX];
    int compact[JKMAX]; // tfg_join_keys_equal: the column holds pair i's key at row i (collated)
};

__device__ __forceinline__ uint64_t jk_mix(uint64_t h, uint64_t w) {
    h = (h ^ w) * 0xbf58476d1ce4e5b9ull;
    return h ^ (h >> 31);
}

// the collator's sort key of String row r: [s, s + len)  (BinCollatorSortKey<true> right-trims)
__device__ __forceinline__ const uint8_t *jk_sort_key(const JoinKeyCols &k, int j, int64_t r, int64_t &len) {
    const uint64_t s = r ? k.offsets[j][r - 1] : 0, e = k.offsets[j][r];
    const uint8_t *c = (const uint8_t *)k.col[j] + s;
    len = (int64_t)(e - s) - 1; // rows end with '\0'
    if (k.collator[j] == TFG_COLLATOR_BIN_PADDING)
        while (len > 0 && c[len - 1] == ' ') --len;
    return c;
}

__global__ void join_key_hash_kernel(JoinKeyCols k, int64_t n, uint64_t *out, uint8_t *out_null) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        uint64_t h = 0x2545F4914F6CDD1Dull;
        uint8_t isnull = 0;
        for (int j = 0; j < k.nkeys; ++j) {
            if (k.nullmap[j] && k.nullmap[j][r]) {
                isnull = 1;
                break;
            }
            const int wd = k.width[j];
            if (wd == 0) {
                int64_t len;
                const uint8_t *c = jk_sort_key(k, j, r, len);
                uint64_t w = 0;
                for (int64_t i = 0; i < len; ++i) {
                    w |= (uint64_t)c[i] << ((i & 7) * 8);
                    if ((i & 7) == 7) {
                        h = jk_mix(h, w);
                        w = 0;
                    }
                }
                h = jk_mix(h, w ^ ((uint64_t)len << 56)); // tail word tagged with the length
            } else if (wd <= 8) {
                h = jk_mix(h, jload_bits(k.col[j], wd, r));
            } else {
                const uint64_t *p = (const uint64_t *)k.col[j] + (int64_t)(wd / 8) * r;
                for (int i = 0; i < wd / 8; ++i) h = jk_mix(h, p[i]);
            }
        }
        // fmix64 so the partition radix (the product's high bits) sees every input bit
        h ^= h >> 33;
        h *= 0xff51afd7ed558ccdull;
        h ^= h >> 33;
        h *= 0xc4ceb9aa6b8f5d35ull;
        h ^= h >> 33;
        out[r] = isnull ? 0 : h;
        if (out_null) out_null[r] = isnull;
    }
}

__global__ void join_keys_equal_kernel(JoinKeyCols pk, JoinKeyCols bk, const uint32_t *pidx, const uint32_t *bidx,
                                       const uint8_t *pass_in, int64_t n, uint8_t *pass_out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bool eq = pass_in ? pass_in[i] != 0 : true;
        const int64_t p = pidx[i], b = bidx[i];
        for (int j = 0; j < pk.nkeys && eq; ++j) {
            const int wd = pk.width[j];
            if (wd == 0) {
                int64_t lp, lb;
                const uint8_t *cp = jk_sort_key(pk, j, pk.compact[j] ? i : p, lp);
                const uint8_t *cb = jk_sort_key(bk, j, bk.compact[j] ? i : b, lb);
                eq = lp == lb;
                for (int64_t t = 0; t < lp && eq; ++t) eq = cp[t] == cb[t];
            } else if (wd <= 8) {
                eq = jload_bits(pk.col[j], wd, p) == jload_bits(bk.col[j], wd, b);
            } else {
                const uint64_t *a = (const uint64_t *)pk.col[j] + (int64_t)(wd / 8) * p;
                const uint64_t *c = (const uint64_t *)bk.col[j] + (int64_t)(wd / 8) * b;
                for (int t = 0; t < wd / 8 && eq; ++t) eq = a[t] == c[t];
            }
        }
        pass_out[i] = eq ? 1 : 0;
    }
}

int join_key_cols(int nkeys, const int *types, const int *collators, const void *const *cols,
                  const uint64_t *const *offsets, const uint8_t *const *nullmaps, JoinKeyCols &k) {
    TFG_CHECK(nkeys >= 1 && nkeys <= JKMAX && types && cols, TFG_ERR_INVALID_ARG, "join keys: need 1-%d key columns",
              JKMAX);
    k = JoinKeyCols{};
    k.nkeys = nkeys;
    for (int j = 0; j < nkeys; ++j) {
        k.col[j] = cols[j];
        k.nullmap[j] = nullmaps ? nullmaps[j] : nullptr;
        k.collator[j] = collators ? collators[j] : TFG_COLLATOR_NONE;
        TFG_CHECK(collator_known(k.collator[j]), TFG_ERR_NOT_IMPLEMENTED, "join key collator %d not supported",
                  k.collator[j]);
        if (types[j] == TFG_STRING) {
            TFG_CHECK(offsets && offsets[j], TFG_ERR_INVALID_ARG, "String join key %d without offsets", j);
            k.offsets[j] = offsets[j];
            k.width[j] = 0;
        } else {
            const size_t w = type_width(types[j]);
            TFG_CHECK(w == 1 || w == 2 || w == 4 || w == 8 || w == 16, TFG_ERR_ILLEGAL_TYPE,
                      "unsupported join key type %d", types[j]);
            k.width[j] = (int)w;
        }
    }
    return TFG_OK;
}

} // namespace

extern "C" {

int tfg_join_key_hash(tfg_ctx *ctx, int nkeys, const int *key_types, const int *key_collators,
                      const void *const *key_cols, const uint64_t *const *key_offsets,
                      const uint8_t *const *key_nullmaps, int64_t n, uint64_t *out_keys, uint8_t *out_nullmap) {
    TFG_CHECK(ctx && (n == 0 || out_keys), TFG_ERR_INVALID_ARG, "null argument");
    JoinKeyCols k;
    if (int rc = join_key_cols(nkeys, key_types, key_collators, key_cols, key_offsets, key_nullmaps, k)) return rc;
    if (n <= 0) return TFG_OK;
    for (int j = 0; j < nkeys; ++j) TFG_CHECK(key_cols[j], TFG_ERR_INVALID_ARG, "null key column %d", j);
    if (int rc = set_device(ctx)) return rc;
    // String keys under a case-insensitive collator: their sort-key columns (GeneralCI weights)
    CollatedStrings cs[JKMAX];
    for (int j = 0; j < nkeys; ++j) {
        if (k.width[j] != 0 || !collator_transforms(k.collator[j])) continue;
        if (int rc = collate_strings(ctx, k.collator[j], (const uint8_t *)k.col[j], k.offsets[j], k.nullmap[j], nullptr,
                                     nullptr, n, cs[j]))
            return rc;
        k.col[j] = cs[j].chars;
        k.offsets[j] = cs[j].offsets();
        k.collator[j] = TFG_COLLATOR_NONE;
    }
    hipLaunchKernelGGL(join_key_hash_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, ctx->stream, k, n, out_keys,
                       out_nullmap);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_join_keys_equal(tfg_ctx *ctx, int nkeys, const int *key_types, const int *key_collators,
                        const void *const *probe_cols, const uint64_t *const *probe_offsets,
                        const void *const *build_cols, const uint64_t *const *build_offsets, const uint32_t *probe_idx,
                        const uint32_t *build_idx, const uint8_t *pass_in, int64_t n_pairs, uint8_t *out_pass) {
    TFG_CHECK(ctx && (n_pairs == 0 || (probe_idx && build_idx && out_pass)), TFG_ERR_INVALID_ARG, "null argument");
    JoinKeyCols pk, bk;
    if (int rc = join_key_cols(nkeys, key_types, key_collators, probe_cols, probe_offsets, nullptr, pk)) return rc;
    if (int rc = join_key_cols(nkeys, key_types, key_collators, build_cols, build_offsets, nullptr, bk)) return rc;
    if (n_pairs <= 0) return TFG_OK;
    if (int rc = set_device(ctx)) return rc;
    // case-insensitive String keys: the sort keys of the pairs' rows, pair i at row i
    CollatedStrings cp[JKMAX], cb[JKMAX];
    for (int j = 0; j < nkeys; ++j) {
        if (pk.width[j] != 0 || !collator_transforms(pk.collator[j])) continue;
        if (int rc = collate_strings(ctx, pk.collator[j], (const uint8_t *)pk.col[j], pk.offsets[j], nullptr, probe_idx,
                                     nullptr, n_pairs, cp[j]))
            return rc;
        if (int rc = collate_strings(ctx, bk.collator[j], (const uint8_t *)bk.col[j], bk.offsets[j], nullptr, build_idx,
                                     nullptr, n_pairs, cb[j]))
            return rc;
        pk.col[j] = cp[j].chars;
        pk.offsets[j] = cp[j].offsets();
        bk.col[j] = cb[j].chars;
        bk.offsets[j] = cb[j].offsets();
        pk.collator[j] = bk.collator[j] = TFG_COLLATOR_NONE;
        pk.compact[j] = bk.compact[j] = 1;
    }
    hipLaunchKernelGGL(join_keys_equal_kernel, dim3(stream_grid(n_pairs, 256)), dim3(256), 0, ctx->stream, pk, bk,
                       probe_idx, build_idx, pass_in, n_pairs, out_pass);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_join_create(tfg_ctx *ctx, int key_type, int64_t expected_build_rows, tfg_join **out) {
    TFG_CHECK(ctx && out, TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(type_width(key_type) > 0 && type_width(key_type) <= 8 && !is_float_type(key_type), TFG_ERR_ILLEGAL_TYPE,
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

int tfg_join_create_v2(tfg_ctx *ctx, int key_type, int64_t expected_build_rows, int flags, tfg_join **out) {
    if (int rc = tfg_join_create(ctx, key_type, expected_build_rows, out)) return rc;
    (*out)->v2 = true;
    (*out)->tagged = (flags & TFG_JOIN_V2_TAGGED) != 0;
    return TFG_OK;
}

int tfg_join_destroy(tfg_join *j) {
    if (!j) return TFG_OK;
    (void)hipSetDevice(j->ctx->device);
    (void)hipStreamSynchronize(j->ctx->stream);
    if (j->keys) (void)hipFree(j->keys);
    if (j->nulls) (void)hipFree(j->nulls);
    for (int w = 0; w < JMAXW; ++w)
        if (j->pay[w]) (void)hipFree(j->pay[w]);
    free_build(j);
    delete j;
    return TFG_OK;
}

int tfg_join_build(tfg_join *j, const void *keys, const uint8_t *key_nullmap, int64_t n) {
    return build_rows(j, keys, key_nullmap, n, 0, nullptr);
}

int tfg_join_build_rows(tfg_join *j, const void *keys, const uint8_t *key_nullmap, int64_t n, int npay,
                        const void *const *pay) {
    return build_rows(j, keys, key_nullmap, n, npay, pay);
}

int tfg_join_finalize(tfg_join *j) {
    TFG_CHECK(j, TFG_ERR_INVALID_ARG, "join is null");
    if (j->finalized) return TFG_OK;
    if (int rc = set_device(j->ctx)) return rc;
    Ctx *ctx = j->ctx;
    if (j->bw < 0) j->bw = 0;
    if (j->v2) { // HashJoinPointerTable::init + build
        const int64_t n = j->n_rows;
        uint64_t size = 1024;
        while (size < (uint64_t)(2 * n) && size < (1ull << 32)) size <<= 1;
        uint32_t deg = 0;
        while ((1ull << deg) < size) ++deg;
        j->v2_size = size;
        j->v2_shift = 64 - deg;
        TFG_HIP(hipMalloc(&j->heads, size * 8));
        TFG_HIP(hipMalloc(&j->next, std::max<int64_t>(n, 1) * 16)); // {key, next} links
        TFG_HIP(hipMemsetAsync(j->heads, 0, size * 8, ctx->stream));
        if (n > 0) {
            ProfScope _ps(ctx, "join.v2.build");
            hipLaunchKernelGGL(join_v2_build_kernel, dim3(stream_grid(n, 256, 16384)), dim3(256), 0, ctx->stream, j->keys,
                               j->nulls, n, j->heads, j->v2_shift, (int)j->tagged, (uint4 *)j->next);
            TFG_LAUNCH_CHECK();
        }
        j->n_inserted = n;
        j->P = 1;
        j->finalized = true;
        return TFG_OK;
    }
    // partitions of ~JFILL build rows (table load ~0.63); the staged scatter takes P <= 4096
    uint32_t P = 1;
    while ((int64_t)P * JFILL < j->n_rows && P < 4096u) P <<= 1;
    j->P = P;
    j->slot_shift = 64 - (int)bits_of(P) - (int)bits_of(JCAP / JGS);
    const int64_t n = j->n_rows;
    const int brw = 1 + j->bw;
    TFG_HIP(hipMalloc(&j->brec, std::max<int64_t>(n, 1) * 8 * brw));
    TFG_HIP(hipMalloc(&j->brows, std::max<int64_t>(n, 1) * 4));
    TFG_HIP(hipMalloc(&j->boff, (P + 1) * 8));
    PartLayout L = make_layout(n, P);
    void *tmp;
    if (int rc = scratch_get(ctx, part_tmp_bytes(L, (size_t)brw * 8, true), &tmp)) return rc;
    PCols pc{};
    pc.ncols = brw;
    pc.in[0] = j->keys;
    pc.out[0] = j->brec;
    pc.width[0] = 8;
    for (int w = 0; w < j->bw; ++w) {
        pc.in[1 + w] = j->pay[w];
        pc.width[1 + w] = 8;
    }
    pc.key0 = 1;
    pc.aos = brw >= 2;
    pc.two_pass = 1;
    SelJoin sel{j->keys, j->nulls, 8, fib_shift(P)};
    RowPred pred{};
    if (int rc = run_partition<SelJoin, false>(ctx, sel, pred, L, pc, j->brows, nullptr, j->boff, tmp, "join.build.hist",
                                               "join.build.scatter"))
        return rc;
    std::vector<uint64_t> hb(P + 1);
    TFG_HIP(hipMemcpyAsync(hb.data(), j->boff, (P + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    j->n_inserted = (int64_t)hb[P];
    j->max_part = 0;
    for (uint32_t p = 0; p < P; ++p) j->max_part = std::max<uint64_t>(j->max_part, hb[p + 1] - hb[p]);
    j->finalized = true;
    return TFG_OK;
}

int tfg_join_stats(tfg_join *j, uint64_t *rows, uint64_t *partitions) {
    TFG_CHECK(j, TFG_ERR_INVALID_ARG, "join is null");
    if (rows) *rows = (uint64_t)j->n_inserted;
    if (partitions) *partitions = j->P;
    return TFG_OK;
}

int tfg_join_mark(tfg_ctx *ctx, const uint32_t *probe_idx, const uint8_t *pass, int64_t n_pairs, uint8_t *flags) {
    TFG_CHECK(ctx && (n_pairs == 0 || (probe_idx && flags)), TFG_ERR_INVALID_ARG, "null argument");
    if (n_pairs <= 0) return TFG_OK;
    hipLaunchKernelGGL(join_mark_kernel, dim3(stream_grid(n_pairs, 256)), dim3(256), 0, ctx->stream, probe_idx, pass,
                       n_pairs, flags);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_join_probe(tfg_join *j, int kind, const void *keys, const uint8_t *key_nullmap, int64_t n,
                   uint32_t *out_probe_idx, uint32_t *out_build_idx, uint64_t capacity, uint64_t *out_count_dev,
                   uint64_t *out_count_host) {
    TFG_CHECK(j && (n == 0 || keys) && (capacity == 0 || out_probe_idx), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(j->bw <= 0, TFG_ERR_LOGICAL, "index-pair probe of a join built with payload columns");
    void *op[JMAXW] = {out_probe_idx, nullptr};
    void *ob[JMAXW] = {out_build_idx, nullptr};
    return probe_common(j, kind, keys, key_nullmap, n, 0, nullptr, op, ob, nullptr, capacity, out_count_dev,
                        out_count_host);
}

int tfg_join_probe_rows(tfg_join *j, int kind, const void *keys, const uint8_t *key_nullmap, int64_t n, int npay,
                        const void *const *probe_pay, void *const *out_probe, void *const *out_build,
                        uint8_t *out_build_null, uint64_t capacity, uint64_t *out_count_host) {
    TFG_CHECK(j && (n == 0 || keys) && (capacity == 0 || out_probe), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(npay >= 1 && npay <= JMAXW, TFG_ERR_INVALID_ARG, "materialising probe needs 1-%d probe payload columns",
              JMAXW);
    if (!j->finalized)
        if (int rc = tfg_join_finalize(j)) return rc;
    void *op[JMAXW] = {}, *ob[JMAXW] = {};
    for (int w = 0; w < npay && capacity; ++w) {
        TFG_CHECK(out_probe[w], TFG_ERR_INVALID_ARG, "null probe output column");
        op[w] = out_probe[w];
    }
    for (int w = 0; w < j->bw && kind <= TFG_JOIN_LEFT && capacity; ++w) {
        TFG_CHECK(out_build && out_build[w], TFG_ERR_INVALID_ARG, "null build output column");
        ob[w] = out_build[w];
    }
    return probe_common(j, kind, keys, key_nullmap, n, npay, probe_pay, op, ob,
                        kind == TFG_JOIN_LEFT ? out_build_null : nullptr, capacity, nullptr, out_count_host);
}

} // extern "C"
