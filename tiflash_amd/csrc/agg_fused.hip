// agg_fused.hip — fused filter -> GROUP BY (a5 + a9-a17) for the C2 signatures, one launch.
//
// Reference: FilterTransformAction::transform (DataStreams/FilterTransformAction.cpp:72-173)
// feeding Aggregator::executeOnBlock (Interpreters/Aggregator.cpp:1127-1246) with a key64
// HashMap and sum / count states (AggregateFunctionSum.h:64-172, AggregateFunctionCount.h:46),
// merged per TwoLevelHashTable bucket (MergingBuckets, Aggregator.cpp:2940-3097).
//
// The two-kernel path (tile-sorted partition -> bucket kernel, agg.hip) writes every kept row to
// HBM as a 16-byte record and reads it back: 3.1 GB of staging traffic on top of the 2.4 GB of
// input for C2.  Here one persistent workgroup per CU (cooperative launch: all resident) owns one
// of 256 buckets for the whole input, its LDS hash table alive from the first row to the last.
// The input streams through in rounds of 256 tiles x 2048 rows, staged through a 32 MB ring
// small enough to stay in the Infinity Cache.  Each workgroup runs two roles concurrently, on
// separate waves (separate vmcnt domains, so neither role's waits cover the other's memory):
//   producer (waves 8-15), round i: load its tile of round i (two rounds ahead), evaluate the
//       predicate, route every kept row to bucket fib(key) >> 56, counting-sort the tile by
//       bucket in LDS, write it write-through (sc1) to ring slot i % 4, drain, then publish one
//       4-byte run entry per bucket {tag(i), start, count} (sc1): the entry is the flag (R2
//       granules, cdna_hip_programming.md Guideline 16);
//   consumer (waves 0-7), round q: poll the 256 run entries of its bucket, scan them, load its
//       records from the 256 tiles (sc1 loads), fold them into the table, then one agent-scope
//       add (sharded per XCD) releases the ring slot to the producers.
// Roles synchronise with LDS-counter barriers of their own waves; the ring slots with global
// counters.  Rows whose bucket table is full (more distinct keys than FUSED_MAXFILL) go to a
// spill list the caller aggregates afterwards, so any distribution is exact.  Every global spin
// is bounded: a timeout sets the error word and both roles leave their loops.
#include "agg_fused.h"

namespace tfg {
namespace {

constexpr int FT = 1024;               // threads per workgroup (16 waves), one workgroup per CU
constexpr int GT = FT / 2;             // threads per role
constexpr int GW = GT / 64;            // waves per role
constexpr int NB = FUSED_BUCKETS;      // buckets = workgroups = producers
constexpr int TR = 2048;               // rows per tile
constexpr int PR = TR / GT;            // input rows per producer thread per tile
constexpr int KS = 4;                  // ring slots
constexpr int CAP = FUSED_TABLE_CAP;   // table cells; side slot CAP holds key 0 (ZeroValueStorage)
constexpr int GS = 4;                  // cells per probe group (two ds_read_b128)
constexpr int NGRP = CAP / GS;
constexpr int MAXFILL = FUSED_MAXFILL; // sticky "full" threshold
constexpr int CR = 4;                  // records per consumer thread per step
constexpr int NSHARD = 8;              // slot-release counters per slot (one per XCD shard)
constexpr int SHARD_WORDS = 16;        // each counter on a 64-byte line of its own
constexpr unsigned SPIN_LIMIT = 1u << 24;

constexpr int OFF_KEYS = 0;
constexpr int OFF_ACC = OFF_KEYS + (CAP + 2) * 8;
constexpr int OFF_CNT = OFF_ACC + (CAP + 2) * 8;
constexpr int OFF_SREC = (OFF_CNT + (CAP + 2) * 4 + 15) & ~15;
constexpr int OFF_HIST = OFF_SREC + TR * 16; // [2][NB] producer: bucket counts of rounds i, i - 1
constexpr int OFF_START = OFF_HIST + 2 * NB * 4; // [2][NB] producer: bucket starts
constexpr int OFF_CENT = OFF_START + 2 * NB * 4; // [2][NB] consumer: run entries of rounds q, q - 1
constexpr int OFF_CPREF = OFF_CENT + 2 * NB * 4; // [2][NB + 4] consumer: record prefix per producer
constexpr int OFF_CTRL = OFF_CPREF + 2 * (NB + 4) * 4;
constexpr int LDS_BYTES = OFF_CTRL + 64;
static_assert(LDS_BYTES <= 160 * 1024, "fused workgroup exceeds the CU's LDS");

struct Ctrl {
    unsigned used;      // claimed table cells
    unsigned full;      // sticky: no more inserts
    unsigned zero_used; // key 0 side slot
    unsigned stop[2];   // per role: a spin timed out, leave the loop (read after a role barrier)
    unsigned bar[2];    // per role: barrier arrivals (monotonic)
    unsigned kept[2];   // producer: rows kept per tile (double-buffered)
    unsigned ctot[2];   // consumer: records per round (double-buffered)
    unsigned pad;
    unsigned long long out_base;
    unsigned long long out_count;
};
static_assert(sizeof(Ctrl) <= 64, "ctrl block");

constexpr size_t RING_REC_BYTES = (size_t)KS * NB * TR * 16;
static_assert(RING_REC_BYTES < 0x7FFFFF00u, "the dropped-store offset must lie outside the ring");
constexpr size_t RING_RUN_BYTES = (size_t)KS * NB * NB * 4;
constexpr size_t CONS_BYTES = (size_t)KS * NSHARD * SHARD_WORDS * 4;
constexpr size_t CTL_BYTES = 64; // err word + cursors

struct FArgs {
    const uint64_t *key;
    const uint64_t *val;
    int64_t n;
    int rounds;
    uint4 *ring_rec;                 // [KS][NB][TR] records {key, value}
    uint32_t *ring_run;              // [KS][NB producer][NB bucket]: tag << 24 | start << 12 | count
    uint32_t *cons_done;             // [KS][NSHARD][SHARD_WORDS]
    uint32_t *err;                   // 1 = a spin timed out
    unsigned long long *cursor;      // [0] spilled rows, [1] groups written
    FusedIO io;
#ifdef TFG_FUSED_TRACE // tools/fused_trace.hip: per-phase timestamps (not in the product build)
    unsigned long long *trace;
#endif
};

#ifdef TFG_FUSED_TRACE
#define FUSED_TRACE(lead, r, k) \
    if (lead) A.trace[((size_t)blockIdx.x * A.rounds + (r)) * 8 + (k)] = wall_clock64()
#else
#define FUSED_TRACE(lead, r, k)
#endif

__device__ __forceinline__ uint32_t round_tag(int r) { return (uint32_t)(r % 255) + 1u; }

// barrier of one role's GW waves: LDS arrival counter, monotonic target (gen)
__device__ __forceinline__ void role_barrier(unsigned *bar, unsigned &gen) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // this wave's LDS writes are done
    gen += GW;
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

// bounded relaxed poll (sc1 loads) until f() holds; false after a timeout (error word set)
template <typename F> __device__ bool spin_until(F &&f, const FArgs &A, unsigned *stop) {
    for (unsigned spins = 0; !f(); ++spins) {
        if (spins >= SPIN_LIMIT || __hip_atomic_load(A.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            __hip_atomic_store(A.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *stop = 1;
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}

// exclusive scan of NB counts by ONE wave (4 per lane): out[p] = sum of in[< p], *total = sum
__device__ __forceinline__ void wave_scan_nb(const uint32_t *in, uint32_t *out, unsigned *total, uint32_t mask) {
    const unsigned lane = threadIdx.x & 63;
    uint32_t v[NB / 64], x = 0;
#pragma unroll
    for (int k = 0; k < NB / 64; ++k) {
        v[k] = in[lane * (NB / 64) + k] & mask;
        x += v[k];
    }
    uint32_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if ((int)lane >= d) inc += y;
    }
    uint32_t off = inc - x;
#pragma unroll
    for (int k = 0; k < NB / 64; ++k) {
        out[lane * (NB / 64) + k] = off;
        off += v[k];
    }
    if (lane == 63) *total = inc;
}

// rows loaded per tile row by a predicate type (-1: data-dependent, e.g. an optional null map)
template <typename P> struct PredLoads { static constexpr int value = -1; };
template <typename T> struct PredLoads<PredT<0, T, true>> { static constexpr int value = 0; };
template <int K, typename T> struct PredLoads<PredT<K, T, false>> { static constexpr int value = K == 0 ? 0 : 1; };

// s_waitcnt vmcnt(N) (expcnt / lgkmcnt not waited), visible to the compiler's wait scoreboard,
// plus the opaque form (R1)
template <int N> __device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | 0x0F70);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename Pred> struct TileRegs {
    Loaded pl[PR];
    uint64_t k[PR], v[PR];
    bool ok[PR];
};

// producer thread pt's rows of its tile of `round` (unconditional loads: rows past n re-read
// row n - 1, so the compiler's wait counts stay static)
template <typename Pred, bool HASVAL>
__device__ __forceinline__ void load_tile(const Pred &pred, const FArgs &A, int round, int pt, TileRegs<Pred> &x) {
    const int64_t base = (int64_t)round * (NB * TR) + (int64_t)blockIdx.x * TR + pt;
#pragma unroll
    for (int j = 0; j < PR; ++j) {
        const int64_t r0 = base + (int64_t)j * GT;
        x.ok[j] = r0 < A.n;
        const int64_t r = x.ok[j] ? r0 : A.n - 1;
        x.pl[j] = pred.load(r);
        x.k[j] = A.key[r];
        if constexpr (HASVAL) x.v[j] = A.val[r];
    }
}

struct FTable {
    uint64_t *keys;
    uint64_t *acc;
    uint32_t *cnt;
    Ctrl *ctrl;

    // probe group: the 32 Fibonacci-product bits below the bucket radix, scaled to NGRP groups
    static __device__ __forceinline__ unsigned slot_group(uint64_t key) {
        const uint32_t below = (uint32_t)(((key * 0x9E3779B97F4A7C15ull) << 8) >> 32);
        return (unsigned)(((uint64_t)below * NGRP) >> 32);
    }

    // cell of each valid key, inserting new keys while allowed (-1 = not in the table); R lookups
    // interleaved so their LDS latency chains overlap
    template <int R>
    __device__ __forceinline__ void find_multi(const uint64_t (&key)[R], const bool (&valid)[R], bool may_insert,
                                               int (&cell)[R]) {
        unsigned grp[R];
        bool live[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            cell[u] = -1;
            live[u] = false;
            if (!valid[u]) continue;
            if (key[u] == 0) { // ZeroValueStorage: same insert rule as table cells
                if (!__hip_atomic_load(&ctrl->zero_used, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                    if (!may_insert) continue;
                    __hip_atomic_store(&ctrl->zero_used, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                cell[u] = CAP;
                continue;
            }
            grp[u] = slot_group(key[u]);
            live[u] = true;
        }
        for (int step = 0; step < NGRP; ++step) {
            uint64_t k[R][GS];
#pragma unroll
            for (int u = 0; u < R; ++u)
                if (live[u]) {
                    const uint4 a = *reinterpret_cast<const uint4 *>(&keys[grp[u] * GS]);
                    const uint4 b = *reinterpret_cast<const uint4 *>(&keys[grp[u] * GS + 2]);
                    k[u][0] = ((uint64_t)a.y << 32) | a.x;
                    k[u][1] = ((uint64_t)a.w << 32) | a.z;
                    k[u][2] = ((uint64_t)b.y << 32) | b.x;
                    k[u][3] = ((uint64_t)b.w << 32) | b.z;
                }
            bool any = false;
#pragma unroll
            for (int u = 0; u < R; ++u) {
                if (!live[u]) continue;
                int hit = -1, empty = -1;
#pragma unroll
                for (int s = 0; s < GS; ++s) {
                    if (k[u][s] == key[u] && hit < 0) hit = s;
                    if (k[u][s] == 0 && empty < 0) empty = s;
                }
                if (hit >= 0 && (empty < 0 || hit < empty)) {
                    cell[u] = (int)(grp[u] * GS + hit);
                    live[u] = false;
                } else if (empty >= 0) {
                    if (!may_insert ||
                        __hip_atomic_load(&ctrl->full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                        live[u] = false; // a definitive miss
                        continue;
                    }
                    const int c = (int)(grp[u] * GS + empty);
                    const uint64_t old = atomicCAS((unsigned long long *)&keys[c], 0ull, (unsigned long long)key[u]);
                    if (old == 0 || old == key[u]) {
                        if (old == 0) {
                            const unsigned nu = atomicAdd(&ctrl->used, 1u) + 1;
                            if (nu >= (unsigned)MAXFILL) ctrl->full = 1;
                        }
                        cell[u] = c;
                        live[u] = false;
                    } else {
                        any = true; // lost the cell to another key: re-read the group
                    }
                } else {
                    grp[u] = grp[u] + 1 == (unsigned)NGRP ? 0 : grp[u] + 1; // full group: the next one
                    any = true;
                }
            }
            if (!any) break;
        }
    }
};

template <int SOP, bool CNT>
__device__ __forceinline__ void fold(FTable &T, int cell, uint64_t v) {
    if constexpr (SOP == 2) atomicAdd((unsigned long long *)&T.acc[cell], (unsigned long long)v);
    if constexpr (SOP == 3) atomicAdd((double *)&T.acc[cell], __longlong_as_double((long long)v));
    if constexpr (CNT) atomicAdd(&T.cnt[cell], 1u);
}

// ---------------------------------------------------------------- producer role (waves 8-15)
// Iteration i sorts round i and finishes round i - 1: rank + scan + place of round i (its tile
// was loaded two iterations ago), then the wait for round i - 1's write-through stores (they
// drained during the sort), publish of round i - 1, the slot wait of round i, then the loads of
// round i + 2 and the stores of round i.  The wait counts leave the youngest (the loads of
// round i + 1, issued after round i - 1's stores) in flight when the load count is static.
template <typename Pred, int SOP>
__device__ __forceinline__ void produce_iteration(const Pred &pred, const FArgs &A, char *lds, int i, TileRegs<Pred> &cur,
                                                  unsigned &gen, const __amdgpu_buffer_rsrc_t &ring) {
    constexpr bool HASVAL = SOP != 0;
    constexpr int PL = PredLoads<Pred>::value;
    constexpr int TILE_LOADS = PL < 0 ? -1 : PR * (PL + 1 + (HASVAL ? 1 : 0));
    uint4 *srec = reinterpret_cast<uint4 *>(lds + OFF_SREC);
    uint32_t *hist = reinterpret_cast<uint32_t *>(lds + OFF_HIST) + (i & 1) * NB;
    uint32_t *start = reinterpret_cast<uint32_t *>(lds + OFF_START) + (i & 1) * NB;
    uint32_t *phist = reinterpret_cast<uint32_t *>(lds + OFF_HIST) + ((i + 1) & 1) * NB;  // round i - 1
    uint32_t *pstart = reinterpret_cast<uint32_t *>(lds + OFF_START) + ((i + 1) & 1) * NB;
    Ctrl *ctrl = reinterpret_cast<Ctrl *>(lds + OFF_CTRL);
    const int pt = (int)threadIdx.x - GT;
    const int b = blockIdx.x;
    const int R = A.rounds;
    FUSED_TRACE(pt == 0 && i < R, i, 0);
    uint32_t kept = 0;
    if (i < R) {
        uint32_t bq[PR]; // bucket | rank << 16, or ~0 (dropped)
#pragma unroll
        for (int j = 0; j < PR; ++j) {
            bq[j] = 0xFFFFFFFFu;
            if (cur.ok[j] && pred.eval(cur.pl[j])) {
                const uint32_t bk = fib_part(cur.k[j], 24);
                bq[j] = bk | (atomicAdd(&hist[bk], 1u) << 16);
            }
        }
        role_barrier(&ctrl->bar[1], gen);
        if (pt < 64) wave_scan_nb(hist, start, &ctrl->kept[i & 1], 0xFFFFFFFFu);
        role_barrier(&ctrl->bar[1], gen);
        kept = ctrl->kept[i & 1];
#pragma unroll
        for (int j = 0; j < PR; ++j) {
            if (bq[j] == 0xFFFFFFFFu) continue;
            const uint32_t s = start[bq[j] & 0xFFFFu] + (bq[j] >> 16);
            srec[s] = make_uint4((unsigned)cur.k[j], (unsigned)(cur.k[j] >> 32), (unsigned)cur.v[j],
                                 (unsigned)(cur.v[j] >> 32));
        }
        FUSED_TRACE(pt == 0, i, 1);
    }
    // round i - 1's stores are complete (every storing wave waits: R1).  Iteration i - 1 issued
    // them before the tile loads of round i + 1 (when i + 1 < R), which may stay in flight.
    if constexpr (TILE_LOADS >= 0) {
        if (i + 1 < R) wait_vm<TILE_LOADS>();
        else wait_vm<0>();
    } else {
        wait_vm<0>();
    }
    role_barrier(&ctrl->bar[1], gen);
    if (i >= 1 && pt < NB && !ctrl->stop[1]) { // publish round i - 1: the run entries are the flags
        const int ps = (i - 1) % KS;
        const uint32_t e = (round_tag(i - 1) << 24) | (pstart[pt] << 12) | phist[pt];
        __hip_atomic_store(A.ring_run + ((size_t)ps * NB + b) * NB + pt, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // round i's slot: its previous round (i - KS) must be consumed by every workgroup
    if (i < R && i >= KS && pt == 0) {
        const uint32_t target = (uint32_t)NB * (uint32_t)(i / KS);
        uint32_t *cd = A.cons_done + (size_t)(i % KS) * NSHARD * SHARD_WORDS;
        spin_until([&] {
            uint32_t s = 0;
#pragma unroll
            for (int h = 0; h < NSHARD; ++h)
                s += __hip_atomic_load(cd + h * SHARD_WORDS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return s >= target;
        }, A, &ctrl->stop[1]);
    }
    role_barrier(&ctrl->bar[1], gen);
    FUSED_TRACE(pt == 0 && i < R, i, 2);
    if (pt < NB) phist[pt] = 0; // round i + 1 counts into it (its readers passed the barrier above)
    if (i >= R) return;
    // round i's stores: a fixed count per thread (the ones past `kept` get an offset outside
    // the ring, which the buffer range check drops), so the compiler's wait counts stay exact;
    // then the tile of round i + 2 into the registers round i just emptied
    {
        const bool live = !ctrl->stop[1];
        const size_t tile_off = ((size_t)(i % KS) * NB + b) * TR * 16;
#pragma unroll
        for (int j = 0; j < TR / GT; ++j) {
            const uint32_t s = (uint32_t)(pt + j * GT);
            const uint4 r4 = srec[s];
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            v4u w;
            w[0] = r4.x;
            w[1] = r4.y;
            w[2] = r4.z;
            w[3] = r4.w;
            const int off = (live && s < kept) ? (int)(tile_off + (size_t)s * 16) : 0x7FFFFF00;
            __builtin_amdgcn_raw_buffer_store_b128(w, ring, off, 0, 16); // sc1
        }
    }
    if (i + 2 < R) load_tile<Pred, HASVAL>(pred, A, i + 2, pt, cur);
    FUSED_TRACE(pt == 0, i, 3);
}

// ---------------------------------------------------------------- consumer role (waves 0-7)
// Iteration q reads round q's run entries, issues round q's record loads (into `nrec`), then
// folds round q - 1's records (loaded an iteration ago, in `rec`) and releases its slot.
template <int SOP, bool CNT>
__device__ __forceinline__ void consume_iteration(const FArgs &A, char *lds, int q, uint32_t &tagv, uint4 (&rec)[CR],
                                                  uint4 (&nrec)[CR], unsigned &gen, const __amdgpu_buffer_rsrc_t &ring) {
    constexpr bool HASVAL = SOP != 0;
    FTable T{reinterpret_cast<uint64_t *>(lds + OFF_KEYS), reinterpret_cast<uint64_t *>(lds + OFF_ACC),
             reinterpret_cast<uint32_t *>(lds + OFF_CNT), reinterpret_cast<Ctrl *>(lds + OFF_CTRL)};
    Ctrl *ctrl = T.ctrl;
    const int ct = threadIdx.x;
    const int b = blockIdx.x;
    const int R = A.rounds;
    auto cent_of = [&](int r) { return reinterpret_cast<uint32_t *>(lds + OFF_CENT) + (r & 1) * NB; };
    auto cpref_of = [&](int r) { return reinterpret_cast<uint32_t *>(lds + OFF_CPREF) + (r & 1) * (NB + 4); };
    // record u of round r at step base -> its ring offset (0 past the end: harmless sc1 load)
    auto rec_off = [&](int r, uint32_t idx, uint32_t tot) -> uint32_t {
        if (idx >= tot) return 0u;
        const uint32_t *ce = cent_of(r), *cp = cpref_of(r);
        uint32_t lo = 0; // producer p: cp[p] <= idx < cp[p + 1]
#pragma unroll
        for (uint32_t st = NB / 2; st > 0; st >>= 1)
            if (cp[lo + st] <= idx) lo += st;
        const uint32_t s = ((ce[lo] >> 12) & 0xFFFu) + (idx - cp[lo]);
        return (uint32_t)((((size_t)(r % KS) * NB + lo) * TR + s) * 16);
    };
    FUSED_TRACE(ct == 0 && q < R, q, 4);
    if (q < R) {
        // round q's run entries (polled during the previous iteration), scan, record loads
        uint32_t *cent = cent_of(q);
        if (ct < NB) {
            const uint32_t want = round_tag(q);
            if ((tagv >> 24) != want) {
                uint32_t *ent = A.ring_run + ((size_t)(q % KS) * NB + ct) * NB + b;
                spin_until([&] {
                    tagv = __hip_atomic_load(ent, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    return (tagv >> 24) == want;
                }, A, &ctrl->stop[0]);
            }
            cent[ct] = tagv;
        }
        role_barrier(&ctrl->bar[0], gen);
        if (ct < 64) wave_scan_nb(cent, cpref_of(q), &ctrl->ctot[q & 1], ctrl->stop[0] ? 0u : 0xFFFu);
        role_barrier(&ctrl->bar[0], gen);
        const uint32_t tot = ctrl->ctot[q & 1];
#pragma unroll
        for (int u = 0; u < CR; ++u) {
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(ring, (int)rec_off(q, (uint32_t)(u * GT + ct), tot), 0, 16);
            nrec[u] = make_uint4(x[0], x[1], x[2], x[3]);
        }
        // round q + 1's run entries fly during the inserts below
        if (ct < NB && q + 1 < R)
            tagv = __hip_atomic_load(A.ring_run + ((size_t)((q + 1) % KS) * NB + ct) * NB + b, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        FUSED_TRACE(ct == 0, q, 5);
    }
    if (q >= 1) { // fold round q - 1
        const int r = q - 1;
        const uint32_t tot = ctrl->ctot[r & 1];
        uint64_t kk[CR], vv[CR];
        bool miss[CR];
        for (uint32_t base = 0; base < tot; base += GT * CR) {
            uint4 cur[CR];
            if (base == 0) {
#pragma unroll
                for (int u = 0; u < CR; ++u) cur[u] = rec[u];
            } else { // rare: more than GT * CR records of one bucket in one round
#pragma unroll
                for (int u = 0; u < CR; ++u) {
                    const auto x = __builtin_amdgcn_raw_buffer_load_b128(ring, (int)rec_off(r, base + (uint32_t)(u * GT + ct), tot), 0, 16);
                    cur[u] = make_uint4(x[0], x[1], x[2], x[3]);
                }
            }
            bool rok[CR];
            int cell[CR];
#pragma unroll
            for (int u = 0; u < CR; ++u) {
                rok[u] = base + (uint32_t)(u * GT + ct) < tot;
                kk[u] = ((uint64_t)cur[u].y << 32) | cur[u].x;
                vv[u] = ((uint64_t)cur[u].w << 32) | cur[u].z;
            }
            T.find_multi<CR>(kk, rok, true, cell);
#pragma unroll
            for (int u = 0; u < CR; ++u) {
                miss[u] = rok[u] && cell[u] < 0;
                if (rok[u] && cell[u] >= 0) fold<SOP, CNT>(T, cell[u], vv[u]);
            }
            if (base + GT * CR < tot) { // more steps: retry this step's misses now
                role_barrier(&ctrl->bar[0], gen);
#pragma unroll
                for (int u = 0; u < CR; ++u) {
                    if (!miss[u]) continue;
                    miss[u] = false;
                    const uint64_t k1[1] = {kk[u]};
                    const bool v1[1] = {true};
                    int c1[1];
                    T.find_multi<1>(k1, v1, false, c1);
                    if (c1[0] >= 0) {
                        fold<SOP, CNT>(T, c1[0], vv[u]);
                    } else {
                        const unsigned long long pos = atomicAdd(&A.cursor[0], 1ull);
                        if (pos < (unsigned long long)A.n) {
                            A.io.spill_key[pos] = kk[u];
                            if constexpr (HASVAL) A.io.spill_val[pos] = vv[u];
                        }
                    }
                }
            }
        }
        if (tot == 0)
#pragma unroll
            for (int u = 0; u < CR; ++u) miss[u] = false;
        // every insert of round r is done and its records are in registers: release the slot,
        // then retry the misses (a miss now means "table full")
        role_barrier(&ctrl->bar[0], gen);
        if (ct == 0)
            __hip_atomic_fetch_add(A.cons_done + (size_t)(r % KS) * NSHARD * SHARD_WORDS + (b % NSHARD) * SHARD_WORDS,
                                   1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int u = 0; u < CR; ++u) {
            if (!miss[u]) continue;
            const uint64_t k1[1] = {kk[u]};
            const bool v1[1] = {true};
            int c1[1];
            T.find_multi<1>(k1, v1, false, c1);
            if (c1[0] >= 0) {
                fold<SOP, CNT>(T, c1[0], vv[u]);
            } else {
                const unsigned long long pos = atomicAdd(&A.cursor[0], 1ull);
                if (pos < (unsigned long long)A.n) { // never past the spill arrays (n rows)
                    A.io.spill_key[pos] = kk[u];
                    if constexpr (HASVAL) A.io.spill_val[pos] = vv[u];
                }
            }
        }
        FUSED_TRACE(ct == 0, r, 6);
    }
}

// SOP: 2 sum into Int64 / UInt64, 3 sum Float64; CNT: a count state
template <typename Pred, int SOP, bool CNT>
__global__ void __launch_bounds__(FT, 1) agg_fused_kernel(Pred pred, FArgs A) {
    constexpr bool HASVAL = SOP != 0;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    FTable T{reinterpret_cast<uint64_t *>(lds + OFF_KEYS), reinterpret_cast<uint64_t *>(lds + OFF_ACC),
             reinterpret_cast<uint32_t *>(lds + OFF_CNT), reinterpret_cast<Ctrl *>(lds + OFF_CTRL)};
    Ctrl *ctrl = T.ctrl;
    const int b = blockIdx.x;
    const int t = threadIdx.x;
    const int R = A.rounds;
    const __amdgpu_buffer_rsrc_t ring = __builtin_amdgcn_make_buffer_rsrc(A.ring_rec, 0, (int)RING_REC_BYTES, 0x00020000);
    for (int c = t; c < CAP + 2; c += FT) {
        T.keys[c] = 0;
        T.acc[c] = 0;
        T.cnt[c] = 0;
    }
    for (int c = t; c < 2 * NB; c += FT) reinterpret_cast<uint32_t *>(lds + OFF_HIST)[c] = 0;
    if (t == 0) {
        ctrl->used = ctrl->full = ctrl->zero_used = 0;
        ctrl->stop[0] = ctrl->stop[1] = ctrl->bar[0] = ctrl->bar[1] = 0;
        ctrl->out_count = 0;
    }
    __syncthreads();
    unsigned gen = 0;
    if (t >= GT) { // producer role: two tiles in flight
        const int pt = t - GT;
        TileRegs<Pred> ta, tb;
        if (R > 0) load_tile<Pred, HASVAL>(pred, A, 0, pt, ta);
        if (R > 1) load_tile<Pred, HASVAL>(pred, A, 1, pt, tb);
        for (int i = 0; i <= R; i += 2) {
            if (ctrl->stop[1]) break; // uniform: written only before a producer barrier
            produce_iteration<Pred, SOP>(pred, A, lds, i, ta, gen, ring);
            if (i + 1 <= R && !ctrl->stop[1]) produce_iteration<Pred, SOP>(pred, A, lds, i + 1, tb, gen, ring);
        }
    } else { // consumer role: records of two rounds in flight
        uint32_t tagv = 0;
        if (t < NB && R > 0)
            tagv = __hip_atomic_load(A.ring_run + (size_t)t * NB + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint4 ra[CR], rb[CR];
        for (int q = 0; q <= R; q += 2) {
            if (ctrl->stop[0]) break; // uniform: written only before a consumer barrier
            consume_iteration<SOP, CNT>(A, lds, q, tagv, rb, ra, gen, ring);
            if (q + 1 <= R && !ctrl->stop[0]) consume_iteration<SOP, CNT>(A, lds, q + 1, tagv, ra, rb, gen, ring);
        }
    }
    __syncthreads();
    // ---- flush the table: groups of bucket b at a region reserved from the global cursor
    if (t == 0) {
        const unsigned long long g = (unsigned long long)ctrl->used + ctrl->zero_used;
        ctrl->out_base = atomicAdd(&A.cursor[1], g);
        A.io.out_cnt[b] = g;
        A.io.tmp_base[b] = ctrl->out_base;
    }
    __syncthreads();
    const unsigned long long ob = ctrl->out_base;
    for (int c = t; c <= CAP; c += FT) {
        const bool occ = c < CAP ? T.keys[c] != 0 : ctrl->zero_used != 0;
        if (!occ) continue;
        const unsigned long long pos = ob + atomicAdd(&ctrl->out_count, 1ull);
        A.io.tmp_key[pos] = c < CAP ? T.keys[c] : 0ull;
        A.io.tmp_key_null[pos] = 0;
        if constexpr (SOP != 0) A.io.tmp_sum[pos] = T.acc[c];
        if constexpr (CNT) A.io.tmp_cnt[pos] = T.cnt[c];
    }
}

template <typename Pred, int SOP, bool CNT>
int launch_fused(Ctx *ctx, const Pred &pred, FArgs &A, bool &launched) {
    auto kern = agg_fused_kernel<Pred, SOP, CNT>;
    static int ok = -1; // per instantiation: can one workgroup per CU be resident?
    if (ok < 0) {
        int nb = 0;
        ok = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, FT, LDS_BYTES) == hipSuccess && nb >= 1;
    }
    if (!ok) return TFG_OK;
    Pred p = pred;
    void *args[] = {(void *)&p, (void *)&A};
    hipError_t e = hipLaunchCooperativeKernel((const void *)kern, dim3(NB), dim3(FT), args, LDS_BYTES, ctx->stream);
    if (e == hipErrorCooperativeLaunchTooLarge) {
        (void)hipGetLastError();
        return TFG_OK; // not co-resident on this device: the caller takes the two-kernel path
    }
    TFG_HIP(e);
    launched = true;
    return TFG_OK;
}

} // namespace

size_t fused_scratch_bytes() { return RING_REC_BYTES + RING_RUN_BYTES + CONS_BYTES + CTL_BYTES; }

int agg_fused_consume(Ctx *ctx, int code, const RowPred &pred, const void *keys, const void *vals, int64_t n,
                      const FusedIO &io, void *scratch, uint64_t *spill_count_host, bool &launched) {
    launched = false;
    *spill_count_host = 0;
    int sop = -1;
    switch (code) {
    case 310: case 130: sop = 3; break;
    case 210: case 120: sop = 2; break;
    default: return TFG_OK; // every fused signature has one sum and a count state
    }
    if (n < FUSED_MIN_ROWS || ctx->cu_count < NB) return TFG_OK;
    const int64_t rounds = (n + (int64_t)NB * TR - 1) / ((int64_t)NB * TR);
    FArgs A{};
    A.key = (const uint64_t *)keys;
    A.val = (const uint64_t *)vals;
    A.n = n;
    A.rounds = (int)rounds;
    char *s = (char *)scratch;
    A.ring_rec = (uint4 *)s;
    char *zero = s + RING_REC_BYTES; // run entries, release counters, error word, cursors: zeroed
    A.ring_run = (uint32_t *)zero;
    A.cons_done = (uint32_t *)(zero + RING_RUN_BYTES);
    A.err = (uint32_t *)(zero + RING_RUN_BYTES + CONS_BYTES);
    A.cursor = (unsigned long long *)(zero + RING_RUN_BYTES + CONS_BYTES + 16);
    A.io = io;
    TFG_HIP(hipMemsetAsync(zero, 0, RING_RUN_BYTES + CONS_BYTES + CTL_BYTES, ctx->stream));
    {
        ProfScope _ps(ctx, "agg.fused");
        if (int rc = with_pred(pred, [&](auto pr) -> int {
                using PR = decltype(pr);
                return sop == 3 ? launch_fused<PR, 3, true>(ctx, pr, A, launched)
                                : launch_fused<PR, 2, true>(ctx, pr, A, launched);
            }))
            return rc;
    }
    if (!launched) return TFG_OK;
    uint64_t w[4] = {};
    if (int rc = read_back_u64(ctx, (const uint64_t *)A.err, w, 4)) return rc; // err word, pad, cursors
    TFG_CHECK((w[0] & 0xFFFFFFFFull) == 0, TFG_ERR_LOGICAL,
              "fused aggregation: a workgroup timed out waiting for its peers (not co-resident?)");
    *spill_count_host = w[2];
    return TFG_OK;
}

} // namespace tfg
