// agg_dev.h — device side of the hash GROUP BY (agg.hip): the group state layout, the LDS hash
// table, the row policies and the two bucket kernels.  Kept in a header so the bucket kernels of
// each row-policy family are instantiated in translation units of their own (agg_bucket_*.hip),
// which hipcc builds in parallel.
#pragma once
#include <algorithm>
#include <vector>

#include "common.h"
#include "partition.h"

namespace tfg {

constexpr int AGG_MAX = 4;
constexpr int BT = 512;      // bucket kernel threads (8 waves; 2-3 workgroups per CU)
constexpr int BT_BIG = 1024; // for tables too large for two workgroups per CU (16 waves)
constexpr int BT_QUAD = 256; // wide tiled tables of a quarter CU (four workgroups per CU)
constexpr int LDS_TABLE_BYTES = 100 * 1024;  // preferred table size (two workgroups per CU)
constexpr int LDS_TABLE_MAX = 150 * 1024;    // largest table (one 16-wave workgroup per CU)
constexpr int LDS_CU_BYTES = 160 * 1024;     // gfx950 LDS per CU
constexpr int BUCKET_STATIC_LDS_MAX = 13 * 1024; // upper bound of the bucket kernels' static LDS

enum AccKind { ACC_NONE = 0, ACC_I64 = 1, ACC_F64 = 2, ACC_I128 = 3, ACC_I256 = 4, ACC_ORD = 5, ACC_REF = 6 };
// 64-bit words of an accumulator of kind k
__host__ __device__ constexpr int acc_words(int k) { return k == ACC_I256 ? 4 : k == ACC_I128 ? 2 : k == ACC_NONE ? 0 : 1; }
// ... and in an LDS table: a Decimal256 sum carries a fifth limb there, the sign extension of
// the exact sum, so a sum past Int256 is detected when the table is flushed (lds_add_i256)
__host__ __device__ constexpr int lds_acc_words(int k) { return k == ACC_I256 ? 5 : acc_words(k); }
enum RowMode { MODE_RAW = 0, MODE_PARTIAL = 1, MODE_STATE = 2 };

// Row-reference aggregates (ACC_REF: first_row of any type, min / max of Decimal128 / Decimal256 /
// String).  The state of a group is a u64 reference to one candidate value, 0 = no value yet.
// The candidates of one consume are the aggregator's value store (one entry per group of the
// previous state: refs 1 .. n0) followed by the consumed column (row r: ref n0 + 1 + r; a merge:
// the source aggregator's store).  References order candidates in input order, so "first row" is
// the smallest reference and equal min / max values keep the smallest one (the reference's strict
// changeIfLess / changeIfGreater / changeFirstTime).  After the consume the winning values are
// copied into a new store in group order (agg.hip, ref_materialise) and every state becomes g + 1.
struct RefSrc {
    const uint8_t *v[2];  // [0] store, [1] consumed column: fixed-width values, or String compare bytes
    const uint64_t *o[2]; // String compare bytes: end offsets (row i = [o[i - 1], o[i]) with o[-1] = 0)
    uint64_t n0;          // store entries
    uint64_t n1;          // consumed rows (references n0 + 1 .. n0 + n1)
    uint64_t nb[2];       // String compare bytes: bytes of v[i] when known (~0 otherwise)
    int width;            // fixed: 16 / 32 (signed little-endian limbs compared); 0 = String bytes
    unsigned *err;        // |= 2 on a reference outside 1 .. n0 + n1 or a row without its '\0', |= 4 on
                          // a row's bytes past nb (never dereferenced; the call then fails with
                          // TFG_ERR_LOGICAL)
};

struct AggSpec {
    int key_width; // bytes of the key column (1,2,4,8); 0 = without key
    int n_aggs;
    int kind[AGG_MAX];
    int acc[AGG_MAX];     // AccKind (SUM only)
    int has_cnt[AGG_MAX]; // count slot present
    int src_type[AGG_MAX];
    // LDS layout (byte offsets into dynamic LDS)
    int cap;      // table cells (power of two); slots cap (key 0) and cap+1 (NULL key) follow
    int maxfill;  // sticky "full" threshold
    int acc_off[AGG_MAX];
    int cnt_off[AGG_MAX];
    int ctrl_off;
    int lds_bytes;
    int bt;         // bucket kernel workgroup size (BT or BT_BIG)
    int wkey_off;   // wide keys (key_width 16): LDS byte offset of the 16-byte keys (cells' tags sit in
                    // the u64 key array); 0 for keys of <= 8 bytes
    unsigned *ovf;      // Decimal256 sums: set to 1 when a sum leaves Int256 (TFG_ERR_OVERFLOW); null otherwise
    int bbits;          // bucket radix bits: the in-table slot group comes from the 32 bits of
                        // key * 2^64/phi just below them (one multiply instead of a mixer) ...
    unsigned ngroups;   // ... scaled to the table's cap / GS groups (any count: LDS-sized tables)
    RefSrc ref[AGG_MAX]; // ACC_REF aggregates: this call's candidates
};

// Columnar row source staged by the bucket pass (bucket-major).
struct RowsIO {
    int key_width;                // bytes per key (raw key width, or 8 for STATE rows)
    void *key;                    // key_width bytes per row
    uint8_t *key_null;            // optional
    void *val[AGG_MAX];           // RAW: arg type; PARTIAL: result type; STATE: acc
    uint8_t *val_null[AGG_MAX];   // RAW / PARTIAL: optional null flags
    uint64_t *val_cnt[AGG_MAX];   // STATE: counts
};

// Columnar groups (state / temp).
struct GroupsIO {
    uint64_t *key; // key bits; wide keys: two words (lo, hi) per group
    uint8_t *key_null;
    void *acc[AGG_MAX];
    uint64_t *cnt[AGG_MAX];
};

struct Ctrl {
    unsigned used;
    unsigned full;
    unsigned zero_used;
    unsigned null_used;
    unsigned long long out_count;
    unsigned long long spill_w;
};


__device__ __forceinline__ uint64_t load_bits(const void *p, int width, int64_t i) {
    switch (width) {
    case 1: return ((const uint8_t *)p)[i];
    case 2: return ((const uint16_t *)p)[i];
    case 4: return ((const uint32_t *)p)[i];
    default: return ((const uint64_t *)p)[i];
    }
}

// value of a SUM argument widened to the accumulator
__device__ __forceinline__ void load_sum_value(int type, const void *p, int64_t i, uint64_t &lo, uint64_t &hi, double &f) {
    switch (type) {
    case TFG_INT8: lo = (uint64_t)(int64_t)((const int8_t *)p)[i]; break;
    case TFG_INT16: lo = (uint64_t)(int64_t)((const int16_t *)p)[i]; break;
    case TFG_INT32: case TFG_DECIMAL32: lo = (uint64_t)(int64_t)((const int32_t *)p)[i]; break;
    case TFG_INT64: case TFG_DECIMAL64: lo = ((const uint64_t *)p)[i]; break;
    case TFG_UINT8: lo = ((const uint8_t *)p)[i]; hi = 0; return;
    case TFG_UINT16: lo = ((const uint16_t *)p)[i]; hi = 0; return;
    case TFG_UINT32: lo = ((const uint32_t *)p)[i]; hi = 0; return;
    case TFG_UINT64: lo = ((const uint64_t *)p)[i]; hi = 0; return;
    case TFG_FLOAT32: f = ((const float *)p)[i]; return;
    case TFG_FLOAT64: f = ((const double *)p)[i]; return;
    case TFG_DECIMAL128: lo = ((const uint64_t *)p)[2 * i]; hi = ((const uint64_t *)p)[2 * i + 1]; return;
    default: lo = 0; break;
    }
    hi = (int64_t)lo < 0 ? ~0ull : 0ull; // sign extension into Int128
}

// min / max / first_row (ACC_ORD): the state is one u64 "order key" combined by unsigned max
// (ds_max_u64 / atomicMax), identity 0 — so a zeroed cell is an empty state and partial states merge
// by the same max.  ord_base maps a value to a u64 in the value's order (signed: flip the sign bit;
// floats: IEEE total order, Float32 widened exactly to Float64); max keeps it, min keeps its
// complement, first_row keeps the max (any row of the group is a valid first row).
__host__ __device__ __forceinline__ uint64_t ord_base(int type, uint64_t bits) {
    switch (type) {
    case TFG_INT8: return (uint64_t)(int64_t)(int8_t)bits ^ 0x8000000000000000ull;
    case TFG_INT16: return (uint64_t)(int64_t)(int16_t)bits ^ 0x8000000000000000ull;
    case TFG_INT32: case TFG_DECIMAL32: return (uint64_t)(int64_t)(int32_t)bits ^ 0x8000000000000000ull;
    case TFG_INT64: case TFG_DECIMAL64: return bits ^ 0x8000000000000000ull;
    case TFG_FLOAT32: case TFG_FLOAT64: {
        uint64_t b = bits;
        if (type == TFG_FLOAT32) {
            float f;
            uint32_t u = (uint32_t)bits;
            memcpy(&f, &u, 4);
            const double d = (double)f;
            memcpy(&b, &d, 8);
        }
        return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
    }
    default: return bits; // unsigned: zero-extended
    }
}
__host__ __device__ __forceinline__ uint64_t ord_unbase(int type, uint64_t k) {
    switch (type) {
    case TFG_INT8: case TFG_INT16: case TFG_INT32: case TFG_DECIMAL32: case TFG_INT64: case TFG_DECIMAL64:
        return k ^ 0x8000000000000000ull; // sign-extended; the caller stores the type's width
    case TFG_FLOAT32: case TFG_FLOAT64: {
        const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
        if (type == TFG_FLOAT64) return b;
        double d;
        memcpy(&d, &b, 8);
        const float f = (float)d; // exact: the value was a Float32
        uint32_t u;
        memcpy(&u, &f, 4);
        return u;
    }
    default: return k;
    }
}
__host__ __device__ __forceinline__ uint64_t ord_enc(int kind, int type, uint64_t bits) {
    const uint64_t b = ord_base(type, bits);
    return kind == TFG_AGG_MIN ? ~b : b;
}
__host__ __device__ __forceinline__ uint64_t ord_dec(int kind, int type, uint64_t k) {
    return ord_unbase(type, kind == TFG_AGG_MIN ? ~k : k);
}

// three-way compare of candidates a, b (>= 1) of a RefSrc: signed limbs, or bytes then length
// (memcmp order of the compare bytes: raw rows, or collator sort keys)
__device__ __forceinline__ int ref_cmp(const RefSrc &R, uint64_t a, uint64_t b) {
    if (a - 1 >= R.n0 + R.n1 || b - 1 >= R.n0 + R.n1) { // 0 wraps: out of range too
        if (R.err) atomicOr(R.err, 2u);
        return 0;
    }
    const int sa = a > R.n0, sb = b > R.n0;
    const uint64_t ia = sa ? a - R.n0 - 1 : a - 1, ib = sb ? b - R.n0 - 1 : b - 1;
    if (R.width) {
        const int nw = R.width >> 3;
        const uint64_t *pa = reinterpret_cast<const uint64_t *>(R.v[sa]) + ia * nw;
        const uint64_t *pb = reinterpret_cast<const uint64_t *>(R.v[sb]) + ib * nw;
        const int64_t ha = (int64_t)pa[nw - 1], hb = (int64_t)pb[nw - 1];
        if (ha != hb) return ha < hb ? -1 : 1;
        for (int k = nw - 2; k >= 0; --k)
            if (pa[k] != pb[k]) return pa[k] < pb[k] ? -1 : 1;
        return 0;
    }
    const uint64_t a0 = ia ? R.o[sa][ia - 1] : 0, a1 = R.o[sa][ia] - 1; // the row's '\0' excluded:
    const uint64_t b0 = ib ? R.o[sb][ib - 1] : 0, b1 = R.o[sb][ib] - 1; // both rows end with it
    if (a1 + 1 <= a0 || b1 + 1 <= b0) { // a row of no bytes (no '\0'): malformed offsets
        if (R.err) atomicOr(R.err, 2u);
        return 0;
    }
    if (a1 >= R.nb[sa] || b1 >= R.nb[sb]) { // a row past its buffer's bytes
        const unsigned was = R.err ? atomicOr(R.err, 4u) : 4u;
#ifdef TFG_EXP_POOL
        if (!(was & 4u))
            printf("EXP ref_cmp bound: a=%llu b=%llu n0=%llu n1=%llu a0=%llu a1=%llu nb=%llu b0=%llu b1=%llu nb=%llu "
               "v=%p %p o=%p %p\n",
               (unsigned long long)a, (unsigned long long)b, (unsigned long long)R.n0, (unsigned long long)R.n1,
               (unsigned long long)a0, (unsigned long long)a1, (unsigned long long)R.nb[sa], (unsigned long long)b0,
               (unsigned long long)b1, (unsigned long long)R.nb[sb], R.v[0], R.v[1], R.o[0], R.o[1]);
#else
        (void)was;
#endif
        return 0;
    }
    const uint8_t *pa = R.v[sa] + a0, *pb = R.v[sb] + b0;
    const uint64_t la = a1 - a0, lb = b1 - b0, m = la < lb ? la : lb;
    for (uint64_t k = 0; k < m; ++k)
        if (pa[k] != pb[k]) return pa[k] < pb[k] ? -1 : 1;
    return la < lb ? -1 : la > lb ? 1 : 0;
}
// does candidate a replace the state b (0 = empty)?
__device__ __forceinline__ bool ref_better(int kind, const RefSrc &R, uint64_t a, uint64_t b) {
    if (b == 0) return true;
    if (kind == TFG_AGG_FIRST_ROW) return a < b;
    int c = ref_cmp(R, a, b);
    if (kind == TFG_AGG_MIN) c = -c;
    return c > 0 || (c == 0 && a < b);
}
// lock-free fold of candidate `mine` into a u64 state cell (LDS or global): every CAS attempt is
// independent, so lanes of one wave contending for a cell never wait on each other
__device__ __forceinline__ void ref_combine(uint64_t *cell, uint64_t mine, const RefSrc &R, int kind) {
    if (mine == 0) return;
    uint64_t cur = __hip_atomic_load(cell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (ref_better(kind, R, mine, cur)) {
        const uint64_t prev = atomicCAS((unsigned long long *)cell, (unsigned long long)cur, (unsigned long long)mine);
        if (prev == cur) return;
        cur = prev;
    }
}

__device__ __forceinline__ void lds_add_i128(uint64_t *cell, uint64_t lo, uint64_t hi) {
    const uint64_t old = atomicAdd((unsigned long long *)&cell[0], (unsigned long long)lo);
    const uint64_t carry = (old + lo) < old ? 1ull : 0ull;
    if (hi + carry) atomicAdd((unsigned long long *)&cell[1], (unsigned long long)(hi + carry)); // 0: nothing to add
}

// Decimal256 sum state (AggregateFunctionSumData<Decimal256>, boost checked_int256_t): four
// 64-bit limbs added limb by limb with LDS atomics, plus a fifth that receives the addend's sign
// extension and the carry out of limb 3.  Every adder carries its own carry-outs into the next
// limb (a carry from x_k + c_k itself, or from the atomic add), so the five limbs end at the
// exact sum whatever the interleaving of concurrent adders: it fits Int256 iff limb 4 is the
// sign extension of limb 3 (checked_int256_t throws past that: types.h:35; checked at flush).
__device__ __forceinline__ void lds_add_i256(uint64_t *cell, uint64_t x0, uint64_t x1, uint64_t x2, uint64_t x3) {
    uint64_t old = atomicAdd((unsigned long long *)&cell[0], (unsigned long long)x0);
    uint64_t c = (old + x0) < old ? 1ull : 0ull;
    uint64_t t = x1 + c;
    uint64_t ca = t < c ? 1ull : 0ull;
    old = atomicAdd((unsigned long long *)&cell[1], (unsigned long long)t);
    c = ((old + t) < old ? 1ull : 0ull) + ca;
    t = x2 + c;
    ca = t < c ? 1ull : 0ull;
    old = atomicAdd((unsigned long long *)&cell[2], (unsigned long long)t);
    c = ((old + t) < old ? 1ull : 0ull) + ca;
    t = x3 + c;
    ca = t < c ? 1ull : 0ull;
    old = atomicAdd((unsigned long long *)&cell[3], (unsigned long long)t);
    c = ((old + t) < old ? 1ull : 0ull) + ca;
    atomicAdd((unsigned long long *)&cell[4], (unsigned long long)(((int64_t)x3 < 0 ? ~0ull : 0ull) + c));
}

// five-limb register form (a[0..4] += x[0..3] sign-extended); fits Int256 iff a[4] == sign(a[3])
__host__ __device__ __forceinline__ void add_i320(uint64_t *a, const uint64_t *x) {
    uint64_t c = 0;
    for (int k = 0; k < 5; ++k) {
        const uint64_t xk = k < 4 ? x[k] : ((int64_t)x[3] < 0 ? ~0ull : 0ull);
        const uint64_t t = xk + c;
        const uint64_t c1 = t < c ? 1ull : 0ull;
        const uint64_t s = a[k] + t;
        c = (s < t ? 1ull : 0ull) + c1;
        a[k] = s;
    }
}
__host__ __device__ __forceinline__ bool fits_i256(const uint64_t *a5) {
    return a5[4] == ((int64_t)a5[3] < 0 ? ~0ull : 0ull);
}

// register form: a += x (mod 2^256)
__host__ __device__ __forceinline__ void add_i256(uint64_t *a, const uint64_t *x) {
    uint64_t c = 0;
    for (int k = 0; k < 4; ++k) {
        const uint64_t t = x[k] + c;
        const uint64_t c1 = t < c ? 1ull : 0ull;
        const uint64_t s = a[k] + t;
        c = (s < t ? 1ull : 0ull) + c1;
        a[k] = s;
    }
}

// Tag of a wide (16-byte packed) key: a 64-bit mix of both halves with bit 1 set (never 0) and
// bit 0 clear.  The bucket radix and the in-table slot group come from tag * 2^64/phi exactly
// as they come from the key itself for 8-byte keys; bit 0 of a stored tag marks "key published".
__host__ __device__ __forceinline__ uint64_t wide_tag(uint64_t lo, uint64_t hi) {
    uint64_t x = lo * 0x9E3779B97F4A7C15ull ^ hi;
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    return (x | 2ull) & ~1ull;
}

// one staged row held in registers; NA = number of aggregates (compile time, keeps VGPRs low);
// W: the signature has a Decimal256 sum, whose values carry two more limbs (x2, x3)
template <int NA, bool W> struct RowHi {
    uint64_t x2[NA], x3[NA];
};
template <int NA> struct RowHi<NA, false> {};
template <int NA, bool W = false> struct RowValT : RowHi<NA, W> {
    uint64_t key;
    uint8_t knull;
    uint8_t vnull[NA];
    uint64_t lo[NA], hi[NA], cnt[NA];
};

// raw argument bits of a RAW row widened to the integer accumulator (sign / zero extension)
__device__ __forceinline__ void widen_raw(int type, uint64_t &lo, uint64_t &hi) {
    switch (type) {
    case TFG_INT8: lo = (uint64_t)(int64_t)(int8_t)lo; break;
    case TFG_INT16: lo = (uint64_t)(int64_t)(int16_t)lo; break;
    case TFG_INT32: case TFG_DECIMAL32: lo = (uint64_t)(int64_t)(int32_t)lo; break;
    case TFG_INT64: case TFG_DECIMAL64: break;
    case TFG_DECIMAL128: return;
    default: hi = 0; return; // unsigned: zero-extended already
    }
    hi = (int64_t)lo < 0 ? ~0ull : 0ull;
}

struct Table {
    uint64_t *keys;
    char *base;
    Ctrl *ctrl;
    const AggSpec &S;
    __device__ Table(char *lds, const AggSpec &s)
        : keys(reinterpret_cast<uint64_t *>(lds)), base(lds), ctrl(reinterpret_cast<Ctrl *>(lds + s.ctrl_off)), S(s) {}

    __device__ void clear() {
        uint32_t *w = reinterpret_cast<uint32_t *>(base);
        const int words = S.ctrl_off / 4;
        for (int i = threadIdx.x; i < words; i += blockDim.x) w[i] = 0;
        if (threadIdx.x == 0) {
            ctrl->used = ctrl->full = ctrl->zero_used = ctrl->null_used = 0;
            ctrl->spill_w = 0;
        }
    }

    // returns the cell of `key`, inserting it when allowed; -1 = not in the table
    __device__ __forceinline__ int find_or_insert(uint64_t key, bool is_null, bool may_insert, bool force) {
        // side slots (ZeroValueStorage for key 0, and the NULL key) obey the same insert rule as
        // table cells: while older groups are pending (may_insert == false) a key that is not in
        // the table yet must be deferred, or it would be emitted twice
        if (is_null || key == 0) {
            unsigned *used = is_null ? &ctrl->null_used : &ctrl->zero_used;
            if (!__hip_atomic_load(used, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                if (!may_insert) return -1;
                __hip_atomic_store(used, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            return is_null ? S.cap + 1 : S.cap;
        }
        uint64_t k1[1] = {key};
        bool n1[1] = {false}, v1[1] = {true};
        int c1[1];
        find_or_insert_multi<1>(k1, n1, v1, may_insert, c1, force);
        return c1[0];
    }

    // One probe step reads a group of GS = 4 consecutive cells (two ds_read_b128) and compares
    // them all: groups of 4 at fill <= 5/8 rarely overflow, so almost every lookup finishes in
    // one step (single-cell linear probing had long worst-case chains, and a wave waits for its
    // slowest lane).  Groups overflow linearly into the next group.
    static constexpr int GS = 4;
    __device__ __forceinline__ unsigned slot_group(uint64_t key) const {
        const uint32_t below = (uint32_t)(((key * 0x9E3779B97F4A7C15ull) << S.bbits) >> 32);
        return (unsigned)(((uint64_t)below * S.ngroups) >> 32);
    }
    // A new key first reserves one of the maxfill cells (ctrl->used counts reservations, so
    // concurrent inserts can never fill the table past maxfill: no headroom for in-flight
    // inserts is needed), then claims its empty cell by CAS; a lost race returns the reservation.
    __device__ __forceinline__ bool reserve(bool force) {
        const unsigned n = atomicAdd(&ctrl->used, 1u);
        if (force || n < (unsigned)S.maxfill) return true;
        ctrl->full = 1;
        atomicSub(&ctrl->used, 1u);
        return false;
    }
    __device__ __forceinline__ int try_claim(int cell, uint64_t key, bool force, bool &done) {
        // returns the cell when `key` now owns it, -1 otherwise (done = a definitive miss)
        if (!force && __hip_atomic_load(&ctrl->full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            done = true;
            return -1;
        }
        if (!reserve(force)) {
            done = true;
            return -1;
        }
        const uint64_t old = atomicCAS((unsigned long long *)&keys[cell], 0ull, (unsigned long long)key);
        if (old == 0) {
            done = true;
            return cell;
        }
        atomicSub(&ctrl->used, 1u);
        if (old == key) {
            done = true;
            return cell;
        }
        return -1; // lost the race to another key: re-read the group
    }

    // find_or_insert for R rows at once with their probe sequences interleaved: every round
    // issues the LDS reads of all still-probing rows back to back, so R dependent LDS-latency
    // chains overlap instead of running one after the other (a wave waits for its longest chain).
    template <int R>
    __device__ __forceinline__ void find_or_insert_multi(const uint64_t (&key)[R], const bool (&is_null)[R],
                                                         const bool (&valid)[R], bool may_insert, int (&cell)[R],
                                                         bool force = false) {
        const unsigned ng = S.ngroups;
        unsigned grp[R];
        bool live[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            cell[u] = -1;
            live[u] = false;
            if (!valid[u]) continue;
            if (is_null[u] || key[u] == 0) {
                cell[u] = find_or_insert(key[u], is_null[u], may_insert, force);
                continue;
            }
            grp[u] = slot_group(key[u]);
            live[u] = true;
        }
        for (int step = 0; step < (int)ng; ++step) {
            uint64_t k[R][GS];
#pragma unroll
            for (int u = 0; u < R; ++u) // every live row's group read before any compare
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
                if (hit >= 0 && (empty < 0 || hit < empty)) { // found before the first empty cell
                    cell[u] = (int)(grp[u] * GS + hit);
                    live[u] = false;
                } else if (empty >= 0) {
                    if (!may_insert) {
                        live[u] = false; // miss
                        continue;
                    }
                    bool done = false;
                    const int c = try_claim((int)(grp[u] * GS + empty), key[u], force, done);
                    if (done) {
                        cell[u] = c;
                        live[u] = false;
                    } else {
                        any = true; // raced: re-read this group
                    }
                } else {
                    grp[u] = grp[u] + 1 == ng ? 0 : grp[u] + 1; // full group: overflow into the next
                    any = true;
                }
            }
            if (!any) break;
        }
    }

    // Home-group lookup of R keys at once, branch-free: cell[u] = the key's cell when it sits in
    // its home group — the common case once a bucket's groups exist (cells of a group fill in
    // order and are never freed, so a match anywhere in the group is the key's cell) — else -1
    // (key 0, a key in an overflow group, a key not inserted yet): the caller's slow path.
    template <int R>
    __device__ __forceinline__ void find_home(const uint64_t (&key)[R], int (&cell)[R]) const {
        unsigned grp[R];
        uint64_t k[R][GS];
#pragma unroll
        for (int u = 0; u < R; ++u) grp[u] = slot_group(key[u]);
#pragma unroll
        for (int u = 0; u < R; ++u) { // every row's group read before any compare
            const uint4 a = *reinterpret_cast<const uint4 *>(&keys[grp[u] * GS]);
            const uint4 b = *reinterpret_cast<const uint4 *>(&keys[grp[u] * GS + 2]);
            k[u][0] = ((uint64_t)a.y << 32) | a.x;
            k[u][1] = ((uint64_t)a.w << 32) | a.z;
            k[u][2] = ((uint64_t)b.y << 32) | b.x;
            k[u][3] = ((uint64_t)b.w << 32) | b.z;
        }
#pragma unroll
        for (int u = 0; u < R; ++u) {
            int c = -1;
#pragma unroll
            for (int s = GS - 1; s >= 0; --s) c = k[u][s] == key[u] ? s : c;
            cell[u] = (c >= 0 && key[u] != 0) ? (int)(grp[u] * GS) + c : -1;
        }
    }

    // Wide keys (keys128 / packed String keys).  A cell is claimed by a 64-bit CAS of the key's
    // tag into keys[cell]; the claimant then writes the 16-byte key to wkeys[cell] and
    // republishes the tag with bit 0 set.  A reader whose tag equals a cell's unpublished tag
    // re-reads the group (the claimant never waits on anything, so the wait is short); equal
    // published tags are confirmed by comparing the full key, so tag collisions only cost a
    // probe step.  Every key has exactly one cell: a key cannot be claimed behind an unresolved
    // cell of the same tag.
    template <int R>
    __device__ __forceinline__ void find_wide_multi(const uint64_t (&lo)[R], const uint64_t (&hi)[R],
                                                    const uint64_t (&tag)[R], const bool (&valid)[R], bool may_insert,
                                                    int (&cell)[R], bool force = false) {
        const unsigned ng = S.ngroups;
        uint4 *wk = reinterpret_cast<uint4 *>(base + S.wkey_off);
        unsigned grp[R];
        bool live[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            cell[u] = -1;
            live[u] = valid[u];
            grp[u] = slot_group(tag[u]);
        }
        for (;;) {
            uint64_t k[R][GS];
            // the tags are read with relaxed atomic loads: other waves CAS and publish them
            // concurrently, and every round must see their current values
#pragma unroll
            for (int u = 0; u < R; ++u)
                if (live[u])
#pragma unroll
                    for (int s = 0; s < GS; ++s)
                        k[u][s] = __hip_atomic_load(&keys[grp[u] * GS + s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            // the group's slots as masks: empty, published same tag, unpublished same tag.  Only
            // slots before the first empty one count; the first published same-tag slot is the
            // candidate unless an unpublished one comes before it (then the group is re-read).
            // One 16-byte key read a row, every row's issued together (a slot-by-slot scan reads
            // and compares the keys one dependent LDS round trip after another)
            int hit[R], empty[R], cand[R];
            bool pend[R];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                hit[u] = empty[u] = cand[u] = -1;
                pend[u] = false;
                if (!live[u]) continue;
                unsigned em = 0, mm = 0, pm = 0;
#pragma unroll
                for (int s = 0; s < GS; ++s) {
                    const uint64_t st = k[u][s];
                    const bool same = (st | 1ull) == (tag[u] | 1ull);
                    em |= (st == 0 ? 1u : 0u) << s;
                    mm |= (same && (st & 1ull) ? 1u : 0u) << s;
                    pm |= (same && !(st & 1ull) ? 1u : 0u) << s;
                }
                const unsigned lim = em ? (em & (0u - em)) - 1u : (1u << GS) - 1u;
                mm &= lim;
                pm &= lim;
                empty[u] = em ? __ffs(em) - 1 : -1;
                pend[u] = pm && (!mm || (pm & (0u - pm)) < (mm & (0u - mm)));
                cand[u] = (!pend[u] && mm) ? __ffs(mm) - 1 : -1;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            uint4 q[R];
#pragma unroll
            for (int u = 0; u < R; ++u)
                if (cand[u] >= 0) q[u] = wk[grp[u] * GS + cand[u]];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                if (cand[u] < 0) continue;
                if ((((uint64_t)q[u].y << 32) | q[u].x) == lo[u] && (((uint64_t)q[u].w << 32) | q[u].z) == hi[u]) {
                    hit[u] = cand[u];
                    continue;
                }
                // another key with the same tag (a 62-bit tag collision): the slots after it, one
                // by one, to the first empty / unpublished same-tag / matching one
                empty[u] = -1;
                for (int s = cand[u] + 1; s < GS; ++s) {
                    const uint64_t st = k[u][s];
                    if (st == 0) {
                        empty[u] = s;
                        break;
                    }
                    if ((st | 1ull) != (tag[u] | 1ull)) continue;
                    if (!(st & 1ull)) {
                        pend[u] = true;
                        break;
                    }
                    const uint4 q2 = wk[grp[u] * GS + s];
                    if ((((uint64_t)q2.y << 32) | q2.x) == lo[u] && (((uint64_t)q2.w << 32) | q2.z) == hi[u]) {
                        hit[u] = s;
                        break;
                    }
                }
            }
            bool any = false;
#pragma unroll
            for (int u = 0; u < R; ++u) {
                if (!live[u]) continue;
                if (hit[u] >= 0) {
                    cell[u] = (int)(grp[u] * GS + hit[u]);
                    live[u] = false;
                } else if (pend[u]) {
                    any = true; // a same-tag key is being published: re-read this group
                } else if (empty[u] >= 0) {
                    if (!may_insert) {
                        live[u] = false;
                        continue;
                    }
                    if (!force && __hip_atomic_load(&ctrl->full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                        live[u] = false;
                        continue;
                    }
                    if (!reserve(force)) {
                        live[u] = false;
                        continue;
                    }
                    const int c = (int)(grp[u] * GS + empty[u]);
                    const uint64_t old = atomicCAS((unsigned long long *)&keys[c], 0ull, (unsigned long long)tag[u]);
                    if (old != 0) atomicSub(&ctrl->used, 1u);
                    if (old == 0) {
                        uint4 w;
                        w.x = (unsigned)lo[u];
                        w.y = (unsigned)(lo[u] >> 32);
                        w.z = (unsigned)hi[u];
                        w.w = (unsigned)(hi[u] >> 32);
                        wk[c] = w;
                        __hip_atomic_store((unsigned long long *)&keys[c], (unsigned long long)(tag[u] | 1ull),
                                           __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        // read back: the loop's exit now depends on the publish, so it cannot be
                        // deferred past the loop (see the exit below)
                        if (__hip_atomic_load((unsigned long long *)&keys[c], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP) != (tag[u] | 1ull))
                            any = true;
                        cell[u] = c;
                        live[u] = false;
                    } else {
                        any = true; // raced: re-read the group
                    }
                } else {
                    grp[u] = grp[u] + 1 == ng ? 0 : grp[u] + 1;
                    any = true;
                }
            }
            // leave the loop together: a lane that exits waits at the loop's end for the whole
            // wave, and the compiler may sink a claimant's publish store there (after the loop) —
            // a lane of the same wave re-reading that pending cell would then spin forever
            if (__ballot(any) == 0) break;
        }
    }

    __device__ __forceinline__ uint64_t *acc_cell(int i, int cell) const {
        return reinterpret_cast<uint64_t *>(base + S.acc_off[i]) + (int64_t)cell * lds_acc_words(S.acc[i]);
    }
    __device__ __forceinline__ uint64_t *cnt_cell(int i, int cell) const {
        return reinterpret_cast<uint64_t *>(base + S.cnt_off[i]) + cell;
    }

    // fold a register-resident row (mode) into cell
    template <int NA, bool W> __device__ __forceinline__ void add_row(int cell, const RowValT<NA, W> &v, int mode) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int kind = S.kind[i];
            if (S.acc[i] == ACC_REF) { // row references: NULL rows of min / max arrive without a reference
                if (mode != MODE_STATE && v.vnull[i]) continue;
                ref_combine(acc_cell(i, cell), v.lo[i], S.ref[i], kind);
                continue;
            }
            if (S.acc[i] == ACC_ORD) { // min / max / first_row: max of order keys
                if (mode == MODE_STATE) {
                    atomicMax((unsigned long long *)acc_cell(i, cell), (unsigned long long)v.lo[i]);
                    if (S.has_cnt[i]) atomicAdd((unsigned long long *)cnt_cell(i, cell), (unsigned long long)v.cnt[i]);
                    continue;
                }
                if (v.vnull[i]) continue;
                atomicMax((unsigned long long *)acc_cell(i, cell), (unsigned long long)ord_enc(kind, S.src_type[i], v.lo[i]));
                if (S.has_cnt[i]) atomicAdd((unsigned long long *)cnt_cell(i, cell), 1ull);
                continue;
            }
            if (mode == MODE_STATE) {
                if constexpr (W)
                    if (S.acc[i] == ACC_I256) lds_add_i256(acc_cell(i, cell), v.lo[i], v.hi[i], v.x2[i], v.x3[i]);
                if (S.acc[i] == ACC_I128) lds_add_i128(acc_cell(i, cell), v.lo[i], v.hi[i]);
                else if (S.acc[i] == ACC_F64) atomicAdd((double *)acc_cell(i, cell), __longlong_as_double((long long)v.lo[i]));
                else if (S.acc[i] == ACC_I64) atomicAdd((unsigned long long *)acc_cell(i, cell), (unsigned long long)v.lo[i]);
                if (S.has_cnt[i]) atomicAdd((unsigned long long *)cnt_cell(i, cell), (unsigned long long)v.cnt[i]);
                continue;
            }
            if (kind == TFG_AGG_COUNT_ALL && mode == MODE_RAW) {
                atomicAdd((unsigned long long *)cnt_cell(i, cell), 1ull);
                continue;
            }
            if (v.vnull[i]) continue;
            if (kind != TFG_AGG_SUM) { // COUNT (raw: +1) or partial count (+value)
                atomicAdd((unsigned long long *)cnt_cell(i, cell), mode == MODE_RAW ? 1ull : (unsigned long long)v.lo[i]);
                continue;
            }
            uint64_t lo = v.lo[i], hi = v.hi[i];
            if (S.acc[i] == ACC_F64) {
                const double f = (mode == MODE_RAW && S.src_type[i] == TFG_FLOAT32)
                                     ? (double)__uint_as_float((unsigned)lo)
                                     : __longlong_as_double((long long)lo);
                atomicAdd((double *)acc_cell(i, cell), f);
            } else if (S.acc[i] == ACC_I256) {
                if constexpr (W) {
                    uint64_t x2 = v.x2[i], x3 = v.x3[i];
                    if (mode == MODE_RAW && S.src_type[i] != TFG_DECIMAL256) { // widen to 256 bits
                        widen_raw(S.src_type[i], lo, hi);
                        x2 = x3 = (int64_t)hi < 0 ? ~0ull : 0ull;
                    }
                    lds_add_i256(acc_cell(i, cell), lo, hi, x2, x3);
                }
            } else {
                if (mode == MODE_RAW) widen_raw(S.src_type[i], lo, hi);
                if (S.acc[i] == ACC_I128) lds_add_i128(acc_cell(i, cell), lo, hi);
                else atomicAdd((unsigned long long *)acc_cell(i, cell), (unsigned long long)lo);
            }
            if (S.has_cnt[i]) atomicAdd((unsigned long long *)cnt_cell(i, cell), 1ull);
        }
    }

    // fold group g of `grp` (state) into cell; REF: the signature may hold row-reference aggregates
    // (the tiled fast kernels' signatures never do)
    template <bool REF = true> __device__ __forceinline__ void add_group(int cell, const GroupsIO &grp, int64_t g) {
        for (int i = 0; i < S.n_aggs; ++i) {
            if (S.acc[i] == ACC_I256) {
                const uint64_t *v = (const uint64_t *)grp.acc[i] + 4 * g;
                lds_add_i256(acc_cell(i, cell), v[0], v[1], v[2], v[3]);
            } else if (S.acc[i] == ACC_I128) {
                const uint64_t *v = (const uint64_t *)grp.acc[i] + 2 * g;
                lds_add_i128(acc_cell(i, cell), v[0], v[1]);
            } else if (S.acc[i] == ACC_F64) {
                atomicAdd((double *)acc_cell(i, cell), ((const double *)grp.acc[i])[g]);
            } else if (S.acc[i] == ACC_I64) {
                atomicAdd((unsigned long long *)acc_cell(i, cell), ((const unsigned long long *)grp.acc[i])[g]);
            } else if (S.acc[i] == ACC_ORD) {
                atomicMax((unsigned long long *)acc_cell(i, cell), ((const unsigned long long *)grp.acc[i])[g]);
            } else if (REF && S.acc[i] == ACC_REF) {
                ref_combine(acc_cell(i, cell), ((const uint64_t *)grp.acc[i])[g], S.ref[i], S.kind[i]);
            }
            if (S.has_cnt[i]) atomicAdd((unsigned long long *)cnt_cell(i, cell), grp.cnt[i][g]);
        }
    }

    __device__ void flush(const GroupsIO &out, uint64_t out_base) {
        // output slots: one LDS atomic per wave for its occupied cells (ballot + rank), not one
        // per cell on the one counter
        for (int c0 = 0; c0 < S.cap + 2; c0 += blockDim.x) {
            const int c = c0 + (int)threadIdx.x;
            bool occ = false;
            uint64_t key = 0;
            uint8_t isnull = 0;
            if (c < S.cap) {
                key = keys[c];
                occ = key != 0;
            } else if (c == S.cap) {
                occ = ctrl->zero_used;
            } else if (c == S.cap + 1) {
                occ = ctrl->null_used;
                isnull = 1;
            }
            const uint64_t m = __ballot(occ);
            if (m == 0) continue; // uniform in the wave
            const int lane = (int)__lane_id(), first = __ffsll((unsigned long long)m) - 1;
            unsigned long long wb = 0;
            if (lane == first) wb = atomicAdd(&ctrl->out_count, (unsigned long long)__popcll(m));
            wb = __shfl(wb, first, 64);
            if (!occ) continue;
            const uint64_t pos = out_base + wb + (uint64_t)__popcll(m & ((1ull << lane) - 1));
            if (S.wkey_off) { // wide: the cell's 16-byte key (tags never take the side slots)
                reinterpret_cast<uint4 *>(out.key)[pos] = reinterpret_cast<const uint4 *>(base + S.wkey_off)[c];
            } else {
                out.key[pos] = key;
            }
            out.key_null[pos] = isnull;
            for (int i = 0; i < S.n_aggs; ++i) {
                if (S.acc[i] == ACC_I128 || S.acc[i] == ACC_I256) {
                    const int nw = acc_words(S.acc[i]);
                    const uint64_t *a = acc_cell(i, c);
                    for (int k = 0; k < nw; ++k) ((uint64_t *)out.acc[i])[nw * pos + k] = a[k];
                    if (S.acc[i] == ACC_I256 && !fits_i256(a) && S.ovf) atomicOr(S.ovf, 1u);
                } else if (S.acc[i] != ACC_NONE) {
                    ((uint64_t *)out.acc[i])[pos] = *acc_cell(i, c);
                }
                if (S.has_cnt[i]) out.cnt[i][pos] = *cnt_cell(i, c);
            }
        }
    }
};

// width in bytes of value column i for a row mode
__device__ __forceinline__ int val_width(const AggSpec &S, int mode, int i) {
    if (S.acc[i] == ACC_REF) return 8; // row references in every mode
    // partial min / max / first_row values have the argument's type (the result type)
    if (mode == MODE_PARTIAL && S.acc[i] == ACC_ORD) mode = MODE_RAW;
    if (mode != MODE_RAW) return S.acc[i] == ACC_I256 ? 32 : S.acc[i] == ACC_I128 ? 16 : 8;
    switch (S.src_type[i]) {
    case TFG_DECIMAL256: return 32;
    case TFG_INT8: case TFG_UINT8: return 1;
    case TFG_INT16: case TFG_UINT16: return 2;
    case TFG_INT32: case TFG_UINT32: case TFG_FLOAT32: case TFG_DECIMAL32: return 4;
    case TFG_DECIMAL128: return 16;
    default: return 8;
    }
}

template <int NA, bool W>
__device__ __forceinline__ void load_row(const AggSpec &S, const RowsIO &rows, int mode, int64_t r, RowValT<NA, W> &v) {
    if (rows.key_width != 16) v.key = load_bits(rows.key, rows.key_width, r); // wide keys: WideOps
    v.knull = rows.key_null ? rows.key_null[r] : 0;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        v.lo[i] = v.hi[i] = v.cnt[i] = 0;
        v.vnull[i] = rows.val_null[i] ? rows.val_null[i][r] : 0;
        if (rows.val_cnt[i]) v.cnt[i] = rows.val_cnt[i][r];
        if constexpr (W) v.x2[i] = v.x3[i] = 0;
        if (!rows.val[i]) continue;
        const int w = val_width(S, mode, i);
        if (w == 32) {
            if constexpr (W) {
                const uint4 q = ((const uint4 *)rows.val[i])[2 * r], q2 = ((const uint4 *)rows.val[i])[2 * r + 1];
                v.lo[i] = ((uint64_t)q.y << 32) | q.x;
                v.hi[i] = ((uint64_t)q.w << 32) | q.z;
                v.x2[i] = ((uint64_t)q2.y << 32) | q2.x;
                v.x3[i] = ((uint64_t)q2.w << 32) | q2.z;
            }
        } else if (w == 16) {
            const uint4 q = ((const uint4 *)rows.val[i])[r];
            v.lo[i] = ((uint64_t)q.y << 32) | q.x;
            v.hi[i] = ((uint64_t)q.w << 32) | q.z;
        } else {
            v.lo[i] = load_bits(rows.val[i], w, r);
        }
    }
}

// in-place compaction of the bucket's pending rows: write a register row to slot w
template <int NA, bool W>
__device__ __forceinline__ void store_row(const AggSpec &S, const RowsIO &rows, int mode, int64_t w, const RowValT<NA, W> &v) {
    switch (rows.key_width) {
    case 1: ((uint8_t *)rows.key)[w] = (uint8_t)v.key; break;
    case 2: ((uint16_t *)rows.key)[w] = (uint16_t)v.key; break;
    case 4: ((uint32_t *)rows.key)[w] = (uint32_t)v.key; break;
    case 16: break; // wide keys: WideOps
    default: ((uint64_t *)rows.key)[w] = v.key; break;
    }
    if (rows.key_null) rows.key_null[w] = v.knull;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        if (rows.val_null[i]) rows.val_null[i][w] = v.vnull[i];
        if (rows.val_cnt[i]) rows.val_cnt[i][w] = v.cnt[i];
        if (!rows.val[i]) continue;
        switch (val_width(S, mode, i)) {
        case 1: ((uint8_t *)rows.val[i])[w] = (uint8_t)v.lo[i]; break;
        case 2: ((uint16_t *)rows.val[i])[w] = (uint16_t)v.lo[i]; break;
        case 4: ((uint32_t *)rows.val[i])[w] = (uint32_t)v.lo[i]; break;
        case 8: ((uint64_t *)rows.val[i])[w] = v.lo[i]; break;
        case 32:
            if constexpr (W) {
                uint64_t *o = (uint64_t *)rows.val[i] + 4 * w;
                o[0] = v.lo[i];
                o[1] = v.hi[i];
                o[2] = v.x2[i];
                o[3] = v.x3[i];
            }
            break;
        default: {
            uint4 q;
            q.x = (unsigned)v.lo[i];
            q.y = (unsigned)(v.lo[i] >> 32);
            q.z = (unsigned)v.hi[i];
            q.w = (unsigned)(v.hi[i] >> 32);
            ((uint4 *)rows.val[i])[w] = q;
        }
        }
    }
}

// RPT rows per thread per step: several independent row loads in flight per thread, and one
// barrier per step.  Misses (keys that do not fit the table, or whose older group is still
// pending) are appended to the other row buffer (ping-pong), processed by the next pass.
#ifndef TFG_EXP_RPT
constexpr int RPT = 4;
#else // experiment builds (tools/build_exp.sh) of the bucket kernels only
constexpr int RPT = TFG_EXP_RPT;
#endif

// Row policies of the bucket kernel.  GenericOps handles every signature / mode / null map
// through runtime switches; FastOps<A0,A1,A2> is the compile-time specialisation of the hot
// signatures (8-byte key, no NULLs, RAW rows) — op codes: 0 absent, 1 count, 2 sum into Int64,
// 3 sum Float64, 4 sum Decimal64 into Int128.  Without it the per-row switches cost ~350
// wave-instructions per 64 rows (measured with SQ_INSTS_VALU / SQ_INSTS_SALU).
template <int NA, bool W = false> struct GenericOps {
    using Row = RowValT<NA, W>;
    static constexpr bool WIDE = false;
    __device__ __forceinline__ uint64_t hi(const Row &) const { return 0; }
    const AggSpec &S;
    int mode;
    __device__ __forceinline__ void load(const RowsIO &rows, int64_t r, Row &v) const { load_row<NA, W>(S, rows, mode, r, v); }
    __device__ __forceinline__ uint64_t key(const Row &v) const { return v.key; }
    __device__ __forceinline__ bool knull(const Row &v) const { return v.knull != 0; }
    __device__ __forceinline__ void add(Table &T, int cell, const Row &v) const { T.add_row<NA, W>(cell, v, mode); }
    __device__ __forceinline__ void store(const RowsIO &sp, int64_t w, const Row &v) const { store_row<NA, W>(S, sp, mode, w, v); }
};

// The value ops of FastOps / WideFastOps for R rows of one step (op codes below).  CHECK: cells
// < 0 are skipped (add_multi); otherwise every cell is valid (add_all: rows without a cell of
// their own add into a dummy cell that is never flushed, so no per-row branch).  A Decimal64 ->
// Int128 sum issues every row's returning low-word add before any high-word add, so the carries'
// LDS round trips overlap.
template <int A0, int A1, int A2, bool CHECK, int R, typename Row>
__device__ __forceinline__ void fast_add_rows(Table &T, const int (&cell)[R], const Row (&v)[R]) {
    constexpr int ops[3] = {A0, A1, A2};
    // the op codes fix the accumulator widths (op 4: a two-word Int128 sum, else one word), so
    // a cell's address needs no per-row look at S.acc (T.acc_cell)
    auto acc = [&](int i, int c) __attribute__((always_inline)) {
        return reinterpret_cast<uint64_t *>(T.base + T.S.acc_off[i]) + c * (ops[i] == 4 ? 2 : 1);
    };
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (ops[i] != 4) continue;
        uint64_t old[R];
#pragma unroll
        for (int u = 0; u < R; ++u)
            if (!CHECK || cell[u] >= 0) old[u] = atomicAdd((unsigned long long *)acc(i, cell[u]), (unsigned long long)v[u].v[i]);
#pragma unroll
        for (int u = 0; u < R; ++u) {
            if (CHECK && cell[u] < 0) continue;
            const uint64_t lo = v[u].v[i], carry = (old[u] + lo) < old[u] ? 1ull : 0ull;
            // the high word's addend (sign extension + carry) is 0 for most rows (a non-negative
            // value without carry, a negative one with): those issue no second atomic
            const uint64_t hi = ((int64_t)lo < 0 ? ~0ull : 0ull) + carry;
            if (hi) atomicAdd((unsigned long long *)acc(i, cell[u]) + 1, (unsigned long long)hi);
        }
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
        if (CHECK && cell[u] < 0) continue;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (ops[i] == 1) atomicAdd((unsigned long long *)T.cnt_cell(i, cell[u]), 1ull);
            if (ops[i] == 2) atomicAdd((unsigned long long *)acc(i, cell[u]), (unsigned long long)v[u].v[i]);
            if (ops[i] == 3) atomicAdd((double *)acc(i, cell[u]), __longlong_as_double((long long)v[u].v[i]));
        }
    }
}

template <int A0, int A1, int A2> struct FastOps {
    // rows are staged as interleaved records: key, then one word per summed argument
    static constexpr int op(int i) { return i == 0 ? A0 : (i == 1 ? A1 : A2); }
    static constexpr int NCOL = 1 + (A0 >= 2) + (A1 >= 2) + (A2 >= 2);
    static constexpr bool WIDE = false;
    static constexpr bool NARROWABLE = NCOL == 2; // the tiled partition may write {u32 key}[], {value}[] tiles
    static constexpr int pos(int i) { return 1 + (i > 0 && A0 >= 2) + (i > 1 && A1 >= 2); }
    struct Row {
        uint64_t key;
        uint64_t v[3];
    };
    const AggSpec &S;
    int mode;
    __device__ __forceinline__ void load(const RowsIO &rows, int64_t r, Row &v) const {
        const uint64_t *rec = (const uint64_t *)rows.key + r * NCOL;
        if constexpr (NCOL == 2) {
            const uint4 q = *(const uint4 *)rec;
            v.key = ((uint64_t)q.y << 32) | q.x;
            const uint64_t w = ((uint64_t)q.w << 32) | q.z;
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (op(i) >= 2) v.v[i] = w;
        } else {
            v.key = rec[0];
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (op(i) >= 2) v.v[i] = rec[pos(i)];
        }
    }
    // A tiled row's words as loaded (load_raw), converted to a Row when the step uses them
    // (unraw).  load_raw is branch-free: the same load instructions for a narrow or a 16-byte
    // record, from a per-lane address, so the loads stay in flight across the step before (a load
    // inside a divergent branch, or a loaded register copied at a join, is waited for there).
    // Narrow tile slot: TRS u32 keys, then TRS u64 values; the key is read as 8 bytes (the upper
    // half is the next key, or the first value word: discarded).  Rows past the chunk (ok false)
    // read the first record.
    struct Raw {
        uint64_t w[NCOL];
        bool nar;
    };
    __device__ __forceinline__ void load_raw(const uint64_t *rec, uint64_t slot, int TRS, uint32_t off, bool nar,
                                             bool ok, Raw &r) const {
        if constexpr (NCOL == 2) {
            const uint32_t *ks = reinterpret_cast<const uint32_t *>(rec + slot * 2);
            const uint64_t *kp = nar ? reinterpret_cast<const uint64_t *>(ks + off) : rec + (slot + off) * 2;
            const uint64_t *vp = nar ? reinterpret_cast<const uint64_t *>(ks + TRS) + off : rec + (slot + off) * 2 + 1;
            r.w[0] = *(ok ? kp : rec);
            r.w[1] = *(ok ? vp : rec);
            r.nar = nar;
        } else {
            const uint64_t *p = ok ? rec + (slot + off) * NCOL : rec;
#pragma unroll
            for (int c = 0; c < NCOL; ++c) r.w[c] = p[c];
            r.nar = false;
        }
    }
    __device__ __forceinline__ void unraw(const Raw &r, Row &v) const {
        v.key = r.nar ? (r.w[0] & 0xFFFFFFFFull) : r.w[0];
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (op(i) >= 2) v.v[i] = r.w[pos(i)];
    }
    __device__ __forceinline__ uint64_t key(const Row &v) const { return v.key; }
    __device__ __forceinline__ bool knull(const Row &) const { return false; }
    __device__ __forceinline__ uint64_t hi(const Row &) const { return 0; }
    __device__ __forceinline__ void add(Table &T, int cell, const Row &v) const {
        const int c1[1] = {cell};
        const Row v1[1] = {v};
        fast_add_rows<A0, A1, A2, false>(T, c1, v1);
    }
    template <int R>
    __device__ __forceinline__ void add_multi(Table &T, const int (&cell)[R], const Row (&v)[R]) const {
        fast_add_rows<A0, A1, A2, true>(T, cell, v);
    }
    template <int R>
    __device__ __forceinline__ void add_all(Table &T, const int (&cell)[R], const Row (&v)[R]) const {
        fast_add_rows<A0, A1, A2, false>(T, cell, v);
    }
    __device__ __forceinline__ void store(const RowsIO &sp, int64_t w, const Row &v) const {
        uint64_t *rec = (uint64_t *)sp.key + w * NCOL;
        rec[0] = v.key;
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (op(i) >= 2) rec[pos(i)] = v.v[i];
    }
};

// Wide keys (16-byte packed keys128 / String keys, staged as one uint4 per row): generic
// value handling, the key's two words travel in Row::key and Row::hi.
template <int NA, bool W = false> struct WideOps {
    struct Row : RowValT<NA, W> {
        uint64_t khi;
    };
    static constexpr bool WIDE = true;
    const AggSpec &S;
    int mode;
    __device__ __forceinline__ void load(const RowsIO &rows, int64_t r, Row &v) const {
        load_row<NA, W>(S, rows, mode, r, v);
        const uint4 q = reinterpret_cast<const uint4 *>(rows.key)[r];
        v.key = ((uint64_t)q.y << 32) | q.x;
        v.khi = ((uint64_t)q.w << 32) | q.z;
    }
    __device__ __forceinline__ uint64_t key(const Row &v) const { return v.key; }
    __device__ __forceinline__ uint64_t hi(const Row &v) const { return v.khi; }
    __device__ __forceinline__ bool knull(const Row &) const { return false; }
    __device__ __forceinline__ void add(Table &T, int cell, const Row &v) const { T.add_row<NA, W>(cell, v, mode); }
    __device__ __forceinline__ void store(const RowsIO &sp, int64_t w, const Row &v) const {
        store_row<NA, W>(S, sp, mode, w, v);
        uint4 q;
        q.x = (unsigned)v.key;
        q.y = (unsigned)(v.key >> 32);
        q.z = (unsigned)v.khi;
        q.w = (unsigned)(v.khi >> 32);
        reinterpret_cast<uint4 *>(sp.key)[w] = q;
    }
};

// Wide keys on the tiled path: records {key lo, key hi, one word per summed argument}; the
// value ops are FastOps' (1 count, 2 Int64 / UInt64 sum, 3 Float64 sum, 4 Decimal64 -> Decimal128)
template <int A0, int A1, int A2> struct WideFastOps {
    static constexpr int op(int i) { return i == 0 ? A0 : (i == 1 ? A1 : A2); }
    static constexpr int NCOL = 2 + (A0 >= 2) + (A1 >= 2) + (A2 >= 2);
    static constexpr bool WIDE = true;
    // one summed argument: narrow tiles (WNARROW, partition.h) hold 20-byte records (nrec_store)
    static constexpr bool NARROWABLE = NCOL == 3;
    static constexpr int pos(int i) { return 2 + (i > 0 && A0 >= 2) + (i > 1 && A1 >= 2); }
    struct Row {
        uint64_t key, khi;
        uint64_t v[3];
    };
    // FastOps::load_raw / unraw.  NCOL 3: 16 bytes from the row's start (key lo, then the narrow
    // hi word or the two hi words) and 8 bytes from its value (offset 12 in a 20-byte record, 16 in
    // a 24-byte one); rows of a narrow slot start at 20-byte steps (4-byte aligned loads)
    struct Raw {
        uint4 q;
        uint64_t w[NCOL == 3 ? 1 : NCOL];
        bool nar;
    };
    __device__ __forceinline__ void load_raw(const uint64_t *rec, uint64_t slot, int, uint32_t off, bool nar, bool ok,
                                             Raw &r) const {
        if constexpr (NCOL == 3) {
            const char *b = nar ? reinterpret_cast<const char *>(rec + slot * 3) + (size_t)off * 20
                                : reinterpret_cast<const char *>(rec + (slot + off) * 3);
            if (!ok) b = reinterpret_cast<const char *>(rec);
            typedef unsigned u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
            typedef unsigned u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
            const u32x4a4 q = *reinterpret_cast<const u32x4a4 *>(b);
            const u32x2a4 w = *reinterpret_cast<const u32x2a4 *>(b + (nar ? 12 : 16));
            r.q = make_uint4(q.x, q.y, q.z, q.w);
            r.w[0] = (uint64_t)w.x | ((uint64_t)w.y << 32);
            r.nar = nar;
        } else {
            const uint64_t *p = ok ? rec + (slot + off) * NCOL : rec;
            const uint4 q = *reinterpret_cast<const uint4 *>(p);
            r.q = q;
#pragma unroll
            for (int c = 2; c < NCOL; ++c) r.w[c] = p[c];
            r.nar = false;
        }
    }
    __device__ __forceinline__ void unraw(const Raw &r, Row &v) const {
        v.key = ((uint64_t)r.q.y << 32) | r.q.x;
        v.khi = r.nar ? wide_wide_hi(r.q.z) : (((uint64_t)r.q.w << 32) | r.q.z);
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (op(i) >= 2) v.v[i] = NCOL == 3 ? r.w[0] : r.w[pos(i)];
    }
    const AggSpec &S;
    int mode;
    __device__ __forceinline__ void load(const RowsIO &rows, int64_t r, Row &v) const {
        const uint64_t *rec = (const uint64_t *)rows.key + r * NCOL; // 8-byte aligned records
        v.key = rec[0];
        v.khi = rec[1];
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (op(i) >= 2) v.v[i] = rec[pos(i)];
    }
    __device__ __forceinline__ uint64_t key(const Row &v) const { return v.key; }
    __device__ __forceinline__ uint64_t hi(const Row &v) const { return v.khi; }
    __device__ __forceinline__ bool knull(const Row &) const { return false; }
    __device__ __forceinline__ void add(Table &T, int cell, const Row &v) const {
        const int c1[1] = {cell};
        const Row v1[1] = {v};
        fast_add_rows<A0, A1, A2, false>(T, c1, v1);
    }
    template <int R>
    __device__ __forceinline__ void add_multi(Table &T, const int (&cell)[R], const Row (&v)[R]) const {
        fast_add_rows<A0, A1, A2, true>(T, cell, v);
    }
    __device__ __forceinline__ void store(const RowsIO &sp, int64_t w, const Row &v) const {
        uint64_t *rec = (uint64_t *)sp.key + w * NCOL;
        rec[0] = v.key;
        rec[1] = v.khi;
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (op(i) >= 2) rec[pos(i)] = v.v[i];
    }
};

template <typename Ops, int BT>
__global__ void __launch_bounds__(BT) agg_bucket_kernel(AggSpec S, RowsIO rows0, RowsIO rows1, int mode,
                                                        const uint64_t *stage_off, GroupsIO old,
                                                        const uint64_t *old_off, GroupsIO out, uint64_t *out_cnt) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    Table T(lds, S);
    const Ops ops{S, mode};
    const int b = blockIdx.x;
    const int64_t rs = (int64_t)stage_off[b];
    int64_t pending = (int64_t)stage_off[b + 1] - rs;
    int64_t os = 0, oe = 0;
    if (old_off) {
        os = (int64_t)old_off[b];
        oe = (int64_t)old_off[b + 1];
    }
    const uint64_t out_base = (uint64_t)os + (uint64_t)rs;
    int64_t old_cursor = os;
    int pass = 0;
    if (threadIdx.x == 0) T.ctrl->out_count = 0;
    while (pending > 0 || old_cursor < oe) {
        const RowsIO &rows = (pass & 1) ? rows1 : rows0;
        const RowsIO &spill = (pass & 1) ? rows0 : rows1;
        ++pass;
        T.clear();
        __syncthreads();
        // phase A: a chunk of existing groups (distinct keys)
        int64_t take = oe - old_cursor;
        if (take > S.maxfill) take = S.maxfill;
        for (int64_t g = old_cursor + threadIdx.x; g < old_cursor + take; g += BT) {
            int cell;
            if constexpr (Ops::WIDE) {
                const uint64_t lo[1] = {old.key[2 * g]}, hi[1] = {old.key[2 * g + 1]};
                const uint64_t tg[1] = {wide_tag(lo[0], hi[0])};
                const bool ok[1] = {true};
                int c1[1];
                T.find_wide_multi<1>(lo, hi, tg, ok, true, c1, true);
                cell = c1[0];
            } else {
                cell = T.find_or_insert(old.key[g], old.key_null[g] != 0, true, true);
            }
            T.add_group(cell, old, g);
        }
        old_cursor += take;
        const bool allow_insert = old_cursor >= oe;
        __syncthreads();
        // phase B: pending rows; misses go to the other buffer for the next pass
        const uint32_t npend = (uint32_t)pending;
        for (uint32_t base = 0; base < npend; base += BT * RPT) {
            typename Ops::Row v[RPT];
            uint64_t ku[RPT];
            bool nu[RPT], vu[RPT], miss[RPT];
            int cells[RPT];
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                const uint32_t i = base + u * BT + threadIdx.x;
                vu[u] = i < npend;
                if (vu[u]) ops.load(rows, rs + i, v[u]);
            }
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                ku[u] = ops.key(v[u]);
                nu[u] = ops.knull(v[u]);
            }
            uint64_t kh[RPT], tg[RPT];
            if constexpr (Ops::WIDE) {
#pragma unroll
                for (int u = 0; u < RPT; ++u) {
                    kh[u] = ops.hi(v[u]);
                    tg[u] = wide_tag(ku[u], kh[u]);
                }
                T.find_wide_multi<RPT>(ku, kh, tg, vu, allow_insert, cells);
            } else {
                T.find_or_insert_multi<RPT>(ku, nu, vu, allow_insert, cells);
            }
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                miss[u] = false;
                if (!vu[u]) continue;
                if (cells[u] >= 0) ops.add(T, cells[u], v[u]);
                else miss[u] = true;
            }
            // inserts of this step are complete before any retry: a retry sees the final key set
            // (a miss means the table was full, or inserts are disabled, so no later step of this
            // pass can insert the key either)
            __syncthreads();
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                if (!miss[u]) continue;
                int cell;
                if constexpr (Ops::WIDE) {
                    const uint64_t lo[1] = {ku[u]}, hi[1] = {kh[u]}, t1[1] = {tg[u]};
                    const bool ok[1] = {true};
                    int c1[1];
                    T.find_wide_multi<1>(lo, hi, t1, ok, false, c1);
                    cell = c1[0];
                } else {
                    cell = T.find_or_insert(ku[u], nu[u], false, false);
                }
                if (cell >= 0) {
                    ops.add(T, cell, v[u]);
                } else {
                    const int64_t w = rs + (int64_t)atomicAdd(&T.ctrl->spill_w, 1ull);
                    ops.store(spill, w, v[u]);
                }
            }
        }
        __syncthreads();
        T.flush(out, out_base);
        __syncthreads();
        pending = (int64_t)T.ctrl->spill_w;
        __syncthreads();
    }
    if (threadIdx.x == 0) out_cnt[b] = T.ctrl->out_count;
}

// Bucket kernel over a tile-sorted partition (run_partition_tiled): bucket b's rows are runs
// in every tile, tile_hist[b * T + t] = start | count << 16.  Pass 0 walks the runs chunk by
// chunk (runs average kept / B rows, ~30 for C2).  Rows that miss (table full / older groups pending) go to
// the bucket's spill regions, reserved once per workgroup from a global cursor, and later passes
// ping-pong between them as in agg_bucket_kernel.  Temp groups go to a region reserved the same
// way; tmp_base[b] tells the compaction where.
struct TiledIn {
    const uint64_t *rec;       // records of the tiled partition (Ops::NCOL words each)
    const uint32_t *tile_hist; // [B][T]; two-level: [1 << fine_bits][T]
    int T;
    int TR;
    // two-level partition (regroup_tiled_kernel): bucket b = coarse c << fine_bits | fine f reads
    // row f of tile_hist over the tiles [tile_base[c], tile_base[c + 1]); null: one level
    const uint32_t *tile_base;
    int fine_bits;
    // XCD-aware bucket order: workgroup w (dispatched to XCD w % 8) takes bucket
    // (w % 8) * (B / 8) + w / 8, so the B / 8 buckets whose runs neighbour each other inside every
    // tile are read by one XCD and share its L2 (the lines a run shares with the next one)
    int xcd_remap;
    uint64_t *spill[2];        // two spill arenas of >= kept rows (records)
    unsigned long long *cursor; // [0] spill rows, [1] temp groups
};

// the 512-thread form runs where two workgroups' tables fit one CU's LDS: held to 128 VGPRs (4
// waves per SIMD) so that both workgroups are resident (at 131 the second never fit)
template <typename Ops, int BT>
__global__ void __launch_bounds__(BT) __attribute__((amdgpu_waves_per_eu(BT <= 512 ? 4 : 1)))
agg_bucket_tiled_kernel(AggSpec S, TiledIn tin, int mode, GroupsIO old,
                                                              const uint64_t *old_off, GroupsIO out, uint64_t *out_cnt,
                                                              uint64_t *tmp_base) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    // rows per thread per step.  Wide rows: one (r06ab, C5, two alternating runs each: 1 row
    // 1.276 / 1.285 ms, 2 rows 1.454 / 1.457, 3 rows 2.155 / 2.151 — 103 VGPRs and no scratch at
    // one row, 272 B of spills at three: more waves' worth of independent steps beat more rows)
    // 8-byte keys: two (r06ad, C2, two alternating runs each: agg.bucket 0.424 ms at four rows,
    // 0.392 at two, 0.407 at one; 0.388 at two with the alternating register sets below)
#ifndef TFG_EXP_WRT
    constexpr int RT = Ops::WIDE ? 1 : 2;
#else
    constexpr int RT = Ops::WIDE ? TFG_EXP_WRT : 2; // experiment: wide rows per thread per step
#endif
    __shared__ unsigned long long s_red[BT / 64];
    __shared__ unsigned long long s_base[3];
    constexpr int CH = BT; // tiles per pass-0 chunk: one per thread
    // per run of the chunk: {its end (chunk row) | narrow << 31, its tile offset minus its start}
    __shared__ uint2 s_run[CH];
    __shared__ uint32_t s_tot;
    __shared__ uint32_t s_wsum[BT / 64];
    // sampled row -> run index of a chunk: s_idx[k] = the run holding row k << idx_sh
#ifndef TFG_EXP_IDXN
    constexpr int IDXN = 2048;
#else
    constexpr int IDXN = TFG_EXP_IDXN;
#endif
    __shared__ uint16_t s_idx[IDXN];
    Table T(lds, S);
    const Ops ops{S, mode};
    const int b = (tin.xcd_remap && (gridDim.x & 7) == 0)
                      ? (int)((blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3))
                      : (int)blockIdx.x;
    const uint32_t *col = tin.tile_hist + (size_t)(tin.tile_base ? (b & ((1 << tin.fine_bits) - 1)) : b) * tin.T;
    const int tbeg = tin.tile_base ? (int)tin.tile_base[b >> tin.fine_bits] : 0;
    const int tend = tin.tile_base ? (int)tin.tile_base[(b >> tin.fine_bits) + 1] : tin.T;
    // rows of this bucket.  e0: this thread's entry of the first chunk of tiles, kept for pass 0
    // (one global round trip less a bucket: C5's buckets span one chunk)
    unsigned long long tot = 0;
    uint32_t e0 = 0;
    {
        int t = tbeg + (int)threadIdx.x;
        if (Ops::WIDE && t < tend) { // (one-level buckets walk ~12K tiles: nothing to keep)
            e0 = col[t];
            tot += e0 >> 16;
            t += BT;
        }
        for (; t < tend; t += BT) tot += col[t] >> 16;
    }
    for (int d = 32; d > 0; d >>= 1) tot += __shfl_down(tot, d, 64);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = tot;
    __syncthreads();
    int64_t os = 0, oe = 0;
    if (old_off) {
        os = (int64_t)old_off[b];
        oe = (int64_t)old_off[b + 1];
    }
    unsigned long long rows_b = 0; // every thread sums the wave totals (no round trip through thread 0)
#pragma unroll
    for (int w = 0; w < BT / 64; ++w) rows_b += s_red[w];
    const bool no_rows = rows_b == 0; // a bucket no kept row reached: pass 0 has nothing to walk
    // thread 0 reserves the spill rows and temp groups; the atomics' results are stored after
    // the table clear below, so their round trip overlaps it
    unsigned long long r0 = 0, r1 = 0;
    if (threadIdx.x == 0) {
        r0 = atomicAdd(&tin.cursor[0], rows_b);
        r1 = atomicAdd(&tin.cursor[1], rows_b + (unsigned long long)(oe - os));
        T.ctrl->out_count = 0;
    }
    if (no_rows && os == oe) { // nothing at all: no table to build or flush
        if (threadIdx.x == 0) {
            out_cnt[b] = 0;
            tmp_base[b] = r1;
        }
        return;
    }
    T.clear(); // pass 0's table
    if (threadIdx.x == 0) {
        s_base[0] = r0;
        s_base[1] = r1;
    }
    __syncthreads();
    const uint64_t sbase = s_base[0], out_base = s_base[1];
    // the two spill regions as plain pointers, chosen per pass by value (an array of RowsIO
    // indexed by the pass would live in scratch memory)
    RowsIO src{};
    src.key = (void *)tin.rec;
    uint64_t *const reg0 = tin.spill[0] + sbase * Ops::NCOL, *const reg1 = tin.spill[1] + sbase * Ops::NCOL;
    int64_t old_cursor = os;
    int64_t pending = -1; // pass 0: the tile runs
    int pass = 0;
    while (pending != 0 || old_cursor < oe) {
        RowsIO rows{}, spill{};
        rows.key = (pass & 1) ? reg0 : reg1;  // pass p >= 1 reads region (p - 1) & 1
        spill.key = (pass & 1) ? reg1 : reg0; // ... and spills into region p & 1
        if (pass > 0) { // pass 0's table was cleared with the prologue
            T.clear();
            __syncthreads();
        }
        if (threadIdx.x == 0) T.ctrl->spill_w = 0;
        int64_t take = oe - old_cursor;
        if (take > S.maxfill) take = S.maxfill;
        for (int64_t g = old_cursor + threadIdx.x; g < old_cursor + take; g += BT) {
            int cell;
            if constexpr (Ops::WIDE) {
                const uint64_t lo[1] = {old.key[2 * g]}, hi[1] = {old.key[2 * g + 1]};
                const uint64_t tg[1] = {wide_tag(lo[0], hi[0])};
                const bool ok1[1] = {true};
                int c1[1];
                T.find_wide_multi<1>(lo, hi, tg, ok1, true, c1, true);
                cell = c1[0];
            } else {
                cell = T.find_or_insert(old.key[g], old.key_null[g] != 0, true, true);
            }
            T.template add_group<false>(cell, old, g);
        }
        old_cursor += take;
        const bool allow_insert = old_cursor >= oe;
        __syncthreads();
        // one step: up to RT rows per thread (v / ok), lookup, add, retry misses after a barrier
        auto step = [&](typename Ops::Row (&v)[RT], bool (&ok)[RT]) __attribute__((always_inline)) {
            uint64_t ku[RT], kh[RT], tg[RT];
            bool nu[RT];
            int cells[RT];
            bool miss[RT];
#pragma unroll
            for (int u = 0; u < RT; ++u) {
                ku[u] = ops.key(v[u]);
                kh[u] = ops.hi(v[u]);
                tg[u] = Ops::WIDE ? wide_tag(ku[u], kh[u]) : 0;
                nu[u] = false;
            }
            if constexpr (!Ops::WIDE) {
                // fast path (8-byte keys, never NULL): the home-group lookup of every row, the
                // adds of the found rows (others into the NULL-key slot, unused by these keys:
                // a dummy), then — one uniform branch — the rare rows that need the full probe
                // (overflow group, insert) or spill
#ifdef TFG_EXP_NOPROBE // profiling experiment only: a hashed cell instead of the table lookup
#pragma unroll
                for (int u = 0; u < RT; ++u) cells[u] = (int)(((uint32_t)ku[u] * 2654435761u) % (uint32_t)S.cap);
#else
                T.find_home<RT>(ku, cells);
#endif
                int acell[RT];
                bool slow[RT], anyslow = false;
#pragma unroll
                for (int u = 0; u < RT; ++u) {
                    slow[u] = ok[u] && cells[u] < 0;
                    anyslow = anyslow || slow[u];
                    acell[u] = (ok[u] && cells[u] >= 0) ? cells[u] : S.cap + 1;
                }
#ifndef TFG_EXP_NOATOM // profiling experiment only: no state update
                ops.add_all(T, acell, v);
#endif
                if (__ballot(anyslow) == 0) return;
#pragma unroll
                for (int u = 0; u < RT; ++u) {
                    if (!slow[u]) continue;
                    int cell = T.find_or_insert(ku[u], false, allow_insert, false);
                    if (cell < 0) cell = T.find_or_insert(ku[u], false, false, false);
                    if (cell >= 0) {
                        ops.add(T, cell, v[u]);
                    } else {
                        const int64_t w = (int64_t)atomicAdd(&T.ctrl->spill_w, 1ull);
                        ops.store(spill, w, v[u]);
                    }
                }
                return;
            }
#ifdef TFG_EXP_NOPROBE // profiling experiment only: a hashed cell instead of the wide lookup
#pragma unroll
            for (int u = 0; u < RT; ++u) cells[u] = (int)((uint32_t)(tg[u] >> 32) % (uint32_t)S.cap);
#else
            if constexpr (Ops::WIDE) T.find_wide_multi<RT>(ku, kh, tg, ok, allow_insert, cells);
            else T.find_or_insert_multi<RT>(ku, nu, ok, allow_insert, cells);
#endif
            int hit[RT];
#pragma unroll
            for (int u = 0; u < RT; ++u) {
                miss[u] = ok[u] && cells[u] < 0;
                hit[u] = ok[u] ? cells[u] : -1;
            }
#ifndef TFG_EXP_NOATOM // profiling experiment only: no state update
            ops.add_multi(T, hit, v);
#endif
            // no barrier per step: a missing row (full table / inserts closed) looks its key up
            // once more and otherwise spills; an insert of the same key by another wave in this
            // step may not be visible yet, so the pass re-checks its spilled rows against the
            // final table before flushing (below) — no key ends up in two groups
#pragma unroll
            for (int u = 0; u < RT; ++u) {
                if (!miss[u]) continue;
                int cell;
                if constexpr (Ops::WIDE) {
                    const uint64_t lo[1] = {ku[u]}, hi[1] = {kh[u]}, t1[1] = {tg[u]};
                    const bool ok1[1] = {true};
                    int c1[1];
                    T.find_wide_multi<1>(lo, hi, t1, ok1, false, c1);
                    cell = c1[0];
                } else {
                    cell = T.find_or_insert(ku[u], false, false, false);
                }
                if (cell >= 0) {
                    ops.add(T, cell, v[u]);
                } else {
                    const int64_t w = (int64_t)atomicAdd(&T.ctrl->spill_w, 1ull);
                    ops.store(spill, w, v[u]);
                }
            }
        };
        if (pass == 0 && no_rows) {
            // only the bucket's older groups (seeded above) pass through
        } else if (pass == 0) {
            // chunks of CH tiles: their runs are concatenated (one packed record per run in LDS:
            // its end row | narrow << 31, and its tile offset minus its start) and row i of the
            // chunk finds its run through a sampled index, so every thread takes RT rows per step
            // whatever the run lengths (packed records vs separate entry / prefix arrays: one
            // dependent LDS read less a row, agg.bucket 0.409 -> 0.404 ms, r05d)
            for (int t0 = tbeg; t0 < tend; t0 += CH) {
                const uint32_t e = (Ops::WIDE && t0 == tbeg) ? e0 : (t0 + (int)threadIdx.x < tend ? col[t0 + threadIdx.x] : 0u);
                uint32_t r_beg, r_end; // this thread's run in chunk rows
                { // block-wide exclusive scan of the run lengths
                    const uint32_t c = e >> 16;
                    uint32_t x = c;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t y = __shfl_up(x, d, 64);
                        if ((int)(threadIdx.x & 63) >= d) x += y;
                    }
                    if ((threadIdx.x & 63) == 63) s_wsum[threadIdx.x >> 6] = x;
                    __syncthreads();
                    uint32_t off = 0;
                    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) off += s_wsum[w];
                    r_beg = off + x - c;
                    r_end = off + x;
                    s_run[threadIdx.x] = make_uint2(r_end | ((e & TILE_NARROW) ? 0x80000000u : 0u),
                                                    (uint32_t)((int)(e & 0x7FFFu) - (int)r_beg));
                    if (threadIdx.x == CH - 1) s_tot = r_end;
                }
                __syncthreads();
                const uint32_t tot = s_tot;
                // the run of row i is the first one ending past i.  A sampled index (every
                // 2^idx_sh-th row's run, as dense as IDXN allows: every row while the chunk has
                // < 2048 rows, every 16th at C2's ~31K, where runs average ~30 rows) starts each
                // row's search at most a few runs before its own: one LDS read plus a short
                // forward walk instead of a binary search (~5 dependent LDS reads and ~30 VALU a
                // row).  Sparser samples made low selectivities walk long stretches of empty runs
                // (1 %: agg.bucket 0.38 ms with a 32-row index)
                uint32_t idx_sh = 0;
                while ((tot >> idx_sh) >= (uint32_t)IDXN) ++idx_sh; // uniform
                for (uint32_t k = (r_beg + (1u << idx_sh) - 1) >> idx_sh; (k << idx_sh) < r_end; ++k)
                    s_idx[k] = (uint16_t)threadIdx.x;
                __syncthreads();
                // software pipeline: the next step's rows are loaded (address search + global
                // loads issued) before this step's LDS probe / atomics, so HBM latency overlaps
                // the table work instead of following it after every step barrier
                // (measured: a thread taking RT consecutive rows instead — one search per RT rows —
                // made the kernel slower, 0.41 -> 0.52 ms: each load instruction then spans 4x the
                // lines, and the run-crossing step diverges)
                auto load_step = [&](uint32_t base, typename Ops::Raw (&v)[RT], bool (&ok)[RT]) __attribute__((always_inline)) {
                    // the RT rows' runs are found together: their index reads, their first run
                    // reads, then forward steps for the rows past their run's end, so the
                    // dependent LDS round trips of the RT rows overlap (one 8-byte read a run)
                    uint32_t ii[RT], lo[RT];
                    uint2 run[RT];
#pragma unroll
                    for (int u = 0; u < RT; ++u) {
                        ii[u] = base + u * BT + threadIdx.x;
                        ok[u] = ii[u] < tot;
                        lo[u] = ok[u] ? s_idx[ii[u] >> idx_sh] : 0u;
                    }
#pragma unroll
                    for (int u = 0; u < RT; ++u) run[u] = s_run[lo[u]];
                    for (;;) {
                        bool walk[RT], any = false;
#pragma unroll
                        for (int u = 0; u < RT; ++u) {
                            walk[u] = ok[u] && (run[u].x & 0x7FFFFFFFu) <= ii[u];
                            lo[u] += walk[u] ? 1u : 0u;
                            any = any || walk[u];
                        }
                        if (!any) break;
#pragma unroll
                        for (int u = 0; u < RT; ++u)
                            if (walk[u]) run[u] = s_run[lo[u]];
                    }
                    // every lane issues the same loads (Ops::load_raw: no branch, no copy of a
                    // loaded register), so they stay in flight until the step that uses them.
                    // (r06o: with a load in a narrow / wide branch and the loop-carried copy of
                    // the rows, each load was waited for where it was issued — the wide kernel took
                    // 1.64 ms, 0.89 ms with synthetic rows and no loads at all)
#pragma unroll
                    for (int u = 0; u < RT; ++u) {
                        const uint32_t off = run[u].y + ii[u];
                        // the tile's slot: T * TRS rows stay below 2^32 (the ABI caps n below 2^32)
                        const uint64_t slot = (uint64_t)(uint32_t)(t0 + (int)lo[u]) * (uint32_t)tin.TR;
#ifdef TFG_EXP_NOLOAD // profiling experiment only: a synthetic row of the bucket instead of its record
                        if constexpr (Ops::WIDE) {
                            v[u].q = make_uint4((uint32_t)(b * 1000 + (int)((off * 2654435761u) % 600u)) + 1u, 0x6B000000u,
                                                9u << 24, 0u);
                            v[u].w[0] = off;
                            v[u].nar = true;
                        } else {
                            v[u].w[0] = (uint64_t)(b * 4000 + (int)((off * 2654435761u) % 3906u)) + 1u;
                            v[u].w[1] = off;
                            v[u].nar = false;
                        }
                        continue;
#endif
                        ops.load_raw(tin.rec, slot, tin.TR, off, Ops::NARROWABLE && (run[u].x >> 31), ok[u], v[u]);
                    }
                };
                auto run_step = [&](const typename Ops::Raw (&r)[RT], const bool (&okr)[RT]) __attribute__((always_inline)) {
                    typename Ops::Row v[RT];
                    bool ok[RT];
#pragma unroll
                    for (int u = 0; u < RT; ++u) {
                        ops.unraw(r[u], v[u]);
                        ok[u] = okr[u];
                    }
                    step(v, ok);
                };
                constexpr uint32_t SZ = BT * RT;
                // two register sets, alternating: the next step's rows load into the set the
                // current step does not use.  Each set has one load site, inside the loop, so
                // no loaded register is copied at the loop head (a copy waits for its load).
                // The loads are unconditional — rows past the chunk read its first record — so
                // neither set is merged at a branch's end either
                typename Ops::Raw ra[RT], rb[RT];
                bool oka[RT], okb[RT];
                bool have_b = false;
                for (uint32_t base = 0;; base += 2 * SZ) {
                    const bool have_a = base < tot;
                    load_step(base, ra, oka);
                    if (have_b) run_step(rb, okb); // the previous round's second step
                    if (!have_a) break;
                    have_b = base + SZ < tot;
                    load_step(base + SZ, rb, okb);
                    run_step(ra, oka);
                }
                __syncthreads();
            }
        } else {
            const uint32_t npend = (uint32_t)pending;
            for (uint32_t base = 0; base < npend; base += BT * RT) {
                typename Ops::Row v[RT];
                bool ok[RT];
#pragma unroll
                for (int u = 0; u < RT; ++u) {
                    const uint32_t i = base + u * BT + threadIdx.x;
                    ok[u] = i < npend;
                    if (ok[u]) ops.load(rows, i, v[u]);
                }
                step(v, ok);
            }
        }
        ++pass;
        __syncthreads();
        { // re-check this pass's spilled rows against the final table: found -> add, else keep
            // (kept rows are compacted in place; a chunk is read before any of it is rewritten)
            const uint32_t nsp = (uint32_t)T.ctrl->spill_w;
            __shared__ unsigned long long s_keep;
            if (threadIdx.x == 0) s_keep = 0;
            for (uint32_t c0 = 0; c0 < nsp; c0 += BT) {
                typename Ops::Row v1[1];
                const bool have = c0 + threadIdx.x < nsp;
                if (have) ops.load(spill, c0 + threadIdx.x, v1[0]);
                __syncthreads();
                if (have) {
                    int cell;
                    const uint64_t ku = ops.key(v1[0]);
                    if constexpr (Ops::WIDE) {
                        const uint64_t lo[1] = {ku}, hi[1] = {ops.hi(v1[0])}, t1[1] = {wide_tag(ku, ops.hi(v1[0]))};
                        const bool ok1[1] = {true};
                        int c1[1];
                        T.find_wide_multi<1>(lo, hi, t1, ok1, false, c1);
                        cell = c1[0];
                    } else {
                        cell = T.find_or_insert(ku, false, false, false);
                    }
                    if (cell >= 0) ops.add(T, cell, v1[0]);
                    else ops.store(spill, (int64_t)atomicAdd(&s_keep, 1ull), v1[0]);
                }
                __syncthreads();
            }
            if (nsp && threadIdx.x == 0) T.ctrl->spill_w = s_keep;
        }
        __syncthreads();
        T.flush(out, out_base);
        __syncthreads();
        pending = (int64_t)T.ctrl->spill_w;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out_cnt[b] = T.ctrl->out_count;
        tmp_base[b] = out_base;
    }
}

template <typename Ops> struct OpsTag { using type = Ops; };

template <typename Ops>
void launch_bucket_one(int B, const AggSpec &S, hipStream_t st, const RowsIO &rows, const RowsIO &rows1, int mode,
                       const uint64_t *stage_off, const GroupsIO &old, const uint64_t *ooff, const GroupsIO &tmp,
                       uint64_t *new_cnt) {
    if (S.bt == BT_BIG)
        hipLaunchKernelGGL((agg_bucket_kernel<Ops, BT_BIG>), dim3(B), dim3(BT_BIG), S.lds_bytes, st, S, rows, rows1, mode,
                           stage_off, old, ooff, tmp, new_cnt);
    else
        hipLaunchKernelGGL((agg_bucket_kernel<Ops, BT>), dim3(B), dim3(BT), S.lds_bytes, st, S, rows, rows1, mode,
                           stage_off, old, ooff, tmp, new_cnt);
}

template <typename Ops>
void launch_bucket_one_tiled(int B, const AggSpec &S, hipStream_t st, const TiledIn &tin, int mode, const GroupsIO &old,
                             const uint64_t *ooff, const GroupsIO &tmp, uint64_t *new_cnt, uint64_t *tmp_base) {
    if (S.bt == BT_BIG)
        hipLaunchKernelGGL((agg_bucket_tiled_kernel<Ops, BT_BIG>), dim3(B), dim3(BT_BIG), S.lds_bytes, st, S, tin, mode,
                           old, ooff, tmp, new_cnt, tmp_base);
    else
        hipLaunchKernelGGL((agg_bucket_tiled_kernel<Ops, BT>), dim3(B), dim3(BT), S.lds_bytes, st, S, tin, mode, old,
                           ooff, tmp, new_cnt, tmp_base);
}

// calls f(OpsTag<FastOps<...>>{}) for the op-code `fast` of fast_signature; false for other codes
template <typename F> bool with_fast_ops(int fast, F &&f) {
    switch (fast) {
    case 310: f(OpsTag<FastOps<3, 1, 0>>{}); return true;
    case 210: f(OpsTag<FastOps<2, 1, 0>>{}); return true;
    case 410: f(OpsTag<FastOps<4, 1, 0>>{}); return true;
    case 300: f(OpsTag<FastOps<3, 0, 0>>{}); return true;
    case 200: f(OpsTag<FastOps<2, 0, 0>>{}); return true;
    case 400: f(OpsTag<FastOps<4, 0, 0>>{}); return true;
    case 100: f(OpsTag<FastOps<1, 0, 0>>{}); return true;
    case 231: f(OpsTag<FastOps<2, 3, 1>>{}); return true;
    case 221: f(OpsTag<FastOps<2, 2, 1>>{}); return true;
    case 331: f(OpsTag<FastOps<3, 3, 1>>{}); return true;
    case 441: f(OpsTag<FastOps<4, 4, 1>>{}); return true;
    default: return false;
    }
}

// true for the op-codes with a FastOps specialisation (with_fast_ops); any other code must take
// the generic path from the start (its rows are staged columnar, not as FastOps records)
inline bool fast_code_supported(int fast) {
    switch (fast) {
    case 310: case 210: case 410: case 300: case 200: case 400: case 100: case 231: case 221: case 331: case 441:
        return true;
    default:
        return false;
    }
}

// Bucket kernel launches per row-policy family (agg_bucket_fast.hip, agg_bucket_wide.hip,
// agg_bucket_generic.hip).  false: the code names no specialisation of that family.
bool launch_bucket_fast(int fast, int B, const AggSpec &S, hipStream_t st, const RowsIO &rows, const RowsIO &rows1,
                        int mode, const uint64_t *stage_off, const GroupsIO &old, const uint64_t *ooff,
                        const GroupsIO &tmp, uint64_t *new_cnt);
bool launch_bucket_fast_tiled(int fast, int B, const AggSpec &S, hipStream_t st, const TiledIn &tin, int mode,
                              const GroupsIO &old, const uint64_t *ooff, const GroupsIO &tmp, uint64_t *new_cnt,
                              uint64_t *tmp_base);
bool launch_bucket_wide_tiled(int code, int B, const AggSpec &S, hipStream_t st, const TiledIn &tin, int mode,
                              const GroupsIO &old, const uint64_t *ooff, const GroupsIO &tmp, uint64_t *new_cnt,
                              uint64_t *tmp_base);
// WideOps (key_width 16) or GenericOps over n_aggs aggregates; w256: a Decimal256 sum
void launch_bucket_generic(bool wide, bool w256, int B, const AggSpec &S, hipStream_t st, const RowsIO &rows,
                           const RowsIO &rows1, int mode, const uint64_t *stage_off, const GroupsIO &old,
                           const uint64_t *ooff, const GroupsIO &tmp, uint64_t *new_cnt);

} // namespace tfg
