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
#include <type_traits>

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
    int key0; // column 0 holds the 8-byte key the selector loads (its staged copy reuses that load)
    int aos;  // all columns 8 bytes, written as interleaved records of ncols words at out[0]
    int in_stride;            // > 1: the 8-byte input columns are words of records of this many words
    const uint32_t *perm_in;  // staged path: perm output = perm_in[row] instead of row
    int two_pass;             // the caller's tmp holds part_tmp_bytes(L, row_bytes, perm): large P may
                              // run as two radix passes (64 wide, then the full radix)
};

// Key columns hashed with IColumn::updateWeakHash32 semantics.
struct KeyCols {
    const void *col[4];
    const uint8_t *nullmap[4];
    int type[4];
    int nkeys;
};

// Float -> UInt64 as the reference's implicit conversion (intHashCRC32(UInt64, UInt32) called with
// a Float, Columns/ColumnVector.cpp:528) compiles on x86-64 (clang, SSE4.2, no AVX-512):
// cvttsd2si(x) | (cvttsd2si(x - 2^63) & (cvttsd2si(x) >> 63)), where cvttsd2si yields INT64_MIN
// for NaN and out-of-range values.  Pinned by tests/golden/float_weak_hash.json.
template <typename F> __device__ __forceinline__ int64_t cvtt_i64(F x) {
    return (x >= (F)-9223372036854775808.0 && x < (F)9223372036854775808.0) ? (int64_t)x : INT64_MIN;
}
template <typename F> __device__ __forceinline__ uint64_t float_to_u64_x86(F x) {
    const int64_t a = cvtt_i64<F>(x);
    const int64_t b = cvtt_i64<F>(x - (F)9223372036854775808.0);
    return (uint64_t)(a | (b & (a >> 63)));
}

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
        case TFG_FLOAT32: h = crc32c_u64(t, h, float_to_u64_x86(((const float *)c)[r])); break;
        case TFG_FLOAT64: h = crc32c_u64(t, h, float_to_u64_x86(((const double *)c)[r])); break;
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
// A selector maps a row to its partition (0xFFFFFFFF drops the row).  The work is split into
// load(r) — the global loads — and part(crc, loaded, r), so kernels can issue the loads of
// many rows before any of them is consumed (memory-level parallelism).
constexpr uint32_t TWO_PASS_MIN = 1024; // P above this partitions in two passes (see run_two_pass)
constexpr uint32_t TWO_PASS_P1 = 64;

// Internal radix of a key (aggregation buckets, join partitions): Fibonacci hashing, the top
// `bits` bits of key * 2^64/phi.  These radices never leave the device (unlike the exchange
// selector, which must reproduce fillSelector's CRC32-C routing), so a one-multiply hash
// replaces the eight LDS table lookups of the CRC.
__device__ __forceinline__ uint32_t fib_part(uint64_t key, uint32_t shift) {
    return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 32 >> shift); // shift = 32 - bits (32 -> 0)
}
inline uint32_t fib_shift(uint32_t parts) { // parts is a power of two
    uint32_t b = 0;
    while ((1u << b) < parts) ++b;
    return 32 - b;
}

struct Loaded {
    uint64_t bits;
    uint32_t null;
    uint64_t hi = 0; // wide-key selectors: the key's second word
};

// A selector with `static constexpr bool wide_key = true` loads a 16-byte key (Loaded::bits,
// Loaded::hi) that becomes words 0 and 1 of the staged records.
template <typename S, typename = void> struct SelWideKey : std::false_type {};
template <typename S> struct SelWideKey<S, std::void_t<decltype(S::wide_key)>> : std::integral_constant<bool, S::wide_key> {};

__device__ __forceinline__ uint64_t load_width(const void *p, int width, int64_t i) {
    switch (width) {
    case 1: return ((const uint8_t *)p)[i];
    case 2: return ((const uint16_t *)p)[i];
    case 4: return ((const uint32_t *)p)[i];
    default: return ((const uint64_t *)p)[i];
    }
}

struct SelArray {
    const uint32_t *sel;
    static constexpr bool needs_crc = false;
    static constexpr bool fib_radix = false;
    __device__ __forceinline__ Loaded load(int64_t r) const { return Loaded{sel[r], 0}; }
    __device__ __forceinline__ uint32_t part(const uint32_t (*)[256], const Loaded &l, int64_t) const {
        return (uint32_t)l.bits;
    }
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const { return part(t, load(r), r); }
};

// fillSelector over the weak hash of key columns: part = (UInt64(h) * P) >> 32
struct SelHashMul {
    KeyCols k;
    uint32_t parts;
    static constexpr bool needs_crc = true;
    static constexpr bool fib_radix = false;
    __device__ __forceinline__ Loaded load(int64_t) const { return Loaded{0, 0}; }
    __device__ __forceinline__ uint32_t part(const uint32_t (*t)[256], const Loaded &, int64_t r) const {
        uint32_t h = hash_key_row(t, k, r, 0xFFFFFFFFu);
        return (uint32_t)(((uint64_t)h * parts) >> 32);
    }
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const { return part(t, load(r), r); }
};

// second pass of a two-pass radix partition: the key is word 0 of the first pass's records
struct SelRec8 {
    const uint64_t *rec;
    int stride; // record words
    uint32_t shift;
    static constexpr bool needs_crc = false;
    static constexpr bool fib_radix = false; // already the second pass
    __device__ __forceinline__ Loaded load(int64_t r) const { return Loaded{rec[r * stride], 0u}; }
    __device__ __forceinline__ uint32_t part(const uint32_t (*)[256], const Loaded &l, int64_t) const {
        return fib_part(l.bits, shift);
    }
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const { return part(t, load(r), r); }
};

// Per-row predicate: `pred_col Op scalar` (nullable -> drop), or a UInt8 mask, or none.
struct RowPred {
    int kind; // 0 none, 1 mask, 2 compare
    int type;
    const void *col;
    const uint8_t *nullmap;
    Num b;
    int op;
    __device__ __forceinline__ Loaded load(int64_t r) const {
        Loaded l{0, 0};
        if (kind == 0) return l;
        l.bits = kind == 1 ? ((const uint8_t *)col)[r] : load_width(col, (int)type_width_dev(type), r);
        if (nullmap) l.null = nullmap[r];
        return l;
    }
    __device__ static size_t type_width_dev(int t) {
        switch (t) {
        case TFG_INT8: case TFG_UINT8: return 1;
        case TFG_INT16: case TFG_UINT16: return 2;
        case TFG_INT32: case TFG_UINT32: case TFG_FLOAT32: return 4;
        default: return 8;
        }
    }
    __device__ __forceinline__ bool eval(const Loaded &l) const {
        if (kind == 0) return true;
        if (l.null) return false;
        if (kind == 1) return l.bits != 0;
        switch (type) {
        case TFG_INT8: return cmp_value_num<int8_t>((int8_t)l.bits, b, op);
        case TFG_INT16: return cmp_value_num<int16_t>((int16_t)l.bits, b, op);
        case TFG_INT32: return cmp_value_num<int32_t>((int32_t)l.bits, b, op);
        case TFG_INT64: return cmp_value_num<int64_t>((int64_t)l.bits, b, op);
        case TFG_UINT8: return cmp_value_num<uint8_t>((uint8_t)l.bits, b, op);
        case TFG_UINT16: return cmp_value_num<uint16_t>((uint16_t)l.bits, b, op);
        case TFG_UINT32: return cmp_value_num<uint32_t>((uint32_t)l.bits, b, op);
        case TFG_UINT64: return cmp_value_num<uint64_t>(l.bits, b, op);
        case TFG_FLOAT32: return cmp_value_num<float>(__uint_as_float((unsigned)l.bits), b, op);
        default: return cmp_value_num<double>(__longlong_as_double((long long)l.bits), b, op);
        }
    }
    __device__ __forceinline__ bool operator()(int64_t r) const { return eval(load(r)); }
};

// Compile-time specialised predicates for the hot cases (no per-row type switch):
// KIND 0 = none, 1 = UInt8 mask, 2 = `T col Op scalar`.
template <int KIND, typename T = int64_t, bool NULLS = true> struct PredT {
    const void *col;
    const uint8_t *nullmap;
    Num b;
    int op;
    __device__ __forceinline__ Loaded load(int64_t r) const {
        Loaded l{0, 0};
        if constexpr (KIND == 1) l.bits = ((const uint8_t *)col)[r];
        if constexpr (KIND == 2) {
            T x = ((const T *)col)[r];
            uint64_t bits = 0;
            memcpy(&bits, &x, sizeof(T));
            l.bits = bits;
        }
        if constexpr (KIND != 0 && NULLS)
            if (nullmap) l.null = nullmap[r];
        return l;
    }
    __device__ __forceinline__ bool eval(const Loaded &l) const {
        if constexpr (KIND == 0) return true;
        if constexpr (NULLS)
            if (l.null) return false;
        if constexpr (KIND == 1) return l.bits != 0;
        else {
            T x;
            memcpy(&x, &l.bits, sizeof(T));
            return cmp_value_num<T>(x, b, op);
        }
    }
    __device__ __forceinline__ bool operator()(int64_t r) const { return eval(load(r)); }
};

// Calls f(pred) with the most specialised predicate type for `p`.
template <typename F> int with_pred(const RowPred &p, F &&f) {
    if (p.kind == 0) return f(PredT<0>{nullptr, nullptr, p.b, p.op});
    if (p.nullmap) return f(p); // nullable predicate columns: the generic evaluator
    if (p.kind == 1) return f(PredT<1, int64_t, false>{p.col, nullptr, p.b, p.op});
    switch (p.type) {
    case TFG_INT64: return f(PredT<2, int64_t, false>{p.col, nullptr, p.b, p.op});
    case TFG_INT32: return f(PredT<2, int32_t, false>{p.col, nullptr, p.b, p.op});
    case TFG_FLOAT64: return f(PredT<2, double, false>{p.col, nullptr, p.b, p.op});
    default: return f(p);
    }
}

// Plain `T col Op scalar` predicates (4- or 8-byte T, no null map): a tile can be checked for
// "keeps no row" with 16-byte vector loads of the column (part_scatter_staged_kernel's skip-ahead)
template <typename P> struct PredVec {
    static constexpr bool ok = false;
    using E = uint64_t;
};
template <typename T> struct PredVec<PredT<2, T, false>> {
    static constexpr bool ok = sizeof(T) == 4 || sizeof(T) == 8;
    using E = T;
};
template <typename Pred> __device__ __forceinline__ bool pred_vec_aligned(const Pred &p, uint32_t begin) {
    if constexpr (PredVec<Pred>::ok) {
        using E = typename PredVec<Pred>::E;
        return (((uintptr_t)p.col + (uintptr_t)begin * sizeof(E)) & 15) == 0;
    } else {
        return false;
    }
}
// does any of the rows [tb, tb + per * ST_T) pass?  Thread t reads 16-byte words t, t + ST_T, ...
// of the tile, all in flight together (ST_T: the staged scatter's workgroup size, below)
template <int ST, int MAXR, typename Pred> __device__ __forceinline__ bool tile_any_vec(const Pred &p, uint32_t tb, int per) {
    if constexpr (PredVec<Pred>::ok) {
        using E = typename PredVec<Pred>::E;
        constexpr int EPW = 16 / (int)sizeof(E);
        constexpr int WMAX = (MAXR + EPW - 1) / EPW;
        const uint4 *w = reinterpret_cast<const uint4 *>(reinterpret_cast<const E *>(p.col) + tb);
        const uint32_t words = (uint32_t)per * (uint32_t)(ST / EPW);
        // all of a thread's words in flight at once (the sparse variant only: its spills are off
        // the path it is chosen for)
        constexpr int WB = WMAX;
        bool any = false;
#pragma unroll
        for (int k0 = 0; k0 < WMAX; k0 += WB) {
            uint4 x[WB];
#pragma unroll
            for (int k = 0; k < WB; ++k) {
                const uint32_t i = (uint32_t)(k0 + k) * ST + threadIdx.x;
                if (k0 + k < WMAX && i < words) x[k] = w[i];
            }
#pragma unroll
            for (int k = 0; k < WB; ++k) {
                if (k0 + k >= WMAX || (uint32_t)(k0 + k) * ST + threadIdx.x >= words) continue;
                uint64_t b[4];
                int nb;
                if constexpr (sizeof(E) == 8) {
                    b[0] = (uint64_t)x[k].x | ((uint64_t)x[k].y << 32);
                    b[1] = (uint64_t)x[k].z | ((uint64_t)x[k].w << 32);
                    nb = 2;
                } else {
                    b[0] = x[k].x, b[1] = x[k].y, b[2] = x[k].z, b[3] = x[k].w;
                    nb = 4;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (q >= nb) break;
                    Loaded l{b[q], 0u};
                    any |= p.eval(l);
                }
            }
            if (any) break;
        }
        return any;
    } else {
        return true;
    }
}

// tile_any_vec for NTL consecutive tiles from tb together (NTL x the words in flight)
template <int ST, int MAXR, int NTL, typename Pred>
__device__ __forceinline__ void tile_any_vecn(const Pred &p, uint32_t tb, int per, uint32_t tr, bool (&any)[NTL]) {
#pragma unroll
    for (int t = 0; t < NTL; ++t) any[t] = true;
    if constexpr (PredVec<Pred>::ok) {
        using E = typename PredVec<Pred>::E;
        constexpr int EPW = 16 / (int)sizeof(E);
        constexpr int WMAX = (MAXR + EPW - 1) / EPW;
        const uint32_t words = (uint32_t)per * (uint32_t)(ST / EPW);
        uint4 x[NTL][WMAX];
#pragma unroll
        for (int t = 0; t < NTL; ++t) {
            const uint4 *w = reinterpret_cast<const uint4 *>(reinterpret_cast<const E *>(p.col) + tb + (uint32_t)t * tr);
#pragma unroll
            for (int k = 0; k < WMAX; ++k) {
                const uint32_t i = (uint32_t)k * ST + threadIdx.x;
                if (i < words) x[t][k] = w[i];
            }
        }
#pragma unroll
        for (int t = 0; t < NTL; ++t) {
            bool a = false;
#pragma unroll
            for (int k = 0; k < WMAX; ++k) {
                if ((uint32_t)k * ST + threadIdx.x >= words) continue;
                uint64_t b[4];
                int nb;
                if constexpr (sizeof(E) == 8) {
                    b[0] = (uint64_t)x[t][k].x | ((uint64_t)x[t][k].y << 32);
                    b[1] = (uint64_t)x[t][k].z | ((uint64_t)x[t][k].w << 32);
                    nb = 2;
                } else {
                    b[0] = x[t][k].x, b[1] = x[t][k].y, b[2] = x[t][k].z, b[3] = x[t][k].w;
                    nb = 4;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (q >= nb) break;
                    Loaded l{b[q], 0u};
                    a |= p.eval(l);
                }
            }
            any[t] = a;
        }
    }
}

struct PartLayout {
    int64_t n;
    int64_t seg;   // rows per segment (multiple of PT)
    unsigned G;    // segments = scatter workgroups
    uint32_t P;    // partitions
    unsigned sub = 1;   // histogram workgroups per segment (> 1: counts accumulated atomically)
    int64_t subseg = 0; // rows per histogram workgroup (multiple of PT)
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
    L.sub = 1;
    L.subseg = seg;
    return L;
}

// Layout of the LDS-staged scatter: `mult` long segments per CU (default 1), so
// a destination's rows from one workgroup form a single long run (consecutive tiles continue
// each other's partially written cache lines while they are still in L2) and the P x G count
// table stays small; the histogram pass splits each segment over `sub` workgroups to keep the
// chip full.
inline PartLayout make_wide_layout(int64_t n, uint32_t P, int cu_count, unsigned gmax, int mult = 1) {
    PartLayout L;
    L.n = n;
    L.P = P;
    int64_t g = std::min<int64_t>((int64_t)cu_count * mult, gmax);
    if (g < 1) g = 1;
    int64_t seg = (n + g - 1) / g;
    seg = std::max<int64_t>((seg + PT - 1) / PT * PT, PT);
    g = std::max<int64_t>((n + seg - 1) / seg, 1);
    L.seg = seg;
    L.G = (unsigned)g;
    int64_t sub = std::max<int64_t>(1, 2048 / g);
    int64_t subseg = (seg + sub - 1) / sub;
    subseg = std::max<int64_t>((subseg + PT - 1) / PT * PT, (int64_t)8 * PT);
    L.subseg = std::min(subseg, seg);
    L.sub = (unsigned)((seg + L.subseg - 1) / L.subseg);
    return L;
}

template <typename Sel, typename Pred>
__global__ void __launch_bounds__(PT) part_hist_kernel(Sel sel, Pred pred, PartLayout L, uint32_t *counts) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[]; // P entries (+ crc tables)
    uint32_t(*crc)[256] = reinterpret_cast<uint32_t(*)[256]>(hist + ((L.P + 3) & ~3u));
    for (uint32_t p = threadIdx.x; p < L.P; p += PT) hist[p] = 0;
    if constexpr (Sel::needs_crc) load_crc_lds(crc);
    __syncthreads();
    const unsigned g = blockIdx.x / L.sub, sg = blockIdx.x % L.sub;
    const int64_t begin = (int64_t)g * L.seg + (int64_t)sg * L.subseg;
    int64_t end = std::min<int64_t>(begin + L.subseg, (int64_t)g * L.seg + L.seg);
    if (end > L.n) end = L.n;
    int64_t r = begin + threadIdx.x;
    constexpr int U = 8;
    for (; r + (U - 1) * PT < end; r += U * PT) { // U rows' loads in flight per thread, then compute
        Loaded pl[U], kl[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            pl[u] = pred.load(r + u * PT);
            kl[u] = sel.load(r + u * PT);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t p = pred.eval(pl[u]) ? sel.part(crc, kl[u], r + u * PT) : 0xFFFFFFFFu;
            if (p < L.P) atomicAdd(&hist[p], 1u);
        }
    }
    for (; r < end; r += PT) {
        if (!pred(r)) continue;
        uint32_t p = sel(crc, r);
        if (p < L.P) atomicAdd(&hist[p], 1u);
    }
    __syncthreads();
    if (L.sub == 1) {
        for (uint32_t p = threadIdx.x; p < L.P; p += PT) counts[(int64_t)p * L.G + g] = hist[p];
    } else {
        for (uint32_t p = threadIdx.x; p < L.P; p += PT)
            if (hist[p]) atomicAdd(&counts[(int64_t)p * L.G + g], hist[p]);
    }
}

__device__ __forceinline__ void scatter_row(const PCols &cols, int64_t r, uint64_t pos) {
    const int64_t ri = cols.in_stride > 1 ? r * cols.in_stride : r; // 8-byte columns of records
    if (cols.aos) {
        for (int j = 0; j < cols.ncols; ++j)
            ((uint64_t *)cols.out[0])[pos * cols.ncols + j] = ((const uint64_t *)cols.in[j])[ri];
        return;
    }
    if (cols.in_stride > 1) {
        for (int j = 0; j < cols.ncols; ++j) ((uint64_t *)cols.out[j])[pos] = ((const uint64_t *)cols.in[j])[ri];
        return;
    }
    for (int j = 0; j < cols.ncols; ++j) {
        switch (cols.width[j]) {
        case 1: ((uint8_t *)cols.out[j])[pos] = ((const uint8_t *)cols.in[j])[r]; break;
        case 2: ((uint16_t *)cols.out[j])[pos] = ((const uint16_t *)cols.in[j])[r]; break;
        case 4: ((uint32_t *)cols.out[j])[pos] = ((const uint32_t *)cols.in[j])[r]; break;
        case 8: ((uint64_t *)cols.out[j])[pos] = ((const uint64_t *)cols.in[j])[r]; break;
        case 32: // Decimal256 sums (two-phase aggregation states)
            ((uint4 *)cols.out[j])[2 * pos] = ((const uint4 *)cols.in[j])[2 * r];
            ((uint4 *)cols.out[j])[2 * pos + 1] = ((const uint4 *)cols.in[j])[2 * r + 1];
            break;
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
            if (perm) perm[pos] = cols.perm_in ? cols.perm_in[r] : (uint32_t)r;
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
                if (perm) perm[pos] = cols.perm_in ? cols.perm_in[r] : (uint32_t)r;
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
inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }
inline uint32_t bits_of_pow2(uint32_t p) {
    uint32_t b = 0;
    while ((1u << b) < p) ++b;
    return b;
}
// ... plus, for callers that set PCols::two_pass, the first pass's records (row_bytes per row),
// row ids and offsets
inline size_t part_tmp_bytes(const PartLayout &L, size_t row_bytes, bool perm) {
    size_t b = part_tmp_bytes(L);
    if (L.P > TWO_PASS_MIN && row_bytes)
        b += align256((size_t)L.n * row_bytes) + (perm ? align256((size_t)L.n * 4) : 0) + align256((TWO_PASS_P1 + 1) * 8);
    return b;
}

__global__ void gather_part_offsets_kernel(const uint64_t *offs, PartLayout L, uint64_t *out);

// ---------------------------------------------------------------- LDS-staged scatter
// Scattering rows one by one into P >= 256 destinations leaves each wave store instruction
// touching ~64 different cache lines (measured ~0.8 TB/s).  The staged form counting-sorts a
// tile of TR rows by destination in LDS first (LDS atomics give each row its rank inside its
// destination), then streams the sorted tile out: consecutive lanes write consecutive
// addresses of one destination run, so stores coalesce into runs of TR/P rows.
constexpr int ST_T = 1024;     // threads (16 waves)
constexpr uint32_t TILE_NARROW = 0x8000u; // tile_hist start bit: the tile holds narrow records
// narrow 16-byte keys (WNARROW tiles): bytes 11-14 zero, so the high word keeps bytes 8-10 and the
// length / NULL byte 15 in 32 bits
__host__ __device__ __forceinline__ bool wide_hi_narrowable(uint64_t hi) { return ((hi >> 24) & 0xFFFFFFFFull) == 0; }
__host__ __device__ __forceinline__ uint32_t wide_narrow_hi(uint64_t hi) {
    return (uint32_t)(hi & 0xFFFFFFull) | ((uint32_t)(hi >> 56) << 24);
}
__host__ __device__ __forceinline__ uint64_t wide_wide_hi(uint32_t h) {
    return (uint64_t)(h & 0xFFFFFFu) | ((uint64_t)(h >> 24) << 56);
}
// A narrow tile's rows are 20-byte records back to back from the slot's start: key lo (2 words),
// narrow hi (1 word), value (2 words), 4-byte aligned.  A run of n rows is then one stretch of 20n
// bytes; as three arrays (u64 lo [TRS], u32 hi [TRS], u64 value [TRS]) every run began and ended
// inside a partly used line of each array, and the readers fetched 1.8x the records' bytes
// (C5: bucket kernel 3.65 GB and regroup 3.61 GB for 2.0 GB of records, r06j)
__device__ __forceinline__ void nrec_store(uint64_t *slot, uint32_t pos, uint64_t lo, uint32_t hi, uint64_t val) {
    uint32_t *p = reinterpret_cast<uint32_t *>(slot) + (size_t)pos * 5;
    p[0] = (uint32_t)lo;
    p[1] = (uint32_t)(lo >> 32);
    p[2] = hi;
    p[3] = (uint32_t)val;
    p[4] = (uint32_t)(val >> 32);
}
__device__ __forceinline__ void nrec_load(const uint64_t *slot, uint32_t pos, uint64_t &lo, uint32_t &hi, uint64_t &val) {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(slot) + (size_t)pos * 5;
    const uint32_t a = p[0], b = p[1], c = p[2], d = p[3], e = p[4];
    lo = (uint64_t)a | ((uint64_t)b << 32);
    hi = c;
    val = (uint64_t)d | ((uint64_t)e << 32);
}
constexpr int ST_MAXR = 8;     // rows per thread per tile (TR <= 8192 < 2^16: ranks pack in 16 bits)
// tiles a round in the sparse variant's all-false check (four measured slower: 0 % C2 0.364 vs
// 0.344 ms, r05ad — not memory-level parallelism but the per-round barriers bound it)
constexpr int SKIP_NT = 2;
constexpr int FLAG_TPS_MAX = 512; // tiles a segment may have for the tile-flag pre-pass

// tile_flags[g * tps + k] = does tile k of segment g keep a row?  One 256-thread workgroup a tile,
// its predicate words read as 16-byte vectors (a full, aligned tile) or row by row, all in flight
// together: the predicate column streams at HBM rate across the whole chip (the partition kernel,
// one workgroup a CU walking its tiles in turn, reads it at ~3.3 TB/s)
constexpr int TF_T = 256;
template <typename Pred>
__global__ void __launch_bounds__(TF_T) tile_flags_kernel(Pred pred, PartLayout L, int TR, int tps, uint8_t *flags) {
    const uint32_t gseg = blockIdx.x / (uint32_t)tps, k = blockIdx.x % (uint32_t)tps;
    const int64_t begin = (int64_t)gseg * L.seg, end = std::min<int64_t>(begin + L.seg, L.n);
    const int64_t tb = begin + (int64_t)k * TR, te = std::min<int64_t>(tb + TR, end);
    bool any = false;
    if (tb < te) {
        if constexpr (PredVec<Pred>::ok) {
            using E = typename PredVec<Pred>::E;
            constexpr int EPW = 16 / (int)sizeof(E);
            const E *col = reinterpret_cast<const E *>(pred.col);
            const bool vec = ((((uintptr_t)(col + tb)) & 15) == 0);
            const int64_t nv = vec ? (te - tb) / EPW : 0; // whole 16-byte words
            const uint4 *w = reinterpret_cast<const uint4 *>(col + tb);
            constexpr int WB = 8;
            for (int64_t i0 = threadIdx.x; i0 < nv && !any; i0 += (int64_t)WB * TF_T) {
                uint4 x[WB];
#pragma unroll
                for (int q = 0; q < WB; ++q)
                    if (i0 + (int64_t)q * TF_T < nv) x[q] = w[i0 + (int64_t)q * TF_T];
#pragma unroll
                for (int q = 0; q < WB; ++q) {
                    if (i0 + (int64_t)q * TF_T >= nv) continue;
                    uint64_t b[4];
                    int nb;
                    if constexpr (sizeof(E) == 8) {
                        b[0] = (uint64_t)x[q].x | ((uint64_t)x[q].y << 32);
                        b[1] = (uint64_t)x[q].z | ((uint64_t)x[q].w << 32);
                        nb = 2;
                    } else {
                        b[0] = x[q].x, b[1] = x[q].y, b[2] = x[q].z, b[3] = x[q].w;
                        nb = 4;
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        if (e >= nb) break;
                        Loaded l{b[e], 0u};
                        any |= pred.eval(l);
                    }
                }
            }
            for (int64_t r = tb + nv * EPW + threadIdx.x; r < te; r += TF_T) any |= pred.eval(pred.load(r));
        } else {
            for (int64_t r = tb + threadIdx.x; r < te; r += TF_T) any |= pred.eval(pred.load(r));
        }
    }
    any = __syncthreads_or(any);
    if (threadIdx.x == 0) flags[blockIdx.x] = any ? 1 : 0;
}

struct StagedGeom {
    int TR;          // rows per tile (multiple of ST_T)
    int stage_off[PCOLS];
    int perm_off;
    int crc_off;
    int red_off;
    int lds_bytes;
    // tile-sorted mode (TILED kernels): tile k of segment g is written, sorted by destination, to
    // rows [(g * tps + k) * TR, + kept) of the output, and tile_hist[p * T + tile] receives the
    // destination's start inside the tile | its row count << 16
    uint32_t *tile_hist;
    int tps; // tiles per segment
    int T;   // tiles
    // TILED: runs may be padded to `align` records inside a tile (a tile slot is then
    // TRS = TR + (align - 1) * P rows); make_tiled_geom keeps them dense (align 1)
    int align;
    int TRS;
    // TILED two-level form: the selector returns a (P << fine_bits)-way radix; the tile is sorted
    // by its top bits (radix >> fine_bits) and every workgroup adds its rows' full radices into
    // fine_counts (LDS histogram at fh_off, one global atomic per non-zero bin at the end)
    int fine_bits;
    int fh_off;
    uint32_t *fine_counts;
    // TILED: two words the next kernel (the bucket kernel's cursors) needs zeroed — written by
    // workgroup 0 here instead of by a memset launch of their own
    unsigned long long *zero2;
    // VSKIP with flags: tile_flags[t] = tile t keeps a row (tile_flags_kernel, a pass of its own
    // over the predicate column with every workgroup of the chip), so all-false tiles are skipped
    // without reading a word of theirs in this kernel
    const uint8_t *tile_flags;
    int allow_narrow; // TILED narrow tiles (u32 keys) permitted: consumers that read records
                      // word by word (regroup_scatter_kernel) need the wide form
};

// LDS bytes a staged-scatter workgroup uses: one workgroup per CU.
constexpr size_t STAGE_LDS_BUDGET = (size_t)150 * 1024;

inline bool make_staged_geom(uint32_t P, const PCols &cols, bool perm, bool crc, StagedGeom &g, int fine_bits = 0) {
    if (P > 4096) return false;
    size_t row_bytes = 2 + (perm ? 4 : 0);
    for (int j = 0; j < cols.ncols; ++j) row_bytes += cols.width[j];
    const size_t fh_bytes = fine_bits ? ((size_t)P << fine_bits) * 4 : 0;
    const size_t fixed = (size_t)P * 16 + (crc ? 8192 : 0) + 16 * (PCOLS + 2) + fh_bytes;
    const size_t budget = STAGE_LDS_BUDGET; // LDS per workgroup (default: one workgroup per CU)
    if (fixed + row_bytes * ST_T * 2 > budget) return false;
    int tr = (int)((budget - fixed) / row_bytes) / ST_T * ST_T;
    if (tr > ST_T * ST_MAXR) tr = ST_T * ST_MAXR;
    g.TR = tr;
    g.align = 1;
    g.TRS = tr;
    size_t off = (size_t)P * 16 + (size_t)tr * 2;
    off = (off + 15) & ~size_t(15);
    for (int j = 0; j < cols.ncols; ++j) {
        g.stage_off[j] = (int)off;
        off += ((size_t)tr * cols.width[j] + 15) & ~size_t(15);
    }
    g.perm_off = (int)off;
    if (perm) off += (size_t)tr * 4;
    g.crc_off = (int)((off + 15) & ~size_t(15));
    g.red_off = g.crc_off + (crc ? 8192 : 0);
    g.fh_off = g.red_off + (ST_T / 64 + 2) * 4; // red[]: per-wave sums + the tile total
    g.fine_bits = fine_bits;
    g.fine_counts = nullptr;
    g.zero2 = nullptr;
    g.tile_flags = nullptr;
    g.allow_narrow = 1;
    g.lds_bytes = g.fh_off + (int)fh_bytes;
    return true;
}

// NC8 > 0: compile-time fast path for exactly NC8 columns of 8 bytes (keys, payloads); the
// column loops unroll and no per-row width switch remains.  NC8 == 0: any widths.
template <typename Sel, typename Pred, int NC8, bool AOS = false, bool TILED = false, bool VSKIP = false>
__global__ void __launch_bounds__(ST_T, 4) part_scatter_staged_kernel(Sel sel, Pred pred, PartLayout L,
                                                                   const uint64_t *offs, PCols cols, uint32_t *perm,
                                                                   StagedGeom g) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const uint32_t P = L.P;
    uint64_t *run = reinterpret_cast<uint64_t *>(lds);
    uint32_t *pstart = reinterpret_cast<uint32_t *>(lds); // TILED: padded run starts (run[] is unused)
    uint32_t *hist = reinterpret_cast<uint32_t *>(run + P);
    uint32_t *start = hist + P;
    uint16_t *sb = reinterpret_cast<uint16_t *>(start + P);
    uint32_t *sperm = reinterpret_cast<uint32_t *>(lds + g.perm_off);
    uint32_t(*crc)[256] = reinterpret_cast<uint32_t(*)[256]>(lds + g.crc_off);
    uint32_t *red = reinterpret_cast<uint32_t *>(lds + g.red_off); // ST_T/64 + 1 words
    if constexpr (!TILED)
        for (uint32_t p = threadIdx.x; p < P; p += ST_T) run[p] = offs[(int64_t)p * L.G + blockIdx.x];
    if constexpr (TILED)
        if (g.zero2 && blockIdx.x == 0 && threadIdx.x < 2) g.zero2[threadIdx.x] = 0ull;
    if constexpr (Sel::needs_crc) load_crc_lds(crc);
    // row indices fit 32 bits (the ABI caps n below 2^32)
    const uint32_t begin = (uint32_t)((int64_t)blockIdx.x * L.seg);
    const uint32_t end = (uint32_t)std::min<int64_t>((int64_t)begin + L.seg, L.n);
    const int per = g.TR / ST_T;
    const int ncols = NC8 > 0 ? NC8 : cols.ncols;
    // narrow tiles (TILED {key, value} records of an 8-byte key): a tile whose kept keys all fit
    // 32 bits is written as a u32 key array + a u64 value array (12 B a row instead of 16), and
    // its tile_hist entries carry TILE_NARROW; red[ST_T / 64 + 1] collects "a wide key was seen"
    constexpr bool NARROW = TILED && AOS && NC8 == 2 && !SelWideKey<Sel>::value;
    // ... and of a 16-byte key + one value word (keys128 / key_string with one summed argument): a
    // tile whose kept keys all have bytes 11-14 zero (<= 11 key bytes: every k%08d String key) is
    // written as u64 key lo [TRS], u32 key hi [TRS] (bytes 8-10 and 15), u64 value [TRS]: 20 B a
    // row instead of 24 (wide_narrow_hi / wide_wide_hi convert)
    constexpr bool WNARROW = TILED && AOS && NC8 == 3 && SelWideKey<Sel>::value;
    uint32_t *fh = reinterpret_cast<uint32_t *>(lds + g.fh_off); // TILED && fine_bits: P << fine_bits bins
    if (TILED && g.fine_bits)
        for (uint32_t p = threadIdx.x; p < (P << g.fine_bits); p += ST_T) fh[p] = 0;
    bool spec = true; // the previous tile kept a row (workgroup-uniform): keys load with the predicate
    // VSKIP (input the caller expects to keep almost nothing): all-false tiles of a plain column
    // predicate are checked with vector loads (16-byte aligned column and segment start).  Not
    // the default: the extra live state spills 6 VGPRs of the kept-row path (partition +2 %, r05q)
    const bool skip_vec = VSKIP && TILED && PredVec<Pred>::ok && pred_vec_aligned(pred, begin);
    __shared__ uint8_t s_flags[VSKIP ? FLAG_TPS_MAX : 1];
    if constexpr (VSKIP) {
        if (g.tile_flags) { // this segment's tile flags (the host checks tps <= FLAG_TPS_MAX)
            for (int k = threadIdx.x; k < g.tps; k += ST_T) s_flags[k] = g.tile_flags[(size_t)blockIdx.x * g.tps + k];
            __syncthreads();
            spec = false; // the first tile is checked too
        }
    }
    for (uint32_t tb = begin; tb < end; tb += (uint32_t)g.TR) {
        if constexpr (TILED) {
            bool use_flags = false;
            if constexpr (VSKIP) use_flags = g.tile_flags != nullptr;
            if (!spec || use_flags) {
                // the previous tile kept no row: skip ahead over tiles whose predicate keeps
                // nothing — one predicate read and one barrier each, their runs written empty —
                // to the next tile that keeps a row (FilterTransformAction.cpp:134-138).  (Two
                // tiles a round, their loads in flight together, cost the kept-row path 40 %:
                // the partition kernel ran out of VGPRs, r05k)
                while (tb < end) {
                    if constexpr (VSKIP) {
                        if (g.tile_flags) { // one LDS byte a tile (loaded at the start), no barrier
                            if (s_flags[(tb - begin) / (uint32_t)g.TR]) break;
                            tb += (uint32_t)g.TR;
                            continue;
                        }
                        if (skip_vec && tb + (uint32_t)SKIP_NT * (uint32_t)g.TR <= end) {
                            // SKIP_NT whole tiles a round, all their words in flight together
                            bool a[SKIP_NT];
                            tile_any_vecn<ST_T, ST_MAXR, SKIP_NT>(pred, tb, per, (uint32_t)g.TR, a);
                            int keep = SKIP_NT; // the first tile of the round that keeps a row
#pragma unroll
                            for (int t = 0; t < SKIP_NT; ++t)
                                if (keep == SKIP_NT && __syncthreads_or(a[t])) keep = t;
                            tb += (uint32_t)keep * (uint32_t)g.TR;
                            if (keep < SKIP_NT) break;
                            continue;
                        }
                    }
                    bool any = false;
                    if (skip_vec && tb + (uint32_t)g.TR <= end) {
                        // a whole tile of a plain `T col Op scalar` predicate: its column words
                        // read as 16-byte vectors, all of a thread's in flight at once (one HBM
                        // round trip a tile instead of one a row)
                        any = tile_any_vec<ST_T, ST_MAXR>(pred, tb, per);
                    } else {
#pragma unroll
                        for (int j = 0; j < ST_MAXR; ++j) {
                            const uint32_t r = tb + (uint32_t)j * ST_T + threadIdx.x;
                            if (j < per && r < end) any = any || pred.eval(pred.load(r));
                        }
                    }
                    if (__syncthreads_or(any)) break;
                    if constexpr (!VSKIP) { // VSKIP: the caller zeroed the whole table up front (one
                                            // memset instead of P strided 4-byte stores a tile)
                        const uint32_t tile = blockIdx.x * (uint32_t)g.tps + (tb - begin) / (uint32_t)g.TR;
                        for (uint32_t p = threadIdx.x; p < P; p += ST_T) g.tile_hist[(size_t)p * g.T + tile] = 0u;
                    }
                    tb += (uint32_t)g.TR;
                }
                if (tb >= end) break;
                spec = !use_flags; // this tile keeps a row (with flags: its keys load for kept rows only)
            }
        }
        for (uint32_t p = threadIdx.x; p < P; p += ST_T) hist[p] = 0;
        if ((NARROW || WNARROW) && threadIdx.x == 0) red[ST_T / 64 + 1] = 0;
        __syncthreads();
        // 1. destination + rank of every row of the tile
        uint32_t bq[ST_MAXR]; // destination (low 16 bits) | rank inside the tile (high 16 bits)
        constexpr int VC = NC8 > 0 ? NC8 : 1;
        uint64_t v[VC][ST_MAXR]; // NC8 path: payload words, loaded before the ranks / scan
        constexpr bool WK = SelWideKey<Sel>::value && NC8 >= 2;
        const int c0 = NC8 > 0 && cols.key0 ? (WK ? 2 : 1) : 0;
        constexpr int HB = ST_MAXR / 2; // two half-batches keep the live loaded values small
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            Loaded pl[HB], kl[HB];
            // the half-batch's loads first: predicate and key words together, unless the
            // previous tile kept no row (workgroup-uniform): then the predicate first and the keys
            // of the rows it keeps only, so all-false input reads no key word
            // (FilterTransformAction.cpp:134-138 skips all-false blocks)
            bool keep[HB];
#pragma unroll
            for (int q = 0; q < HB; ++q) {
                const int j = h * HB + q;
                const uint32_t r = tb + (uint32_t)j * ST_T + threadIdx.x;
                if (j < per && r < end) {
                    pl[q] = pred.load(r);
                    if (spec) kl[q] = sel.load(r);
                }
            }
#pragma unroll
            for (int q = 0; q < HB; ++q) {
                const int j = h * HB + q;
                const uint32_t r = tb + (uint32_t)j * ST_T + threadIdx.x;
                keep[q] = j < per && r < end && pred.eval(pl[q]);
                if (!spec && keep[q]) kl[q] = sel.load(r);
            }
#pragma unroll
            for (int q = 0; q < HB; ++q) { // ... then destinations
                const int j = h * HB + q;
                bq[j] = 0xFFFFFFFFu;
                const uint32_t r = tb + (uint32_t)j * ST_T + threadIdx.x;
                if (keep[q]) {
                    uint32_t b = sel.part(crc, kl[q], r);
                    if (TILED && g.fine_bits && b < (P << g.fine_bits)) {
                        atomicAdd(&fh[b], 1u);
                        b >>= g.fine_bits;
                    }
                    if (b < P) bq[j] = b;
                }
                if constexpr (NC8 > 0) v[0][j] = kl[q].bits;
                if constexpr (WK) v[VC > 1 ? 1 : 0][j] = kl[q].hi;
                if constexpr (NC8 == 0) {
                    if (bq[j] != 0xFFFFFFFFu) bq[j] |= atomicAdd(&hist[bq[j]], 1u) << 16;
                }
            }
        }
        if constexpr (NC8 > 0) {
            // payload loads in flight across the LDS rank / scan phases
            const uint32_t stride = cols.in_stride > 1 ? (uint32_t)cols.in_stride : 1u;
#pragma unroll
            for (int c = 0; c < NC8; ++c) {
                if (c < c0) continue;
                const uint64_t *src = reinterpret_cast<const uint64_t *>(cols.in[c]);
#pragma unroll
                for (int j = 0; j < ST_MAXR; ++j)
                    if (bq[j] != 0xFFFFFFFFu) v[c][j] = src[(size_t)(tb + (uint32_t)j * ST_T + threadIdx.x) * stride];
            }
#pragma unroll
            for (int j = 0; j < ST_MAXR; ++j)
                if (bq[j] != 0xFFFFFFFFu) bq[j] |= atomicAdd(&hist[bq[j]], 1u) << 16;
            if constexpr (NARROW) {
                bool wide = false;
#pragma unroll
                for (int j = 0; j < ST_MAXR; ++j) wide |= bq[j] != 0xFFFFFFFFu && (v[0][j] >> 32) != 0;
                if (wide) red[ST_T / 64 + 1] = 1;
            }
            if constexpr (WNARROW) {
                bool wide = false;
#pragma unroll
                for (int j = 0; j < ST_MAXR; ++j) wide |= bq[j] != 0xFFFFFFFFu && !wide_hi_narrowable(v[1][j]);
                if (wide) red[ST_T / 64 + 1] = 1;
            }
        }
        __syncthreads();
        // 2. exclusive scan of the tile histogram -> start of each destination inside the tile
        //    (TILED: the low 16 bits scan the counts, the high 16 bits the counts padded to the
        //    run alignment; both totals stay below 2^16)
        {
            const uint32_t chunk = (P + ST_T - 1) / ST_T;
            const uint32_t p0 = threadIdx.x * chunk;
            const uint32_t am = TILED ? (uint32_t)g.align - 1 : 0u;
            auto cnt2 = [&](uint32_t h) -> uint32_t { return TILED ? (h | (((h + am) & ~am) << 16)) : h; };
            uint32_t s = 0;
            for (uint32_t p = p0; p < p0 + chunk && p < P; ++p) s += cnt2(hist[p]);
            const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
            uint32_t x = s;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d, 64);
                if (lane >= (unsigned)d) x += y;
            }
            if (lane == 63) red[wave] = x;
            __syncthreads();
            uint32_t off = x - s;
            for (unsigned w = 0; w < wave; ++w) off += red[w];
            for (uint32_t p = p0; p < p0 + chunk && p < P; ++p) {
                if constexpr (TILED) {
                    start[p] = off & 0xFFFFu;
                    pstart[p] = off >> 16;
                } else {
                    start[p] = off;
                }
                off += cnt2(hist[p]);
            }
            if (threadIdx.x == ST_T - 1) red[ST_T / 64] = TILED ? (off & 0xFFFFu) : off; // rows kept in this tile
        }
        __syncthreads();
        const uint32_t kept = red[ST_T / 64];
        spec = kept != 0;
        const uint32_t tile = blockIdx.x * (uint32_t)g.tps + (tb - begin) / (uint32_t)g.TR;
        const bool narrow = (NARROW || WNARROW) && g.allow_narrow && red[ST_T / 64 + 1] == 0;
        if constexpr (TILED)
            for (uint32_t p = threadIdx.x; p < P; p += ST_T)
                g.tile_hist[(size_t)p * g.T + tile] = pstart[p] | (narrow ? TILE_NARROW : 0u) | (hist[p] << 16);
        // 3. place rows in LDS in destination order
        uint32_t sl[ST_MAXR];
#pragma unroll
        for (int j = 0; j < ST_MAXR; ++j) {
            if (bq[j] == 0xFFFFFFFFu) continue;
            sl[j] = start[bq[j] & 0xFFFFu] + (bq[j] >> 16);
            sb[sl[j]] = (uint16_t)(bq[j] & 0xFFFFu);
            if (perm) {
                const uint32_t row = tb + (uint32_t)j * ST_T + threadIdx.x;
                sperm[sl[j]] = cols.perm_in ? cols.perm_in[row] : row;
            }
        }
        if constexpr (NC8 > 0) {
#pragma unroll
            for (int c = 0; c < NC8; ++c) {
                uint64_t *st = reinterpret_cast<uint64_t *>(lds + g.stage_off[c]);
#pragma unroll
                for (int j = 0; j < ST_MAXR; ++j)
                    if (bq[j] != 0xFFFFFFFFu) st[sl[j]] = v[c][j];
            }
        } else {
            for (int c = 0; c < ncols; ++c) {
                char *st = lds + g.stage_off[c];
                const int w = cols.width[c];
                if (w <= 8) {
                    uint64_t v[ST_MAXR];
#pragma unroll
                    for (int j = 0; j < ST_MAXR; ++j)
                        if (bq[j] != 0xFFFFFFFFu) v[j] = load_width(cols.in[c], w, tb + (uint32_t)j * ST_T + threadIdx.x);
#pragma unroll
                    for (int j = 0; j < ST_MAXR; ++j) {
                        if (bq[j] == 0xFFFFFFFFu) continue;
                        switch (w) {
                        case 1: ((uint8_t *)st)[sl[j]] = (uint8_t)v[j]; break;
                        case 2: ((uint16_t *)st)[sl[j]] = (uint16_t)v[j]; break;
                        case 4: ((uint32_t *)st)[sl[j]] = (uint32_t)v[j]; break;
                        default: ((uint64_t *)st)[sl[j]] = v[j]; break;
                        }
                    }
                } else {
                    const int q = w / 16; // 16- or 32-byte values as 1-2 uint4
#pragma unroll
                    for (int j = 0; j < ST_MAXR; ++j)
                        if (bq[j] != 0xFFFFFFFFu)
                            for (int h = 0; h < q; ++h)
                                ((uint4 *)st)[sl[j] * q + h] = ((const uint4 *)cols.in[c])[(size_t)(tb + (uint32_t)j * ST_T + threadIdx.x) * q + h];
                }
            }
        }
        __syncthreads();
        // 4. stream the sorted tile out: lanes of a run write consecutive addresses
        for (uint32_t s = threadIdx.x; s < kept; s += ST_T) {
            const uint32_t b = sb[s];
            uint64_t gp;
            if constexpr (TILED) gp = (uint64_t)tile * (uint32_t)g.TRS + pstart[b] + (s - start[b]);
            else gp = run[b] + (s - start[b]);
            if (perm) perm[gp] = sperm[s];
            if (WNARROW && narrow) { // 20-byte records (nrec_store) in the tile's slot
                const uint32_t pos = pstart[b] + (s - start[b]);
                nrec_store(reinterpret_cast<uint64_t *>(cols.out[0]) + (size_t)tile * (uint32_t)g.TRS * 3, pos,
                           reinterpret_cast<const uint64_t *>(lds + g.stage_off[0])[s],
                           wide_narrow_hi(reinterpret_cast<const uint64_t *>(lds + g.stage_off[1])[s]),
                           reinterpret_cast<const uint64_t *>(lds + g.stage_off[2])[s]);
            } else if (NARROW && narrow) { // u32 keys, then u64 values, in the tile's slot
                const uint32_t pos = pstart[b] + (s - start[b]);
                uint32_t *ks = reinterpret_cast<uint32_t *>(reinterpret_cast<uint64_t *>(cols.out[0]) +
                                                            (size_t)tile * (uint32_t)g.TRS * 2);
                ks[pos] = (uint32_t)reinterpret_cast<const uint64_t *>(lds + g.stage_off[0])[s];
                reinterpret_cast<uint64_t *>(ks + g.TRS)[pos] = reinterpret_cast<const uint64_t *>(lds + g.stage_off[1])[s];
            } else if constexpr (AOS && NC8 == 2) { // one 16-byte record store per row
                const uint64_t a0 = reinterpret_cast<const uint64_t *>(lds + g.stage_off[0])[s];
                const uint64_t a1 = reinterpret_cast<const uint64_t *>(lds + g.stage_off[1])[s];
                typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
                u64x2 rec;
                rec.x = a0;
                rec.y = a1;
                reinterpret_cast<u64x2 *>(cols.out[0])[gp] = rec; // (nontemporal stores measured no different, r05h)
            } else if constexpr (AOS) {
#pragma unroll
                for (int c = 0; c < NC8; ++c)
                    ((uint64_t *)cols.out[0])[gp * NC8 + c] = reinterpret_cast<const uint64_t *>(lds + g.stage_off[c])[s];
            } else if constexpr (NC8 > 0) {
#pragma unroll
                for (int c = 0; c < NC8; ++c)
                    ((uint64_t *)cols.out[c])[gp] = reinterpret_cast<const uint64_t *>(lds + g.stage_off[c])[s];
            } else {
                for (int c = 0; c < ncols; ++c) {
                    const char *st = lds + g.stage_off[c];
                    switch (cols.width[c]) {
                    case 1: ((uint8_t *)cols.out[c])[gp] = ((const uint8_t *)st)[s]; break;
                    case 2: ((uint16_t *)cols.out[c])[gp] = ((const uint16_t *)st)[s]; break;
                    case 4: ((uint32_t *)cols.out[c])[gp] = ((const uint32_t *)st)[s]; break;
                    case 8: ((uint64_t *)cols.out[c])[gp] = ((const uint64_t *)st)[s]; break;
                    case 32:
                        ((uint4 *)cols.out[c])[2 * gp] = ((const uint4 *)st)[2 * s];
                        ((uint4 *)cols.out[c])[2 * gp + 1] = ((const uint4 *)st)[2 * s + 1];
                        break;
                    default: ((uint4 *)cols.out[c])[gp] = ((const uint4 *)st)[s]; break;
                    }
                }
            }
        }
        __syncthreads();
        if constexpr (!TILED)
            for (uint32_t p = threadIdx.x; p < P; p += ST_T) run[p] += hist[p];
        __syncthreads();
    }
    if constexpr (TILED) {
        // tile slots past the segment's last row (a short last segment: it has fewer than tps
        // tiles) hold no run: their entries are zeroed, as every consumer walks all T tiles
        const uint32_t visited = (end - begin + (uint32_t)g.TR - 1) / (uint32_t)g.TR;
        for (uint32_t k = visited; k < (uint32_t)g.tps; ++k)
            for (uint32_t p = threadIdx.x; p < P; p += ST_T)
                g.tile_hist[(size_t)p * g.T + blockIdx.x * (uint32_t)g.tps + k] = 0u;
    }
    if (TILED && g.fine_bits)
        for (uint32_t p = threadIdx.x; p < (P << g.fine_bits); p += ST_T)
            if (fh[p]) atomicAdd(&g.fine_counts[p], fh[p]);
}

template <typename Sel, bool STABLE = true>
int run_partition(Ctx *ctx, const Sel &sel, const RowPred &pred, const PartLayout &L0, const PCols &cols,
                  uint32_t *perm, uint32_t *part_out, uint64_t *offsets_out, void *tmp,
                  const char *hist_name = "part.hist", const char *scatter_name = "part.scatter");

// Radix partition into P > TWO_PASS_MIN destinations in two passes: the staged scatter's runs
// per destination shrink with P (a tile of ~8K rows into 4096 destinations writes ~2-row runs),
// so pass 1 scatters into 64 radix groups (long runs), and pass 2 partitions those records by
// the full radix — every pass-2 tile then holds rows of one or two groups, so its rows go to
// at most ~128 destinations.  Bytes: 2x the scatter traffic, at full write efficiency.
template <typename Sel>
int run_two_pass(Ctx *ctx, const Sel &sel, const RowPred &pred, const PartLayout &L0, const PCols &cols,
                 uint32_t *perm, uint64_t *offsets_out, void *tmp, const char *hist_name, const char *scatter_name) {
    const int nc = cols.ncols;
    char *x = (char *)tmp + part_tmp_bytes(L0);
    uint64_t *inter = (uint64_t *)x;
    x += align256((size_t)L0.n * nc * 8);
    uint32_t *perm1 = nullptr;
    if (perm) {
        perm1 = (uint32_t *)x;
        x += align256((size_t)L0.n * 4);
    }
    uint64_t *offs1 = (uint64_t *)x;
    Sel s1 = sel;
    s1.shift = fib_shift(TWO_PASS_P1);
    PCols c1 = cols;
    c1.out[0] = inter;
    c1.two_pass = 0;
    if (int rc = run_partition<Sel, false>(ctx, s1, pred, make_layout(L0.n, TWO_PASS_P1), c1, perm1, nullptr, offs1,
                                           tmp, hist_name, scatter_name))
        return rc;
    uint64_t kept = 0;
    if (int rc = read_back_u64(ctx, offs1 + TWO_PASS_P1, &kept, 1)) return rc;
    SelRec8 s2{inter, nc, fib_shift(L0.P)};
    PCols c2 = cols;
    for (int c = 0; c < nc; ++c) c2.in[c] = inter + c;
    c2.in_stride = nc;
    c2.perm_in = perm1;
    c2.key0 = 1;
    c2.two_pass = 0;
    RowPred all{};
    return run_partition<SelRec8, false>(ctx, s2, all, make_layout((int64_t)kept, L0.P), c2, perm, nullptr, offsets_out,
                                         tmp, hist_name, scatter_name);
}

template <typename Sel, bool STABLE>
int run_partition(Ctx *ctx, const Sel &sel, const RowPred &pred, const PartLayout &L0, const PCols &cols,
                  uint32_t *perm, uint32_t *part_out, uint64_t *offsets_out, void *tmp,
                  const char *hist_name, const char *scatter_name) {
    TFG_CHECK(L0.P >= 1 && L0.P <= (STABLE ? PMAX : PMAX_UNSTABLE), TFG_ERR_INVALID_ARG, "partition count %u out of range", L0.P);
    if constexpr (!STABLE && Sel::fib_radix) {
        bool all8 = cols.ncols >= 1 && cols.ncols <= 3 && (cols.aos || cols.ncols == 1);
        for (int c = 0; c < cols.ncols; ++c) all8 = all8 && cols.width[c] == 8;
        if (cols.two_pass && all8 && !part_out && L0.n > 0 && L0.P > TWO_PASS_MIN)
            return run_two_pass(ctx, sel, pred, L0, cols, perm, offsets_out, tmp, hist_name, scatter_name);
    }
    StagedGeom sg{};
    const bool staged = !STABLE && !part_out && L0.n > 0 && make_staged_geom(L0.P, cols, perm != nullptr, Sel::needs_crc, sg);
    // the staged scatter uses fewer, longer segments (P x G <= P x L0.G: fits the caller's tmp)
    const PartLayout L = staged ? make_wide_layout(L0.n, L0.P, ctx->cu_count, L0.G) : L0;
    const int64_t e = (int64_t)L.P * L.G;
    char *t = (char *)tmp;
    uint32_t *counts = (uint32_t *)t;
    t += ((size_t)e * 4 + 255) / 256 * 256;
    uint64_t *offs = (uint64_t *)t;
    t += ((size_t)(e + 1) * 8 + 255) / 256 * 256;
    void *scan_tmp = t;
    if (L.n > 0) {
        ProfScope _ps(ctx, hist_name);
        if (L.sub > 1) TFG_HIP(hipMemsetAsync(counts, 0, (size_t)e * 4, ctx->stream));
        if (int rc = with_pred(pred, [&](auto pr) -> int {
                hipLaunchKernelGGL((part_hist_kernel<Sel, decltype(pr)>), dim3(L.G * L.sub), dim3(PT),
                                   hist_lds_bytes(L.P, Sel::needs_crc), ctx->stream, sel, pr, L, counts);
                TFG_LAUNCH_CHECK();
                return TFG_OK;
            }))
            return rc;
    } else {
        TFG_HIP(hipMemsetAsync(counts, 0, (size_t)e * 4, ctx->stream));
    }
    if (int rc = exclusive_scan_u32(ctx, counts, offs, e, scan_tmp)) return rc;
    if (staged) {
        int nc8 = cols.ncols;
        for (int c = 0; c < cols.ncols; ++c)
            if (cols.width[c] != 8) nc8 = 0;
        if (nc8 > 3) nc8 = 0;
        TFG_CHECK(!cols.aos || nc8 >= 2, TFG_ERR_INVALID_ARG, "record layout needs 2-3 columns of 8 bytes");
        ProfScope _ps(ctx, scatter_name);
        if (int rc = with_pred(pred, [&](auto pr) -> int {
                using PR = decltype(pr);
                if (cols.aos) {
                    if (nc8 == 2) hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 2, true>), dim3(L.G), dim3(ST_T), sg.lds_bytes, ctx->stream, sel, pr, L, offs, cols, perm, sg);
                    else hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 3, true>), dim3(L.G), dim3(ST_T), sg.lds_bytes, ctx->stream, sel, pr, L, offs, cols, perm, sg);
                    TFG_LAUNCH_CHECK();
                    return TFG_OK;
                }
                switch (nc8) {
                case 1: hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 1>), dim3(L.G), dim3(ST_T), sg.lds_bytes, ctx->stream, sel, pr, L, offs, cols, perm, sg); break;
                case 2: hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 2>), dim3(L.G), dim3(ST_T), sg.lds_bytes, ctx->stream, sel, pr, L, offs, cols, perm, sg); break;
                case 3: hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 3>), dim3(L.G), dim3(ST_T), sg.lds_bytes, ctx->stream, sel, pr, L, offs, cols, perm, sg); break;
                default: hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 0>), dim3(L.G), dim3(ST_T), sg.lds_bytes, ctx->stream, sel, pr, L, offs, cols, perm, sg); break;
                }
                TFG_LAUNCH_CHECK();
                return TFG_OK;
            }))
            return rc;
    } else if (L.n > 0 && (perm || part_out || cols.ncols > 0)) {
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

// Tile-sorted partition (no histogram pass, no scattered stores): every tile of TR rows is
// counting-sorted by destination in LDS and written back contiguously to its own slot; the
// per-(destination, tile) start | count table tells a destination's consumer where its runs are.
// Used where the consumer reads a destination's rows once (the aggregation bucket kernel):
// it replaces the histogram pass (16 B / row) and the scatter's ~P-way store pattern.
struct TiledGeom {
    StagedGeom sg;
    PartLayout L;
    int64_t out_rows; // T * TRS
};

inline bool make_tiled_geom(Ctx *ctx, int64_t n, uint32_t P, const PCols &cols, TiledGeom &tg, int fine_bits = 0) {
    if (n <= 0 || !make_staged_geom(P, cols, false, false, tg.sg, fine_bits)) return false;
    tg.L = make_wide_layout(n, P, ctx->cu_count, 1u << 30, 3); // 3 segments per CU: measured 0.77 vs 0.83 ms at 1
    tg.sg.tps = (int)((tg.L.seg + tg.sg.TR - 1) / tg.sg.TR);
    tg.sg.T = (int)tg.L.G * tg.sg.tps;
    // dense runs (align 1): padding runs to 128 B left every run's last line partly written and
    // measured slower (agg.part.tiled 0.93 vs 0.74 ms on C2, the bucket kernel unchanged)
    tg.sg.align = 1;
    tg.sg.TRS = (tg.sg.TR + (tg.sg.align - 1) * (int)P + 1) & ~1; // even: a narrow tile's values stay 8-byte aligned
    if (tg.sg.TRS >= (int)TILE_NARROW) return false;              // starts must stay below the flag bit
    tg.out_rows = (int64_t)tg.sg.T * tg.sg.TRS;
    return true;
}

// sparse: the caller expects almost every tile to keep no row (its previous input kept fewer rows
// than it has tiles): plain column predicates take the vector all-false check (VSKIP)
template <typename Sel>
int run_partition_tiled(Ctx *ctx, const Sel &sel, const RowPred &pred, TiledGeom tg, const PCols &cols,
                        uint32_t *tile_hist, const char *name, bool sparse = false, uint8_t *flags = nullptr) {
    tg.sg.tile_hist = tile_hist;
    int nc8 = cols.ncols;
    for (int c = 0; c < cols.ncols; ++c)
        if (cols.width[c] != 8) nc8 = 0;
    TFG_CHECK(cols.aos && nc8 >= 1 && nc8 <= 3, TFG_ERR_INVALID_ARG, "tiled partition needs 1-3 word records");
    ProfScope _ps(ctx, name);
    return with_pred(pred, [&](auto pr) -> int {
        using PR = decltype(pr);
        if constexpr (PredVec<PR>::ok) {
            if (sparse) {
                // skipped tiles leave their (destination, tile) entries to this memset
                TFG_HIP(hipMemsetAsync(tg.sg.tile_hist, 0, (size_t)tg.L.P * tg.sg.T * 4, ctx->stream));
                if (flags && tg.sg.tps <= FLAG_TPS_MAX) { // every tile's "keeps a row" first
                    hipLaunchKernelGGL((tile_flags_kernel<PR>), dim3((unsigned)tg.sg.T), dim3(TF_T), 0, ctx->stream, pr,
                                       tg.L, tg.sg.TR, tg.sg.tps, flags);
                    TFG_LAUNCH_CHECK();
                    tg.sg.tile_flags = flags;
                }
                if (nc8 == 1)
                    hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 1, true, true, true>), dim3(tg.L.G),
                                       dim3(ST_T), tg.sg.lds_bytes, ctx->stream, sel, pr, tg.L,
                                       (const uint64_t *)nullptr, cols, (uint32_t *)nullptr, tg.sg);
                else if (nc8 == 2)
                    hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 2, true, true, true>), dim3(tg.L.G),
                                       dim3(ST_T), tg.sg.lds_bytes, ctx->stream, sel, pr, tg.L,
                                       (const uint64_t *)nullptr, cols, (uint32_t *)nullptr, tg.sg);
                else
                    hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 3, true, true, true>), dim3(tg.L.G),
                                       dim3(ST_T), tg.sg.lds_bytes, ctx->stream, sel, pr, tg.L,
                                       (const uint64_t *)nullptr, cols, (uint32_t *)nullptr, tg.sg);
                TFG_LAUNCH_CHECK();
                return TFG_OK;
            }
        }
        if (nc8 == 1) // keys alone (GROUP BY with count() only)
            hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 1, true, true>), dim3(tg.L.G), dim3(ST_T),
                               tg.sg.lds_bytes, ctx->stream, sel, pr, tg.L, (const uint64_t *)nullptr, cols,
                               (uint32_t *)nullptr, tg.sg);
        else if (nc8 == 2)
            hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 2, true, true>), dim3(tg.L.G), dim3(ST_T),
                               tg.sg.lds_bytes, ctx->stream, sel, pr, tg.L, (const uint64_t *)nullptr, cols,
                               (uint32_t *)nullptr, tg.sg);
        else
            hipLaunchKernelGGL((part_scatter_staged_kernel<Sel, PR, 3, true, true>), dim3(tg.L.G), dim3(ST_T),
                               tg.sg.lds_bytes, ctx->stream, sel, pr, tg.L, (const uint64_t *)nullptr, cols,
                               (uint32_t *)nullptr, tg.sg);
        TFG_LAUNCH_CHECK();
        return TFG_OK;
    });
}

// ---------------------------------------------------------------- two-level tiled partition
// P = RS_C << fine_bits destinations with contiguous, destination-major output, no histogram
// pass and no host round trip (the join's probe side, P = 2048 / 4096):
//   pass 1  run_partition_tiled into RS_C coarse radix groups; each tile is written sorted by the
//           coarse radix and the workgroups add every row's full radix into a P-bin histogram;
//   scan    of that histogram -> the destinations' offsets (offsets_out) and append cursors;
//   pass 2  regroup_scatter_kernel: one workgroup per (coarse group, RS_TPC tiles) reads the
//           group's runs (~128 rows each) from those tiles, counting-sorts a batch of RS_BR rows
//           by the fine radix in LDS, claims each fine run's place with one global atomic and
//           writes the runs out contiguously.
// Bytes: 2 x (read + write) of the records, against 2 x (histogram read + read + write) for the
// histogram + scatter form (run_two_pass).  Order inside a destination is unspecified.
constexpr uint32_t RS_C = 64;
constexpr int RS_T = 512, RS_RPT = 4, RS_BR = RS_T * RS_RPT, RS_TPC = 64;

// NT: a streaming (nontemporal) load, for records read once while other data must stay in L2
template <int NW, bool NT = false>
__device__ __forceinline__ void load_rec(const uint64_t *rec, size_t pos, uint64_t (&v)[NW]) {
    if constexpr (NW == 2) { // one 16-byte load
        typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
        const u64x2 *p = reinterpret_cast<const u64x2 *>(rec) + pos;
        u64x2 q;
        if constexpr (NT) q = __builtin_nontemporal_load(p);
        else q = *p;
        v[0] = q.x;
        v[1] = q.y;
    } else {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            if constexpr (NT) v[w] = __builtin_nontemporal_load(rec + pos * NW + w);
            else v[w] = rec[pos * NW + w];
        }
    }
}

template <int NW>
__global__ void __launch_bounds__(RS_T) regroup_scatter_kernel(const uint64_t *rec, const uint32_t *tile_hist, int T,
                                                               int TRS, int fine_bits, uint32_t shift,
                                                               unsigned long long *cursor, uint64_t *out) {
    __shared__ uint32_t tstart[RS_TPC], tpre[RS_TPC + 1];
    __shared__ uint32_t hist[64], hstart[64];
    __shared__ unsigned long long gbase[64];
    __shared__ uint64_t stage[NW][RS_BR];
    __shared__ uint8_t sf[RS_BR];
    const unsigned lane = threadIdx.x & 63;
    const uint32_t c = blockIdx.x % RS_C;
    const int t0 = (int)(blockIdx.x / RS_C) * RS_TPC;
    const int nt = min(RS_TPC, T - t0);
    const uint32_t fmask = (1u << fine_bits) - 1;
    if (threadIdx.x < 64) { // one wave: the runs of group c in tiles t0 .. t0 + nt, scanned
        uint32_t cnt = 0, st = 0;
        if ((int)lane < nt) {
            const uint32_t h = tile_hist[(size_t)c * T + t0 + lane];
            st = h & (TILE_NARROW - 1);
            cnt = h >> 16;
        }
        uint32_t x = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= (unsigned)d) x += y;
        }
        tstart[lane] = st;
        tpre[lane + 1] = x;
        if (lane == 0) tpre[0] = 0;
        hist[lane] = 0;
    }
    __syncthreads();
    const uint32_t R = tpre[nt];
    // a batch's records: row i of the group's concatenated runs -> its run (binary search over
    // the scanned run lengths) -> its record in the tile slot
    auto load_batch = [&](uint32_t b0, uint64_t (&v)[RS_RPT][NW], bool (&val)[RS_RPT]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < RS_RPT; ++u) {
            const uint32_t i = b0 + (uint32_t)u * RS_T + threadIdx.x;
            val[u] = i < R;
            if (!val[u]) continue;
            int lo = 0, hi = nt; // tpre[lo] <= i < tpre[lo + 1]
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (tpre[mid] <= i) lo = mid;
                else hi = mid;
            }
            load_rec<NW>(rec, (size_t)(t0 + lo) * (uint32_t)TRS + tstart[lo] + (i - tpre[lo]), v[u]);
        }
    };
    uint64_t v[RS_RPT][NW];
    bool val[RS_RPT];
    if (R) load_batch(0, v, val);
    // software pipelined: the next batch's loads are issued before this batch's global cursor
    // atomics, barriers and stores, so their latency overlaps them
    for (uint32_t b0 = 0; b0 < R; b0 += RS_BR) {
        uint32_t fq[RS_RPT];
#pragma unroll
        for (int u = 0; u < RS_RPT; ++u) {
            fq[u] = 0xFFFFFFFFu;
            if (!val[u]) continue;
            const uint32_t f = fib_part(v[u][0], shift) & fmask;
            fq[u] = f | (atomicAdd(&hist[f], 1u) << 16);
        }
        uint64_t nv[RS_RPT][NW];
        bool nval[RS_RPT] = {};
        if (b0 + RS_BR < R) load_batch(b0 + RS_BR, nv, nval);
        __syncthreads();
        if (threadIdx.x < 64) {
            const uint32_t h = hist[lane];
            hist[lane] = 0; // for the next batch (its atomics come after two more barriers)
            uint32_t x = h;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d, 64);
                if (lane >= (unsigned)d) x += y;
            }
            hstart[lane] = x - h;
            if (h) gbase[lane] = atomicAdd(&cursor[(c << fine_bits) + lane], (unsigned long long)h);
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < RS_RPT; ++u) {
            if (fq[u] == 0xFFFFFFFFu) continue;
            const uint32_t f = fq[u] & 0xFFFFu, s = hstart[f] + (fq[u] >> 16);
#pragma unroll
            for (int w = 0; w < NW; ++w) stage[w][s] = v[u][w];
            sf[s] = (uint8_t)f;
        }
        __syncthreads();
        const uint32_t kept = min((uint32_t)RS_BR, R - b0);
        for (uint32_t s = threadIdx.x; s < kept; s += RS_T) {
            const uint32_t f = sf[s];
            const uint64_t gp = gbase[f] + (s - hstart[f]);
            if constexpr (NW == 2) {
                typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
                u64x2 q;
                q.x = stage[0][s];
                q.y = stage[1][s];
                reinterpret_cast<u64x2 *>(out)[gp] = q;
            } else {
#pragma unroll
                for (int w = 0; w < NW; ++w) out[gp * NW + w] = stage[w][s];
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < RS_RPT; ++u) {
            val[u] = nval[u];
#pragma unroll
            for (int w = 0; w < NW; ++w) v[u][w] = nv[u][w];
        }
    }
}

// geometry of the two-level form (false: not applicable -> use run_partition)
inline bool make_two_level_geom(Ctx *ctx, int64_t n, uint32_t P, const PCols &cols, TiledGeom &tg) {
    if (P <= RS_C || P > RS_C * 64 || (P & (P - 1)) || cols.ncols < 1 || cols.ncols > 3 || n <= 0) return false;
    for (int c = 0; c < cols.ncols; ++c)
        if (cols.width[c] != 8) return false;
    PCols pc = cols;
    pc.aos = 1;
    if (!make_tiled_geom(ctx, n, RS_C, pc, tg, (int)bits_of_pow2(P / RS_C))) return false;
    tg.sg.allow_narrow = 0;
    return true;
}
inline size_t two_level_tmp_bytes(const TiledGeom &tg, uint32_t P, int ncols) {
    return align256((size_t)tg.out_rows * ncols * 8) + align256((size_t)RS_C * tg.sg.T * 4) + align256((size_t)P * 4) +
           align256((size_t)P * 8) + align256(scan_tmp_bytes(P));
}

// sel: the full P-way radix (its shift for P).  cols: 8-byte columns (key first), written as
// interleaved records of cols.ncols words at cols.out[0].  offsets_out: device u64[P + 1].
template <typename Sel>
int run_partition_two_level(Ctx *ctx, const Sel &sel, const RowPred &pred, TiledGeom tg, uint32_t P, const PCols &cols,
                            uint64_t *offsets_out, void *tmp, const char *name1, const char *name2) {
    const int nc = cols.ncols;
    char *x = (char *)tmp;
    uint64_t *inter = (uint64_t *)x;
    x += align256((size_t)tg.out_rows * nc * 8);
    uint32_t *tile_hist = (uint32_t *)x;
    x += align256((size_t)RS_C * tg.sg.T * 4);
    uint32_t *fine = (uint32_t *)x;
    x += align256((size_t)P * 4);
    unsigned long long *cursor = (unsigned long long *)x;
    x += align256((size_t)P * 8);
    void *scan_tmp = x;
    const int fine_bits = tg.sg.fine_bits;
    TFG_CHECK(P == (RS_C << fine_bits) && fine_bits >= 1 && fine_bits <= 6, TFG_ERR_INVALID_ARG,
              "two-level partition: %u destinations", P);
    TFG_HIP(hipMemsetAsync(fine, 0, (size_t)P * 4, ctx->stream));
    tg.sg.fine_counts = fine;
    PCols c1 = cols;
    c1.aos = 1;
    c1.out[0] = inter;
    if (int rc = run_partition_tiled(ctx, sel, pred, tg, c1, tile_hist, name1)) return rc;
    if (int rc = exclusive_scan_u32(ctx, fine, offsets_out, P, scan_tmp)) return rc;
    TFG_HIP(hipMemcpyAsync(cursor, offsets_out, (size_t)P * 8, hipMemcpyDeviceToDevice, ctx->stream));
    const unsigned grid = RS_C * (unsigned)((tg.sg.T + RS_TPC - 1) / RS_TPC);
    ProfScope _ps(ctx, name2);
    uint64_t *out = (uint64_t *)cols.out[0];
    switch (nc) {
    case 1: hipLaunchKernelGGL(regroup_scatter_kernel<1>, dim3(grid), dim3(RS_T), 0, ctx->stream, inter, tile_hist, tg.sg.T, tg.sg.TRS, fine_bits, sel.shift, cursor, out); break;
    case 2: hipLaunchKernelGGL(regroup_scatter_kernel<2>, dim3(grid), dim3(RS_T), 0, ctx->stream, inter, tile_hist, tg.sg.T, tg.sg.TRS, fine_bits, sel.shift, cursor, out); break;
    default: hipLaunchKernelGGL(regroup_scatter_kernel<3>, dim3(grid), dim3(RS_T), 0, ctx->stream, inter, tile_hist, tg.sg.T, tg.sg.TRS, fine_bits, sel.shift, cursor, out); break;
    }
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

} // namespace tfg
