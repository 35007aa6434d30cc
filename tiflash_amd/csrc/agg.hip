// agg.hip — hash GROUP BY (Aggregator, a9-a17) for gfx950.
//
// Reference: Aggregator::executeOnBlock -> executeImplBatch -> handleOneBatch
// (Interpreters/Aggregator.cpp:776-1024): per row HashTable::emplace (Common/HashTable/HashTable.h:875-1060,
// HashCRC32 key64), then IAggregateFunction::addBatch (AggregateFunctions/IAggregateFunction.h:242-266,
// AggregateFunctionSum.h:64-172, AggregateFunctionCount.h:46); mergeDataImpl / MergingBuckets
// (Aggregator.cpp:2338-2505, 2940-3097); convertToBlockImplFinal (:1651-1780).
//
// GPU design (the radix-bucketed analogue of TwoLevelHashTable's 256 buckets):
//   1. bucket pass — fused predicate + key radix + LDS-histogram partition of the
//      (key, args) rows into B = 2^bucket_bits buckets (bucket = Fibonacci radix of the key, fib_part);
//   2. bucket kernel — one workgroup per bucket builds an open-addressing table in LDS
//      (linear probing, 64-bit ds_cmpst for keys, ds_add_{u64,f64} for states, key 0 and the
//      NULL key in side slots like ZeroValueStorage) seeded with the bucket's existing groups,
//      aggregates the staged rows, and writes its groups out.  If a bucket holds more distinct
//      keys than the LDS table, rows of keys not in the table are compacted in place and the
//      bucket iterates (each pass finalises >= maxfill groups), so any distribution is correct;
//   3. compaction — scan of per-bucket group counts -> groups stored bucket-major as the state.
// Group state is columnar in HBM: key bits (u64), NULL-key flag, per aggregate an accumulator
// (Int64/UInt64/Float64 or Int128) and a non-NULL row count.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"
#include "agg_dev.h"
#include "collation.h"
#include "serial.h"

namespace tfg {

// temp (bucket-strided) groups -> compact state
__global__ void agg_compact_kernel(AggSpec S, GroupsIO tmp, const uint64_t *stage_off, const uint64_t *old_off,
                                   const uint64_t *new_off, GroupsIO dst, const uint64_t *tmp_base) {
    const int b = blockIdx.x;
    const uint64_t src0 = tmp_base ? tmp_base[b] : stage_off[b] + (old_off ? old_off[b] : 0);
    const uint64_t d0 = new_off[b], cnt = new_off[b + 1] - d0;
    for (uint64_t j = threadIdx.x; j < cnt; j += blockDim.x) {
        const uint64_t s = src0 + j, d = d0 + j;
        if (S.key_width == 16) reinterpret_cast<uint4 *>(dst.key)[d] = reinterpret_cast<const uint4 *>(tmp.key)[s];
        else dst.key[d] = tmp.key[s];
        dst.key_null[d] = tmp.key_null[s];
        for (int i = 0; i < S.n_aggs; ++i) {
            if (S.acc[i] == ACC_I256) {
                ((uint4 *)dst.acc[i])[2 * d] = ((const uint4 *)tmp.acc[i])[2 * s];
                ((uint4 *)dst.acc[i])[2 * d + 1] = ((const uint4 *)tmp.acc[i])[2 * s + 1];
            } else if (S.acc[i] == ACC_I128) ((uint4 *)dst.acc[i])[d] = ((const uint4 *)tmp.acc[i])[s];
            else if (S.acc[i] != ACC_NONE) ((uint64_t *)dst.acc[i])[d] = ((const uint64_t *)tmp.acc[i])[s];
            if (S.has_cnt[i]) dst.cnt[i][d] = tmp.cnt[i][s];
        }
    }
}

// ---------------------------------------------------------------- without key (single group)
constexpr int NK_T = 256;
struct NoKeyPartial {
    uint64_t lo[AGG_MAX], hi[AGG_MAX], x2[AGG_MAX], x3[AGG_MAX], x4[AGG_MAX], cnt[AGG_MAX];
    double f[AGG_MAX];
};
// p (5 limbs at lo/hi/x2/x3/x4[i]: the exact sum, see lds_add_i256) += q (4 limbs, or 5 when q5)
__device__ __forceinline__ void nk_add(NoKeyPartial &p, int i, const uint64_t *q, const uint64_t *q4 = nullptr) {
    uint64_t a[5] = {p.lo[i], p.hi[i], p.x2[i], p.x3[i], p.x4[i]};
    add_i320(a, q);
    if (q4) a[4] += *q4 - ((int64_t)q[3] < 0 ? ~0ull : 0ull); // q's own fifth limb instead of its sign
    p.lo[i] = a[0];
    p.hi[i] = a[1];
    p.x2[i] = a[2];
    p.x3[i] = a[3];
    p.x4[i] = a[4];
}

__global__ void __launch_bounds__(NK_T) agg_nokey_kernel(AggSpec S, RowsIO rows, int mode, RowPred pred, int64_t n,
                                                         NoKeyPartial *partials) {
    NoKeyPartial p;
    for (int i = 0; i < AGG_MAX; ++i) p.lo[i] = p.hi[i] = p.x2[i] = p.x3[i] = p.x4[i] = p.cnt[i] = 0, p.f[i] = 0;
    for (int64_t r = (int64_t)blockIdx.x * NK_T + threadIdx.x; r < n; r += (int64_t)gridDim.x * NK_T) {
        if (!pred(r)) continue;
        for (int i = 0; i < S.n_aggs; ++i) {
            if (mode == MODE_RAW && S.kind[i] == TFG_AGG_COUNT_ALL) { p.cnt[i]++; continue; }
            if (S.acc[i] == ACC_REF) { // row r is candidate n0 + 1 + r; first_row takes NULL rows too
                if (S.kind[i] != TFG_AGG_FIRST_ROW && rows.val_null[i] && rows.val_null[i][r]) continue;
                const uint64_t ref = S.ref[i].n0 + 1 + (uint64_t)r;
                if (ref_better(S.kind[i], S.ref[i], ref, p.lo[i])) p.lo[i] = ref;
                continue;
            }
            if (rows.val_null[i] && rows.val_null[i][r]) continue;
            if (S.acc[i] == ACC_ORD) { // min / max / first_row: running max of order keys
                const uint64_t k = ord_enc(S.kind[i], S.src_type[i], load_bits(rows.val[i], val_width(S, mode, i), r));
                p.lo[i] = k > p.lo[i] ? k : p.lo[i];
                p.cnt[i]++;
                continue;
            }
            if (S.kind[i] != TFG_AGG_SUM) {
                p.cnt[i] += mode == MODE_RAW ? 1 : ((const uint64_t *)rows.val[i])[r];
                continue;
            }
            uint64_t lo = 0, hi = 0;
            double f = 0;
            if (S.src_type[i] == TFG_DECIMAL256) {
                nk_add(p, i, (const uint64_t *)rows.val[i] + 4 * r);
                p.cnt[i]++;
                continue;
            }
            load_sum_value(S.src_type[i], rows.val[i], r, lo, hi, f);
            if (S.acc[i] == ACC_F64) p.f[i] += f;
            else if (S.acc[i] == ACC_I256) {
                const uint64_t ext = (int64_t)hi < 0 ? ~0ull : 0ull;
                const uint64_t q[4] = {lo, hi, ext, ext};
                nk_add(p, i, q);
            } else {
                const uint64_t o = p.lo[i];
                p.lo[i] += lo;
                p.hi[i] += hi + (p.lo[i] < o ? 1 : 0);
            }
            p.cnt[i]++;
        }
    }
    // block reduction through LDS, in thread order
    __shared__ NoKeyPartial red[NK_T];
    red[threadIdx.x] = p;
    __syncthreads();
    if (threadIdx.x == 0) {
        NoKeyPartial s = red[0];
        for (int t = 1; t < NK_T; ++t)
            for (int i = 0; i < S.n_aggs; ++i) {
                if (S.acc[i] == ACC_I256) {
                    const uint64_t q[4] = {red[t].lo[i], red[t].hi[i], red[t].x2[i], red[t].x3[i]};
                    nk_add(s, i, q, &red[t].x4[i]);
                } else if (S.acc[i] == ACC_ORD) {
                    s.lo[i] = red[t].lo[i] > s.lo[i] ? red[t].lo[i] : s.lo[i];
                } else if (S.acc[i] == ACC_REF) {
                    if (red[t].lo[i] && ref_better(S.kind[i], S.ref[i], red[t].lo[i], s.lo[i])) s.lo[i] = red[t].lo[i];
                } else {
                    const uint64_t o = s.lo[i];
                    s.lo[i] += red[t].lo[i];
                    s.hi[i] += red[t].hi[i] + (s.lo[i] < o ? 1 : 0);
                }
                s.f[i] += red[t].f[i];
                s.cnt[i] += red[t].cnt[i];
            }
        partials[blockIdx.x] = s;
    }
}

__global__ void agg_nokey_fold_kernel(AggSpec S, const NoKeyPartial *partials, int np, GroupsIO st) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int b = 0; b < np; ++b)
        for (int i = 0; i < S.n_aggs; ++i) {
            const NoKeyPartial &p = partials[b];
            if (S.acc[i] == ACC_F64) ((double *)st.acc[i])[0] += p.f[i];
            else if (S.acc[i] == ACC_I256) { // state (Int256) + partial (5 limbs), checked
                uint64_t *a = (uint64_t *)st.acc[i];
                uint64_t s5[5] = {p.lo[i], p.hi[i], p.x2[i], p.x3[i], p.x4[i]};
                add_i320(s5, a);
                if (!fits_i256(s5) && S.ovf) *S.ovf = 1;
                for (int k = 0; k < 4; ++k) a[k] = s5[k];
            } else if (S.acc[i] == ACC_I128) {
                uint64_t *a = (uint64_t *)st.acc[i];
                const uint64_t o = a[0];
                a[0] += p.lo[i];
                a[1] += p.hi[i] + (a[0] < o ? 1 : 0);
            } else if (S.acc[i] == ACC_I64) ((uint64_t *)st.acc[i])[0] += p.lo[i];
            else if (S.acc[i] == ACC_ORD) {
                uint64_t *a = (uint64_t *)st.acc[i];
                if (p.lo[i] > a[0]) a[0] = p.lo[i];
            } else if (S.acc[i] == ACC_REF) {
                uint64_t *a = (uint64_t *)st.acc[i];
                if (p.lo[i] && ref_better(S.kind[i], S.ref[i], p.lo[i], a[0])) a[0] = p.lo[i];
            }
            if (S.has_cnt[i]) st.cnt[i][0] += p.cnt[i];
        }
}

// ---------------------------------------------------------------- result
struct ResultPtrs {
    void *state[AGG_MAX];
    uint8_t *state_null[AGG_MAX];
    int nullable[AGG_MAX]; // the result column is Nullable (a non-Nullable min / max reports no NULL)
};

// one group's result row: state group s -> output row d
__device__ __forceinline__ void write_result(const AggSpec &S, const GroupsIO &st, uint64_t s, uint64_t d, int key_width,
                                             void *out_keys, uint8_t *out_key_null, const ResultPtrs &res) {
    if (out_keys) {
        const uint64_t k = key_width == 16 ? 0 : st.key[s];
        switch (key_width) {
        case 1: ((uint8_t *)out_keys)[d] = (uint8_t)k; break;
        case 2: ((uint16_t *)out_keys)[d] = (uint16_t)k; break;
        case 4: ((uint32_t *)out_keys)[d] = (uint32_t)k; break;
        case 8: ((uint64_t *)out_keys)[d] = k; break;
        case 16: ((uint4 *)out_keys)[d] = reinterpret_cast<const uint4 *>(st.key)[s]; break;
        default: break;
        }
    }
    if (out_key_null) out_key_null[d] = st.key_null[s];
    for (int i = 0; i < S.n_aggs; ++i) {
        if (S.acc[i] == ACC_REF) continue; // values and NULL flags come from the value store
        if (res.state[i] && S.acc[i] == ACC_ORD) { // min / max: the argument's width
            // no value (a group of NULLs, or no row without key): the type's default, 0
            const bool none = S.has_cnt[i] && st.cnt[i][s] == 0;
            const uint64_t x = none ? 0 : ord_dec(S.kind[i], S.src_type[i], ((const uint64_t *)st.acc[i])[s]);
            switch (val_width(S, MODE_RAW, i)) {
            case 1: ((uint8_t *)res.state[i])[d] = (uint8_t)x; break;
            case 2: ((uint16_t *)res.state[i])[d] = (uint16_t)x; break;
            case 4: ((uint32_t *)res.state[i])[d] = (uint32_t)x; break;
            default: ((uint64_t *)res.state[i])[d] = x; break;
            }
        } else if (res.state[i]) {
            if (S.kind[i] != TFG_AGG_SUM) ((uint64_t *)res.state[i])[d] = st.cnt[i][s];
            else if (S.acc[i] == ACC_I256) {
                ((uint4 *)res.state[i])[2 * d] = ((const uint4 *)st.acc[i])[2 * s];
                ((uint4 *)res.state[i])[2 * d + 1] = ((const uint4 *)st.acc[i])[2 * s + 1];
            } else if (S.acc[i] == ACC_I128) ((uint4 *)res.state[i])[d] = ((const uint4 *)st.acc[i])[s];
            else ((uint64_t *)res.state[i])[d] = ((const uint64_t *)st.acc[i])[s];
        }
        if (res.state_null[i])
            res.state_null[i][d] = ((S.kind[i] == TFG_AGG_SUM || S.acc[i] == ACC_ORD) && S.has_cnt[i] && res.nullable[i])
                                       ? (st.cnt[i][s] == 0) : 0;
    }
}

__global__ void agg_result_kernel(AggSpec S, GroupsIO st, uint64_t n, int key_width, void *out_keys,
                                  uint8_t *out_key_null, ResultPtrs res) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (uint64_t)gridDim.x * blockDim.x)
        write_result(S, st, g, g, key_width, out_keys, out_key_null, res);
}

// the result straight from a tiled consume's bucket-strided groups (pending state): workgroup b
// writes bucket b's cnt[b] groups, found at base[b], to rows off[b].. (off = exclusive scan of cnt)
// — the compaction into a dense state is never run for a consume -> result step
// groups at output rows >= capacity are dropped (a result written before its group count is known)
__global__ void agg_result_buckets_kernel(AggSpec S, GroupsIO st, const uint64_t *cnt, const uint64_t *base,
                                          const uint64_t *off, int key_width, void *out_keys, uint8_t *out_key_null,
                                          ResultPtrs res, uint64_t capacity) {
    const int b = blockIdx.x;
    const uint64_t s0 = base[b], d0 = off[b];
    const uint64_t c = d0 >= capacity ? 0 : min(cnt[b], capacity - d0);
    for (uint64_t j = threadIdx.x; j < c; j += blockDim.x)
        write_result(S, st, s0 + j, d0 + j, key_width, out_keys, out_key_null, res);
}


// The same for B <= RSCAN_MAXB buckets without the scan launches before it: workgroup (b, part)
// sums the counts of buckets 0 .. b - 1 itself (B words from L2), writes rows [part * c / SPLIT,
// (part + 1) * c / SPLIT) of bucket b, and part 0 publishes off[b] (the last bucket also
// off[B] = the group count) for the calls that read the offsets after it
constexpr int RSCAN_MAXB = 1024, RSCAN_SPLIT = 4;
__global__ void __launch_bounds__(256) agg_result_buckets_scan_kernel(AggSpec S, GroupsIO st, const uint64_t *cnt,
                                                                     const uint64_t *base, uint64_t *off, int B,
                                                                     int key_width, void *out_keys, uint8_t *out_key_null,
                                                                     ResultPtrs res, uint64_t capacity) {
    __shared__ uint64_t wsum[4];
    const int b = (int)(blockIdx.x / RSCAN_SPLIT), part = (int)(blockIdx.x % RSCAN_SPLIT);
    uint64_t x = 0;
    for (int i = threadIdx.x; i < b; i += 256) x += cnt[i];
    for (int d = 32; d > 0; d >>= 1) x += __shfl_down(x, d, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = x;
    __syncthreads();
    const uint64_t d0 = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    const uint64_t cb = cnt[b];
    if (part == 0 && threadIdx.x == 0) {
        off[b] = d0;
        if (b == B - 1) off[B] = d0 + cb;
    }
    const uint64_t c = d0 >= capacity ? 0 : min(cb, capacity - d0);
    const uint64_t j0 = c * (uint64_t)part / RSCAN_SPLIT, j1 = c * (uint64_t)(part + 1) / RSCAN_SPLIT;
    const uint64_t s0 = base[b];
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += 256)
        write_result(S, st, s0 + j, d0 + j, key_width, out_keys, out_key_null, res);
}
// ---- the fused String-key result (one packed String key, the groups of a tiled consume still in
// their buckets): the chars of each bucket's keys, their scan, then per bucket its groups' result
// rows with the key bytes written straight into the ColumnString — no packed-key copy, no
// per-group length scan, no unpack pass (convertToBlockImplFinal's insertKeyIntoColumns)
constexpr int RSK_T = 256;
__global__ void __launch_bounds__(RSK_T) pend_key_chars_kernel(const uint4 *keys, const uint64_t *cnt, const uint64_t *base,
                                                           uint64_t *chars) {
    __shared__ uint64_t red[RSK_T / 64];
    const int b = blockIdx.x;
    const uint64_t s0 = base[b], c = cnt[b];
    uint64_t t = 0;
    for (uint64_t j = threadIdx.x; j < c; j += RSK_T) t += ((keys[s0 + j].w >> 24) & 0x7Fu) + 1; // bytes + '\0'
    for (int d = 32; d > 0; d >>= 1) t += __shfl_down(t, d, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t sum = 0;
        for (int w = 0; w < RSK_T / 64; ++w) sum += red[w];
        chars[b] = sum;
    }
}

// workgroup b: bucket b's groups (rows off[b].., chars from choff[b]) in chunks of RSK_T; a
// chunk's key bytes are placed in LDS by a block scan of their lengths and copied out with
// consecutive lanes on consecutive bytes.  Rows >= capacity and chars >= chars_capacity dropped.
__global__ void __launch_bounds__(RSK_T) agg_result_str_keys_kernel(AggSpec S, GroupsIO st, const uint64_t *cnt,
                                                                const uint64_t *base, const uint64_t *off,
                                                                const uint64_t *choff, uint64_t capacity,
                                                                uint64_t chars_capacity, uint8_t *out_chars,
                                                                uint64_t *out_offsets, uint8_t *out_null, ResultPtrs res) {
    __shared__ uint8_t stage[RSK_T * 16];
    __shared__ uint32_t wsum[RSK_T / 64];
    const int b = blockIdx.x;
    const uint64_t s0 = base[b], d0 = off[b];
    const uint64_t c = d0 >= capacity ? 0 : min(cnt[b], capacity - d0);
    const uint4 *keys = reinterpret_cast<const uint4 *>(st.key);
    uint64_t run = choff[b];
    for (uint64_t j0 = 0; j0 < c; j0 += RSK_T) { // uniform
        const uint64_t j = j0 + threadIdx.x;
        const bool have = j < c;
        uint4 q = make_uint4(0, 0, 0, 0);
        uint32_t len1 = 0;
        if (have) {
            q = keys[s0 + j];
            len1 = ((q.w >> 24) & 0x7Fu) + 1;
        }
        uint32_t x = len1; // block exclusive scan of the lengths
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if ((int)(threadIdx.x & 63) >= d) x += y;
        }
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = x;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < RSK_T / 64; ++w) {
            if (w < (int)(threadIdx.x >> 6)) pre += wsum[w];
            tot += wsum[w];
        }
        const uint32_t pos = pre + x - len1;
        if (have) {
            const uint64_t w0 = ((uint64_t)q.y << 32) | q.x, w1 = ((uint64_t)q.w << 32) | q.z;
            for (uint32_t i = 0; i + 1 < len1; ++i)
                stage[pos + i] = (uint8_t)(i < 8 ? w0 >> (i * 8) : w1 >> ((i - 8) * 8));
            stage[pos + len1 - 1] = 0;
            out_offsets[d0 + j] = run + pos + len1;
            if (out_null) out_null[d0 + j] = (uint8_t)(w1 >> 63);
            write_result(S, st, s0 + j, d0 + j, 16, nullptr, nullptr, res);
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < tot; i += RSK_T)
            if (run + i < chars_capacity) out_chars[run + i] = stage[i];
        run += tot;
        __syncthreads(); // stage / wsum are rewritten by the next chunk
    }
}

__global__ void agg_state_add_kernel(AggSpec S, GroupsIO dst, GroupsIO src) { // without-key merge
    if (threadIdx.x || blockIdx.x) return;
    for (int i = 0; i < S.n_aggs; ++i) {
        if (S.acc[i] == ACC_F64) ((double *)dst.acc[i])[0] += ((const double *)src.acc[i])[0];
        else if (S.acc[i] == ACC_I256) { // checked (types.h:35)
            uint64_t *a = (uint64_t *)dst.acc[i];
            const uint64_t *b = (const uint64_t *)src.acc[i];
            uint64_t s5[5] = {a[0], a[1], a[2], a[3], (int64_t)a[3] < 0 ? ~0ull : 0ull};
            add_i320(s5, b);
            if (!fits_i256(s5) && S.ovf) *S.ovf = 1;
            for (int k = 0; k < 4; ++k) a[k] = s5[k];
        }
        else if (S.acc[i] == ACC_I128) {
            uint64_t *a = (uint64_t *)dst.acc[i];
            const uint64_t *b = (const uint64_t *)src.acc[i];
            const uint64_t o = a[0];
            a[0] += b[0];
            a[1] += b[1] + (a[0] < o ? 1 : 0);
        } else if (S.acc[i] == ACC_I64) ((uint64_t *)dst.acc[i])[0] += ((const uint64_t *)src.acc[i])[0];
        else if (S.acc[i] == ACC_ORD) {
            const uint64_t b = ((const uint64_t *)src.acc[i])[0];
            if (b > ((uint64_t *)dst.acc[i])[0]) ((uint64_t *)dst.acc[i])[0] = b;
        } else if (S.acc[i] == ACC_REF) { // the source's store follows the destination's n0 entries
            const uint64_t b = ((const uint64_t *)src.acc[i])[0];
            uint64_t *a = (uint64_t *)dst.acc[i];
            if (b && ref_better(S.kind[i], S.ref[i], S.ref[i].n0 + b, a[0])) a[0] = S.ref[i].n0 + b;
        }
        if (S.has_cnt[i]) dst.cnt[i][0] += src.cnt[i][0];
    }
}

// bucket of a key: Fibonacci radix of the zero-extended key bits (NULL key -> bucket 0)
struct SelBucket {
    const void *key;
    const uint8_t *key_null;
    int width;
    uint32_t shift;
    static constexpr bool needs_crc = false;
    static constexpr bool fib_radix = false;
    __device__ __forceinline__ Loaded load(int64_t r) const {
        return Loaded{load_bits(key, width, r), key_null ? (uint32_t)key_null[r] : 0u};
    }
    __device__ __forceinline__ uint32_t part(const uint32_t (*t)[256], const Loaded &l, int64_t) const {
        return l.null ? 0u : fib_part(l.bits, shift);
    }
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const { return part(t, load(r), r); }
};

// the fast path's selector: 8-byte keys without a NULL map
struct SelBucket8 {
    const uint64_t *key;
    uint32_t shift;
    static constexpr bool needs_crc = false;
    static constexpr bool fib_radix = true;
    __device__ __forceinline__ Loaded load(int64_t r) const { return Loaded{key[r], 0u}; }
    __device__ __forceinline__ uint32_t part(const uint32_t (*)[256], const Loaded &l, int64_t) const {
        return fib_part(l.bits, shift);
    }
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const { return part(t, load(r), r); }
};

// wide keys: the radix of the key's tag (the bucket kernel derives the slot from the same product)
struct SelWide {
    const uint4 *key;
    uint32_t shift;
    static constexpr bool needs_crc = false;
    static constexpr bool fib_radix = false;
    __device__ __forceinline__ Loaded load(int64_t r) const {
        const uint4 q = key[r];
        return Loaded{wide_tag(((uint64_t)q.y << 32) | q.x, ((uint64_t)q.w << 32) | q.z), 0u};
    }
    __device__ __forceinline__ uint32_t part(const uint32_t (*)[256], const Loaded &l, int64_t) const {
        return fib_part(l.bits, shift);
    }
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const { return part(t, load(r), r); }
};

// Wide keys on the tiled path (consume_wide_tiled): the selector hands the 16-byte key to the
// staged partition as record words 0 and 1; the radix is the Fibonacci radix of its tag.
struct SelWide2 { // packed keys (keys128 after pack_keys_kernel)
    const uint4 *key;
    uint32_t shift;
    static constexpr bool needs_crc = false;
    static constexpr bool fib_radix = false;
    static constexpr bool wide_key = true;
    __device__ __forceinline__ Loaded load(int64_t r) const {
        const uint4 q = key[r];
        return Loaded{((uint64_t)q.y << 32) | q.x, 0u, ((uint64_t)q.w << 32) | q.z};
    }
    __device__ __forceinline__ uint32_t part(const uint32_t (*)[256], const Loaded &l, int64_t) const {
        return fib_part(wide_tag(l.bits, l.hi), shift);
    }
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const { return part(t, load(r), r); }
};

// key_string (HashMethodString with the collator's sort key, ColumnsHashing.h:179-241) packed
// while it is loaded, exactly as pack_keys_kernel packs it: bytes 0-14 = the sort key (<= 15
// bytes), byte 15 = its length, NULL = 0x80 in byte 15.  The bytes come from the aligned 8-byte
// words that cover them (an aligned word holding a valid byte never leaves its page).
struct SelWideStr {
    const uint8_t *chars;
    const uint64_t *offsets;
    const uint8_t *nullmap;
    int collator;
    unsigned *err; // set when a sort key is longer than 15 bytes (serialized method needed)
    uint32_t shift;
    static constexpr bool needs_crc = false;
    static constexpr bool fib_radix = false;
    static constexpr bool wide_key = true;
    __device__ __forceinline__ Loaded load(int64_t r) const {
        uint64_t lo = 0, hi = 0;
        if (nullmap && nullmap[r]) return Loaded{0, 0u, 0x80ull << 56};
        const uint64_t s = r ? offsets[r - 1] : 0, e = offsets[r];
        int64_t len = (int64_t)(e - s) - 1; // ColumnString rows end with '\0'
        const uint8_t *c = chars + s;
        if (collator == TFG_COLLATOR_BIN_PADDING)
            while (len > 0 && c[len - 1] == ' ') --len; // BinCollatorSortKey<true>: right-trim
        if (len > 15) {
            atomicOr(err, 1u);
            len = 15;
        }
        if (len > 0) {
            const uintptr_t addr = (uintptr_t)c;
            const uint64_t *w = (const uint64_t *)(addr & ~(uintptr_t)7);
            const int sh = (int)(addr & 7) * 8;
            const int nw = (int)(((addr + len - 1) >> 3) - (addr >> 3)) + 1; // 1..3 words
            const uint64_t w0 = w[0], w1 = nw > 1 ? w[1] : 0ull, w2 = nw > 2 ? w[2] : 0ull;
            lo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
            hi = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
            if (len < 8) {
                lo &= (1ull << (len * 8)) - 1;
                hi = 0;
            } else {
                hi = len == 8 ? 0ull : hi & ((1ull << ((len - 8) * 8)) - 1);
            }
        }
        hi |= (uint64_t)len << 56;
        return Loaded{lo, 0u, hi};
    }
    __device__ __forceinline__ uint32_t part(const uint32_t (*)[256], const Loaded &l, int64_t) const {
        return fib_part(wide_tag(l.bits, l.hi), shift);
    }
    __device__ __forceinline__ uint32_t operator()(const uint32_t (*t)[256], int64_t r) const { return part(t, load(r), r); }
};

// ---------------------------------------------------------------- two-level tiled partition
// Buckets past 256 (10M-group GROUP BYs) leave a one-level tiled partition with runs of < 1 row
// per (bucket, tile).  Pass 1 tiles the rows by the top `coarse` bits of the radix; pass 2
// (regroup_tiled_kernel) walks each coarse bucket's runs in order, cuts them into new tiles of
// RG_TR rows that hold one coarse bucket each, and counting-sorts every tile by the next
// `fine` = 6 bits: the bucket kernel of (coarse c, fine f) then reads runs of ~RG_TR / 64 rows
// from the tiles [tile_base[c], tile_base[c + 1]).
#ifndef TFG_RG_TR
#define TFG_RG_TR 1024 // r06m/n (C5, 512 threads): 1024 rows 0.97 ms, 1536 1.03, 3072 1.94; 512 / 768 /
                       // 1024 threads at 512 / 768 / 1024 rows 1.16 / 1.41 / 1.19
#endif
#ifndef TFG_RG_T
#define TFG_RG_T 512
#endif
constexpr int RG_T = TFG_RG_T;
constexpr int RG_TR = TFG_RG_TR;
constexpr int RG_W = 1024; // pass-1 runs staged in LDS per window
constexpr int RG_FINE_BITS = 6;
constexpr int RG_FINE = 1 << RG_FINE_BITS;

// per coarse bucket: exclusive prefix of its run lengths over the pass-1 tiles (T1 + 1 entries)
__global__ void __launch_bounds__(1024) regroup_prefix_kernel(const uint32_t *hist1, int T1, uint32_t *runpref) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    const int c = blockIdx.x;
    const uint32_t *h = hist1 + (size_t)c * T1;
    uint32_t *out = runpref + (size_t)c * (T1 + 1);
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int t0 = 0; t0 < T1; t0 += 1024) {
        const int t = t0 + (int)threadIdx.x;
        const uint32_t v = t < T1 ? h[t] >> 16 : 0u;
        uint32_t x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if ((int)(threadIdx.x & 63) >= d) x += y;
        }
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = x;
        __syncthreads();
        uint32_t off = carry;
        for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) off += wsum[w];
        if (t < T1) out[t] = off + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry = off + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) out[T1] = carry;
}

// tile_base[c] = first pass-2 tile of coarse bucket c: one 1024-thread workgroup scans the
// buckets' tile counts (B1 <= 1024; a single-thread loop over the buckets' dependent loads took
// 61 us at 256 buckets)
__global__ void __launch_bounds__(1024) regroup_tile_base_kernel(const uint32_t *runpref, int T1, int B1, uint32_t *tile_base) {
    __shared__ uint32_t wsum[16];
    const int c = (int)threadIdx.x;
    const uint32_t v = c < B1 ? (runpref[(size_t)c * (T1 + 1) + T1] + RG_TR - 1) / RG_TR : 0u;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if ((c & 63) >= d) x += y;
    }
    if ((c & 63) == 63) wsum[c >> 6] = x;
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < (c >> 6); ++w) off += wsum[w];
    if (c < B1) tile_base[c] = off + x - v;
    if (c == B1 - 1) tile_base[B1] = off + x;
}

// where pass-2 tile k reads from: its coarse bucket c (-1: past the last tile), the pass-1 runs
// t0 .. t0 + m - 1 that cover its rows [x0, x1) of the bucket.  One thread per tile, all tiles at
// once (the searches' dependent loads overlap across threads instead of heading every
// workgroup of the regroup kernel)
struct RgDesc {
    int c, t0, m;
    uint32_t x0, x1;
};

__global__ void regroup_desc_kernel(const uint32_t *runpref, int T1, const uint32_t *tile_base, int B1, int T2,
                                    RgDesc *desc) {
    const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= T2) return;
    RgDesc d{-1, 0, 0, 0, 0};
    if ((uint32_t)k < tile_base[B1]) {
        int lo = 0, hi = B1; // coarse bucket of tile k: tile_base[c] <= k < tile_base[c + 1]
        while (hi - lo > 1) {
            const int mid = (lo + hi) / 2;
            if (tile_base[mid] <= (uint32_t)k) lo = mid;
            else hi = mid;
        }
        const uint32_t *pr = runpref + (size_t)lo * (T1 + 1);
        const uint32_t n_c = pr[T1];
        const uint32_t x0 = (uint32_t)(k - (int)tile_base[lo]) * RG_TR;
        const uint32_t x1 = min(x0 + (uint32_t)RG_TR, n_c);
        // runs covering [x0, x1): t0 = last tile with pr[t] <= x0, t1 = first with pr[t] >= x1
        int a = 0, b = T1;
        while (b - a > 1) {
            const int mid = (a + b) / 2;
            if (pr[mid] <= x0) a = mid;
            else b = mid;
        }
        int lo2 = a, hi2 = T1; // pr[T1] = n_c >= x1
        while (hi2 - lo2 > 1) {
            const int mid = (lo2 + hi2) / 2;
            if (pr[mid] >= x1) hi2 = mid;
            else lo2 = mid;
        }
        d = RgDesc{lo, a, hi2 - a, x0, x1};
    }
    desc[k] = d;
}

// one workgroup per pass-2 tile (grid = an upper bound; tiles past tile_base[B1] exit)
template <int NCOL>
__global__ void __launch_bounds__(RG_T) regroup_tiled_kernel(const uint64_t *rec1, const uint32_t *hist1, int T1, int TR1,
                                                             const uint32_t *runpref, const RgDesc *desc,
                                                             uint32_t fine_shift, uint64_t *rec2, uint32_t *hist2, int T2,
                                                             int narrow_ok) {
    __shared__ uint64_t stage[RG_TR * NCOL];
    __shared__ uint32_t rpref[RG_W + 2], rent[RG_W + 2];
    __shared__ uint32_t fh[RG_FINE], fs[RG_FINE];
    __shared__ uint32_t s_wide; // a row of this tile has a key that is not narrow (NCOL == 3)
    const int k = blockIdx.x;
    const RgDesc d = desc[k];
    if (threadIdx.x < RG_FINE) fh[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_wide = 0;
    const int c = d.c;
    if (c < 0) return;
    const int t0 = d.t0, m = d.m;
    const uint32_t x0 = d.x0, x1 = d.x1;
    const uint32_t *pr = runpref + (size_t)c * (T1 + 1);
    const uint32_t *hc = hist1 + (size_t)c * T1;
    constexpr int PER = RG_TR / RG_T;
    uint64_t v[PER][NCOL];
    uint32_t bq[PER];
    int64_t row[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) row[q] = -1;
    // the runs t0 .. t0 + m - 1 in windows of RG_W (more than one only when many short or empty
    // runs of a sparse coarse bucket pile up): a row's run is the last j with rpref[j] <= x
    for (int w0 = 0; w0 < m; w0 += RG_W) {
        const int wm = min(RG_W, m - w0);
        for (int j = threadIdx.x; j <= wm; j += RG_T) {
            rpref[j] = pr[t0 + w0 + j];
            rent[j] = j < wm ? hc[t0 + w0 + j] : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint32_t x = x0 + (uint32_t)(q * RG_T + threadIdx.x);
            if (x >= x1 || row[q] >= 0 || x >= rpref[wm]) continue;
            int lo = 0;
            for (int st = wm > 1 ? 1 << (31 - __clz(wm - 1)) : 0; st > 0; st >>= 1)
                if (lo + st < wm && rpref[lo + st] <= x) lo += st;
            // the run's start in its tile (bit 15 of the entry: a narrow tile, NCOL == 3 only)
            const uint32_t e = rent[lo];
            row[q] = (int64_t)(t0 + w0 + lo) * TR1 + (e & (TILE_NARROW - 1)) + (x - rpref[lo]);
            if (NCOL == 3 && (e & TILE_NARROW)) row[q] |= (int64_t)1 << 62;
        }
        __syncthreads();
    }
    bool wide = false;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        bq[q] = 0xFFFFFFFFu;
        if (row[q] < 0) continue;
        if (NCOL == 3 && (row[q] >> 62)) { // narrow pass-1 tile: 20-byte records (nrec_load)
            const int64_t rr = row[q] & (((int64_t)1 << 62) - 1);
            const int64_t tile = rr / TR1, pos = rr - tile * TR1;
            uint32_t h;
            nrec_load(rec1 + (size_t)tile * TR1 * 3, (uint32_t)pos, v[q][0], h, v[q][NCOL - 1]);
            v[q][1] = wide_wide_hi(h);
            row[q] = rr;
            continue;
        }
        const uint64_t *r = rec1 + row[q] * NCOL;
#pragma unroll
        for (int w = 0; w < NCOL; ++w) v[q][w] = r[w];
        if (NCOL == 3) wide |= !wide_hi_narrowable(v[q][1]);
    }
    if (NCOL == 3 && wide) s_wide = 1;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        if (row[q] < 0) continue;
        const uint32_t f = fib_part(wide_tag(v[q][0], v[q][1]), fine_shift) & (RG_FINE - 1);
        bq[q] = f | (atomicAdd(&fh[f], 1u) << 16);
    }
    __syncthreads();
    const bool narrow_out = NCOL == 3 && narrow_ok && !s_wide; // every row of the tile narrow: 20 B a row out
    if (threadIdx.x < 64) { // one wave: exclusive scan of the 64 fine counts
        const uint32_t cnt = fh[threadIdx.x];
        uint32_t xs = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(xs, d, 64);
            if ((int)threadIdx.x >= d) xs += y;
        }
        fs[threadIdx.x] = xs - cnt;
        hist2[(size_t)threadIdx.x * T2 + k] = (xs - cnt) | (narrow_out ? TILE_NARROW : 0u) | (cnt << 16);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        if (bq[q] == 0xFFFFFFFFu) continue;
        const uint32_t s = fs[bq[q] & 0xFFFFu] + (bq[q] >> 16);
#pragma unroll
        for (int w = 0; w < NCOL; ++w) stage[s * NCOL + w] = v[q][w];
    }
    __syncthreads();
    const uint32_t rows = x1 - x0;
    uint64_t *out = rec2 + (size_t)k * RG_TR * NCOL;
    if (narrow_out) { // 20-byte records (nrec_store)
        for (uint32_t i = threadIdx.x; i < rows; i += RG_T)
            nrec_store(out, i, stage[i * NCOL], wide_narrow_hi(stage[i * NCOL + 1]), stage[i * NCOL + NCOL - 1]);
        return;
    }
    for (uint32_t i = threadIdx.x; i < rows * NCOL; i += RG_T) out[i] = stage[i];
}

// ---------------------------------------------------------------- wide-key packing
// keys128 (Aggregator.cpp:394-537 chooses keys128 / nullable_keys128 for several fixed keys of
// <= 16 bytes, packing them with packFixed, Common/ColumnsHashing.h:324-480) and key_string
// (HashMethodString, ColumnsHashing.h:179-241: the key is the collator's sort key of the row)
// become one 16-byte key:
//   fixed keys: the columns' little-endian bytes at consecutive offsets; when the sum of the
//               widths is <= 15, byte 15 holds the NULL bit of each nullable key (its value
//               bytes are then zero), like nullable_keys128's bitmap;
//   String:     the sort-key bytes (<= 15), zero padded, with byte 15 = length; NULL = 0x80.
constexpr int WK_FIXED = 1, WK_STRING = 2;
struct KeyPack {
    int kind;
    int nkeys;
    int width[4];
    int off[4];
    const void *col[4];
    const uint8_t *nullmap[4];
    const uint64_t *offsets; // String
    int collator;
};

__global__ void pack_keys_kernel(KeyPack kp, int64_t n, uint4 *out, unsigned *err) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        uint64_t w[2] = {0, 0};
        if (kp.kind == WK_STRING) {
            if (kp.nullmap[0] && kp.nullmap[0][r]) {
                w[1] = 0x80ull << 56;
            } else {
                const uint64_t s = r ? kp.offsets[r - 1] : 0, e = kp.offsets[r];
                const uint8_t *c = (const uint8_t *)kp.col[0] + s;
                int64_t len = (int64_t)(e - s) - 1; // ColumnString rows end with '\0'
                if (kp.collator == TFG_COLLATOR_BIN_PADDING)
                    while (len > 0 && c[len - 1] == ' ') --len; // BinCollatorSortKey<true>: right-trim
                if (len > 15) {
                    atomicOr(err, 1u);
                    len = 15;
                }
                for (int i = 0; i < (int)len; ++i) w[i >> 3] |= (uint64_t)c[i] << ((i & 7) * 8);
                w[1] |= (uint64_t)len << 56;
            }
        } else {
            uint64_t nb = 0;
            for (int j = 0; j < kp.nkeys; ++j) {
                if (kp.nullmap[j] && kp.nullmap[j][r]) {
                    nb |= 1ull << j;
                    continue;
                }
                const int wd = kp.width[j], o = kp.off[j];
                uint64_t lo = 0, hi = 0;
                if (wd == 16) {
                    lo = ((const uint64_t *)kp.col[j])[2 * r];
                    hi = ((const uint64_t *)kp.col[j])[2 * r + 1];
                } else {
                    lo = load_bits(kp.col[j], wd, r);
                }
                // place wd bytes at byte offset o
                if (o < 8) {
                    w[0] |= lo << (o * 8);
                    if (o > 0) w[1] |= lo >> ((8 - o) * 8);
                    if (wd == 16) w[1] |= hi << (o * 8);
                } else {
                    w[1] |= lo << ((o - 8) * 8);
                }
            }
            if (nb) w[1] |= nb << 56;
        }
        uint4 q;
        q.x = (unsigned)w[0];
        q.y = (unsigned)(w[0] >> 32);
        q.z = (unsigned)w[1];
        q.w = (unsigned)(w[1] >> 32);
        out[r] = q;
    }
}

// packed String keys -> lengths + 1 (the '\0' each ColumnString row ends with)
// n_dev (optional): the group count on the device, <= n slots (a result written before its count
// is read): slots past it get length 0
__global__ void wide_str_len_kernel(const uint4 *keys, uint64_t n, uint64_t *len1, const uint64_t *n_dev) {
    const uint64_t G = n_dev ? min(*n_dev, n) : n;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (uint64_t)gridDim.x * blockDim.x)
        len1[g] = g < G ? ((keys[g].w >> 24) & 0x7Fu) + 1 : 0;
}

// packed keys -> the key columns of the result Block (convertToBlockImplFinal's insertKeyIntoColumns)
struct KeyOut {
    void *col[4];
    uint64_t *offsets;        // String: end offsets
    uint8_t *nullmap[4];
};
__global__ void unpack_keys_kernel(KeyPack kp, const uint4 *keys, const uint64_t *start, uint64_t n, KeyOut ko,
                                   const uint64_t *n_dev) {
    if (n_dev) n = min(*n_dev, n); // the count on the device (wide_str_len_kernel)
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 q = keys[g];
        const uint64_t w[2] = {((uint64_t)q.y << 32) | q.x, ((uint64_t)q.w << 32) | q.z};
        if (kp.kind == WK_STRING) {
            const int len = (int)((w[1] >> 56) & 0x7F);
            const uint64_t s = start[g];
            uint8_t *c = (uint8_t *)ko.col[0] + s;
            for (int i = 0; i < len; ++i) c[i] = (uint8_t)(w[i >> 3] >> ((i & 7) * 8));
            c[len] = 0;
            ko.offsets[g] = s + len + 1;
            if (ko.nullmap[0]) ko.nullmap[0][g] = (w[1] >> 63) ? 1 : 0;
            continue;
        }
        const uint64_t nb = kp.off[kp.nkeys - 1] + kp.width[kp.nkeys - 1] <= 15 ? (w[1] >> 56) : 0;
        for (int j = 0; j < kp.nkeys; ++j) {
            const int wd = kp.width[j], o = kp.off[j];
            if (ko.nullmap[j]) ko.nullmap[j][g] = (nb >> j) & 1;
            if (!ko.col[j]) continue;
            uint64_t lo = o < 8 ? (w[0] >> (o * 8)) | (o > 0 ? w[1] << ((8 - o) * 8) : 0) : w[1] >> ((o - 8) * 8);
            switch (wd) {
            case 1: ((uint8_t *)ko.col[j])[g] = (uint8_t)lo; break;
            case 2: ((uint16_t *)ko.col[j])[g] = (uint16_t)lo; break;
            case 4: ((uint32_t *)ko.col[j])[g] = (uint32_t)lo; break;
            case 8: ((uint64_t *)ko.col[j])[g] = lo; break;
            default: // 16: a single Decimal128 / Int128 key at offset 0
                ((uint64_t *)ko.col[j])[2 * g] = w[0];
                ((uint64_t *)ko.col[j])[2 * g + 1] = w[1];
            }
        }
    }
}

// IColumn::updateWeakHash32 of the key columns, read from their packed form (the sender of a
// two-phase GROUP BY hashes the partial groups it holds packed, without unpacking them first):
// a String key is its bytes (<= 15, right-trimmed already for BIN_PADDING, a sort key already for
// the case-insensitive collators) hashed as ::updateWeakHash32(bytes) (Hash.h:148-214); fixed keys
// are their values as hash_key_row feeds them to crc32q; a NULL key leaves the hash as it is
// (ColumnNullable.cpp:131-173)
struct PackTypes {
    int type[4];
};
__global__ void __launch_bounds__(256) weak_hash_packed_kernel(KeyPack kp, PackTypes pt, const uint4 *keys, int64_t n,
                                                               uint32_t *h) {
    __shared__ uint32_t crc[8][256];
    load_crc_lds(crc);
    __syncthreads();
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (int64_t)gridDim.x * blockDim.x) {
        const uint4 q = keys[g];
        const uint64_t w0 = ((uint64_t)q.y << 32) | q.x, w1 = ((uint64_t)q.w << 32) | q.z;
        uint32_t x = h[g];
        if (kp.kind == WK_STRING) {
            if (!(w1 >> 63)) {
                const int len = (int)((w1 >> 56) & 0x7F);
                const uint64_t hi = w1 & 0x00FFFFFFFFFFFFFFull; // bytes 8..14
                if (len < 8) {
                    x = crc32c_u64(crc, x, w0 | ((uint64_t)len << 56)); // w0 holds only the len bytes
                } else {
                    x = crc32c_u64(crc, x, w0);
                    const int tail = len - 8;
                    if (tail) { // the 8 bytes ending at len, the low 8 - tail of them masked off
                        const int sh = 8 * tail; // bytes [len - 8, len) = (hi:w0) >> 8 * (len - 8)
                        uint64_t word = (w0 >> sh) | (hi << (64 - sh));
                        word &= ~0ull << (8 * (8 - tail));
                        x = crc32c_u64(crc, x, word | (uint64_t)tail);
                    }
                }
            }
            h[g] = x;
            continue;
        }
        const uint64_t nb = kp.off[kp.nkeys - 1] + kp.width[kp.nkeys - 1] <= 15 ? (w1 >> 56) : 0;
        for (int j = 0; j < kp.nkeys; ++j) {
            if ((nb >> j) & 1) continue; // NULL
            const int wd = kp.width[j], o = kp.off[j];
            const uint64_t lo = o < 8 ? (w0 >> (o * 8)) | (o > 0 ? w1 << ((8 - o) * 8) : 0) : w1 >> ((o - 8) * 8);
            uint64_t v;
            switch (pt.type[j]) {
            case TFG_INT8: v = (uint64_t)(int64_t)(int8_t)lo; break;
            case TFG_INT16: v = (uint64_t)(int64_t)(int16_t)lo; break;
            case TFG_INT32: case TFG_DECIMAL32: v = (uint64_t)(int64_t)(int32_t)lo; break;
            case TFG_UINT8: v = lo & 0xFF; break;
            case TFG_UINT16: v = lo & 0xFFFF; break;
            case TFG_UINT32: v = lo & 0xFFFFFFFFull; break;
            case TFG_FLOAT32: {
                const uint32_t u = (uint32_t)lo;
                float f;
                memcpy(&f, &u, 4);
                v = float_to_u64_x86(f);
                break;
            }
            case TFG_FLOAT64: {
                double d;
                memcpy(&d, &lo, 8);
                v = float_to_u64_x86(d);
                break;
            }
            case TFG_DECIMAL128: // a single 16-byte key at offset 0
                x = crc32c_u64(crc, x, w0);
                x = crc32c_u64(crc, x, w1);
                continue;
            default: v = wd == 8 ? lo : lo; break; // Int64 / UInt64 / Decimal64
            }
            x = crc32c_u64(crc, x, v);
        }
        h[g] = x;
    }
}

// ---------------------------------------------------------------- row-reference value stores
// (ACC_REF aggregates, agg_dev.h): the candidates of a consume are the store (refs 1..n0) and the
// consumed column (n0 + 1 + r); after it every group's winning value is copied into a new store in
// group order and the group's reference becomes g + 1.
__global__ void ref_iota_kernel(uint64_t *out, uint64_t n0, int64_t n) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        out[r] = n0 + 1 + (uint64_t)r;
}
// a merge's source states: references into the source's store, after the destination's n0 entries
__global__ void ref_shift_kernel(const uint64_t *in, uint64_t n0, int64_t n, uint64_t *out) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        out[r] = in[r] ? in[r] + n0 : 0;
}

struct RefCol {           // one candidate source
    const uint8_t *val;   // fixed-width values, or String chars
    const uint64_t *off;  // String: end offsets
    const uint8_t *nul;   // NULL flags (null: none)
};
__device__ __forceinline__ const RefCol &ref_pick(uint64_t ref, uint64_t n0, const RefCol &s0, const RefCol &s1,
                                                  uint64_t &idx) {
    idx = ref > n0 ? ref - n0 - 1 : ref - 1;
    return ref > n0 ? s1 : s0;
}
// a state reference must name one of the n0 + n1 candidates: anything else (never dereferenced)
// sets the aggregator's error flag and reads as "no value"
__device__ __forceinline__ bool ref_ok(uint64_t ref, uint64_t lim, unsigned *err) {
    if (ref <= lim) return true;
    if (err) atomicOr(err, 2u);
    return false;
}

__global__ void ref_store_fixed_kernel(uint64_t *acc, uint64_t G, uint64_t n0, uint64_t n1, unsigned *err, int w,
                                       RefCol s0, RefCol s1, uint8_t *val, uint8_t *nul) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t ref = acc[g];
        if (!ref_ok(ref, n0 + n1, err)) ref = acc[g] = 0;
        uint64_t q[4] = {0, 0, 0, 0};
        uint8_t isnull = 1;
        if (ref) {
            uint64_t idx;
            const RefCol &c = ref_pick(ref, n0, s0, s1, idx);
            isnull = c.nul ? (c.nul[idx] != 0) : 0;
            if (!isnull) {
                if (w >= 8) {
                    for (int k = 0; k < w / 8; ++k) q[k] = reinterpret_cast<const uint64_t *>(c.val)[idx * (w / 8) + k];
                } else {
                    q[0] = load_bits(c.val, w, (int64_t)idx);
                }
            }
            acc[g] = g + 1;
        }
        nul[g] = isnull;
        switch (w) { // a NULL or absent value stores the default, 0 (ColumnNullable::insertDefault)
        case 1: val[g] = (uint8_t)q[0]; break;
        case 2: reinterpret_cast<uint16_t *>(val)[g] = (uint16_t)q[0]; break;
        case 4: reinterpret_cast<uint32_t *>(val)[g] = (uint32_t)q[0]; break;
        default:
            for (int k = 0; k < w / 8; ++k) reinterpret_cast<uint64_t *>(val)[g * (w / 8) + k] = q[k];
        }
    }
}

// String store: bytes of each group's value with its '\0' (NULL / absent: the empty String)
__global__ void ref_store_len_kernel(const uint64_t *acc, uint64_t G, uint64_t n0, uint64_t n1, unsigned *err, RefCol s0,
                                     RefCol s1, uint64_t *len) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t ref = acc[g];
        if (!ref_ok(ref, n0 + n1, err)) ref = 0;
        uint64_t l = 1;
        if (ref) {
            uint64_t idx;
            const RefCol &c = ref_pick(ref, n0, s0, s1, idx);
            if (!(c.nul && c.nul[idx])) l = c.off[idx] - (idx ? c.off[idx - 1] : 0);
        }
        len[g] = l;
    }
}
__global__ void ref_store_str_kernel(uint64_t *acc, uint64_t G, uint64_t n0, uint64_t n1, RefCol s0, RefCol s1,
                                     const uint64_t *start, uint8_t *chars, uint8_t *nul) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t ref = acc[g];
        if (ref > n0 + n1) ref = acc[g] = 0; // flagged by ref_store_len_kernel
        uint8_t *o = chars + start[g];
        uint8_t isnull = 1;
        if (ref) {
            uint64_t idx;
            const RefCol &c = ref_pick(ref, n0, s0, s1, idx);
            isnull = c.nul ? (c.nul[idx] != 0) : 0;
            if (!isnull) {
                const uint64_t b = idx ? c.off[idx - 1] : 0, e = c.off[idx];
                for (uint64_t k = b; k < e; ++k) *o++ = c.val[k];
            }
            acc[g] = g + 1;
        }
        if (isnull) *o = 0;
        nul[g] = isnull;
    }
}

} // namespace tfg

using namespace tfg;

// The value store of one ACC_REF aggregate: n entries in group order.  Its buffers are plain
// device allocations that grow on demand (grow_buf) and are reused call after call: the store and
// a spare one are swapped by every rebuild.
struct RefStore {
    uint8_t *val = nullptr;   // fixed: n values of the argument's width; String: chars
    uint64_t *scan = nullptr; // String: n + 1 start offsets (scan + 1 = the end offsets)
    uint8_t *nul = nullptr;   // NULL flags
    uint64_t n = 0, bytes = 0;
    size_t val_cap = 0, scan_cap = 0, nul_cap = 0;
};

// *p holds at least `bytes` (a quarter more when it grows); the old buffer is freed after the
// stream has finished with it
static int grow_buf(Ctx *ctx, void **p, size_t *cap, size_t bytes) {
    bytes = std::max<size_t>(bytes, 16);
    if (*p && *cap >= bytes) return TFG_OK;
    if (*p) {
        TFG_HIP(hipStreamSynchronize(ctx->stream));
        TFG_HIP(hipFree(*p));
        *p = nullptr;
        *cap = 0;
    }
    const size_t nc = bytes + bytes / 4;
    TFG_HIP(hipMalloc(p, nc));
    *cap = nc;
    return TFG_OK;
}

struct tfg_agg {
    Ctx *ctx = nullptr;
    AggSpec S{};
    int key_type = 0;
    bool nokey = false;
    uint32_t B = 1;
    int arg_types[AGG_MAX] = {};
    int arg_nullable[AGG_MAX] = {};
    int result_type[AGG_MAX] = {};
    int result_width[AGG_MAX] = {};
    uint64_t n_groups = 0;
    // double-buffered state
    void *blk[2] = {nullptr, nullptr};
    size_t cap[2] = {0, 0};
    GroupsIO st[2];
    uint64_t *bucket_off[2] = {nullptr, nullptr};
    int cur = 0;
    // A tiled consume (consume_fast_tiled / consume_wide_tiled) leaves its groups where the bucket
    // kernel flushed them: bucket b's pend_cnt[b] groups at pend_base[b] of `pend` (pending).
    // size() and result() read them in place (a consume -> result step never compacts); any other
    // call compacts them into st[] first (pend_compact).
    bool pending = false;
    bool pend_known = false;   // pend_off / pend_total computed
    uint64_t pend_total = 0;
    void *pend_blk = nullptr;
    size_t pend_cap = 0;
    GroupsIO pend{};
    uint64_t *pend_dev = nullptr; // [B] counts, [B] bases, [B + 1] offsets (exclusive scan of the counts),
                                  // [2] the bucket kernels' cursors (kept rows, temp groups)
    uint64_t *pend_ch = nullptr;  // fused String-key result: [B] chars per bucket, [B + 1] their scan
    uint64_t *pend_cnt() const { return pend_dev; }
    uint64_t *pend_base() const { return pend_dev + B; }
    uint64_t *pend_off() const { return pend_dev + 2 * (size_t)B; }
    // after pend_off()[B]: one read-back of two words gives the group count and the kept rows
    unsigned long long *pend_cursor() const { return (unsigned long long *)(pend_dev + 3 * (size_t)B + 1); }
    // groups capacity of the pending buffer for n more rows (allocated once, grown on demand)
    int ensure_pend(size_t groups) {
        if (!pend_dev) TFG_HIP(hipMalloc(&pend_dev, (3 * (size_t)B + 3) * 8));
        if (pend_cap >= groups && pend_blk) return TFG_OK;
        if (pend_blk) {
            TFG_HIP(hipStreamSynchronize(ctx->stream));
            TFG_HIP(hipFree(pend_blk));
            pend_blk = nullptr;
        }
        const size_t nc = std::max<size_t>(groups + groups / 8, 4096);
        TFG_HIP(hipMalloc(&pend_blk, carve_groups(nullptr, nc, pend) + 256));
        pend_cap = nc;
        carve_groups((char *)pend_blk, nc, pend);
        return TFG_OK;
    }
    // row-reference aggregates (ACC_REF: first_row; min / max of Decimal128 / Decimal256 / String):
    // their value stores and the collators of String min / max
    bool has_ref = false;
    int ref_coll[AGG_MAX] = {};
    RefStore store[AGG_MAX], spare[AGG_MAX];
    // per-aggregate row references of a call (consume: the rows' references; merge: the source's,
    // shifted) and the String rebuild's temporaries
    void *ref_rows[AGG_MAX] = {};
    size_t ref_rows_cap[AGG_MAX] = {};
    void *ref_tmp[2] = {};
    size_t ref_tmp_cap[2] = {};
    // wide keys (keys128 / key_string): key_type == TFG_KEYS_WIDE, packing spec, and a device
    // buffer holding the packed keys of the block being consumed / the result being written
    KeyPack kp{};
    int key_types[8] = {};
    int key_collators[8] = {};  // as the packing / dictionary code applies them (NONE for a transformed key)
    int key_transform[8] = {};  // a case-insensitive collator whose sort keys the raw rows are turned into
                                // before a consume (collation.h); 0 = none
    // the serialized method (serial.h): when set, every call goes to `inner`, an aggregator over
    // the dictionary's UInt32 group ids; a packed-key aggregator moves there (carrying its groups)
    // the first time a block's keys do not fit 16 bytes (long String keys, nullable key tuples of
    // 16 bytes).  The creation arguments are kept for that move.
    SerialDict *sdict = nullptr;
    tfg_agg *inner = nullptr;
    bool long_key = false;
    int c_kinds[AGG_MAX] = {}, c_types[AGG_MAX] = {}, c_scales[AGG_MAX] = {};
    tfg_agg_params c_params{};
    // the kept rows of the last tiled consume (pinned, written asynchronously) and its row count
    uint64_t kept_rows = 0; // read with the group count (pend_cursor()[0]); kept_n = 0: unknown
    int64_t kept_n = 0;
    int64_t consumed_n = 0; // rows of the last tiled consume
    void *pack_buf = nullptr;
    size_t pack_cap = 0;
    unsigned *pack_err = nullptr;
    int ensure_pack(size_t rows) {
        if (pack_cap >= rows && pack_buf) return TFG_OK;
        if (pack_buf) {
            TFG_HIP(hipStreamSynchronize(ctx->stream));
            TFG_HIP(hipFree(pack_buf));
            pack_buf = nullptr;
        }
        const size_t nc = std::max<size_t>(rows + rows / 4, 4096);
        TFG_HIP(hipMalloc(&pack_buf, nc * 16));
        pack_cap = nc;
        return TFG_OK;
    }

    size_t group_bytes() const {
        size_t b = (S.key_width == 16 ? 16 : 8) + 1;
        for (int i = 0; i < S.n_aggs; ++i) {
            b += 8 * acc_words(S.acc[i]);
            if (S.has_cnt[i]) b += 8;
        }
        return b;
    }
    // carve a GroupsIO of `n` groups out of `base` (returns bytes used)
    size_t carve_groups(char *base, size_t n, GroupsIO &g) const {
        Carver cv;
        size_t ok = cv.take<uint64_t>(S.key_width == 16 ? 2 * n : n), on = cv.take<uint8_t>(n);
        size_t oa[AGG_MAX] = {}, oc[AGG_MAX] = {};
        for (int i = 0; i < S.n_aggs; ++i) {
            if (S.acc[i] == ACC_I256) oa[i] = cv.take<uint4>(2 * n);
            else if (S.acc[i] == ACC_I128) oa[i] = cv.take<uint4>(n);
            else if (S.acc[i] != ACC_NONE) oa[i] = cv.take<uint64_t>(n);
            if (S.has_cnt[i]) oc[i] = cv.take<uint64_t>(n);
        }
        if (base) {
            g.key = (uint64_t *)(base + ok);
            g.key_null = (uint8_t *)(base + on);
            for (int i = 0; i < AGG_MAX; ++i) {
                g.acc[i] = (i < S.n_aggs && S.acc[i] != ACC_NONE) ? base + oa[i] : nullptr;
                g.cnt[i] = (i < S.n_aggs && S.has_cnt[i]) ? (uint64_t *)(base + oc[i]) : nullptr;
            }
        }
        return cv.off;
    }
    int ensure_state(int idx, size_t n) {
        if (cap[idx] >= n && blk[idx]) return TFG_OK;
        size_t nc = std::max<size_t>(n + n / 2, 1024);
        size_t bytes = carve_groups(nullptr, nc, st[idx]);
        if (blk[idx]) {
            TFG_HIP(hipStreamSynchronize(ctx->stream));
            TFG_HIP(hipFree(blk[idx]));
            blk[idx] = nullptr;
        }
        TFG_HIP(hipMalloc(&blk[idx], bytes));
        cap[idx] = nc;
        carve_groups((char *)blk[idx], nc, st[idx]);
        return TFG_OK;
    }
};

namespace {

// op-code signature for the FastOps specialisations (0 = generic path)
int fast_signature(const AggSpec &S, int mode, int key_width, const uint8_t *key_null, const uint8_t *const *val_nulls) {
    if (mode != MODE_RAW || key_width != 8 || key_null || S.n_aggs > 3) return 0;
    int code = 0;
    for (int i = 0; i < 3; ++i) {
        int op = 0;
        if (i < S.n_aggs) {
            if (val_nulls && val_nulls[i]) return 0;
            const int k = S.kind[i], t = S.src_type[i];
            if (k == TFG_AGG_COUNT_ALL || k == TFG_AGG_COUNT) op = 1;
            else if (S.acc[i] == ACC_I64 && (t == TFG_INT64 || t == TFG_UINT64)) op = 2;
            else if (S.acc[i] == ACC_F64 && t == TFG_FLOAT64) op = 3;
            else if (S.acc[i] == ACC_I128 && t == TFG_DECIMAL64) op = 4;
            else return 0;
            if (S.has_cnt[i] && op != 1) return 0;
        }
        code = code * 10 + op;
    }
    return fast_code_supported(code) ? code : 0; // e.g. count() before sum(): the generic path
}

// ---- the pending state of a tiled consume (tfg_agg::pending)
// groups per bucket -> their output offsets and the total (one host read, cached)
int pend_scan(tfg_agg *a) { // the output offsets on the device (no host read)
    Ctx *ctx = a->ctx;
    void *sp;
    if (int rc = scratch_get(ctx, scan_tmp_bytes(a->B + 1), &sp)) return rc;
    return exclusive_scan_u64(ctx, a->pend_cnt(), a->pend_off(), a->B, sp);
}
// the group count (pend_off()[B]) and, beside it, the kept rows of the tiled consume (the bucket
// kernels' first cursor) in one read-back
int pend_read_total(tfg_agg *a) {
    uint64_t w[2];
    if (int rc = read_back_u64(a->ctx, a->pend_off() + a->B, w, 2)) return rc;
    a->pend_total = w[0];
    a->kept_rows = w[1];
    a->kept_n = a->consumed_n;
    a->pend_known = true;
    return TFG_OK;
}
int pend_counts(tfg_agg *a) {
    if (!a->pending || a->pend_known) return TFG_OK;
    if (int rc = pend_scan(a)) return rc;
    return pend_read_total(a);
}
// pending groups -> the dense bucket-major state st[] (the compaction every other call expects)
int pend_compact(tfg_agg *a) {
    if (!a->pending) return TFG_OK;
    if (int rc = pend_counts(a)) return rc;
    Ctx *ctx = a->ctx;
    const uint32_t B = a->B;
    const int nxt = a->cur ^ 1;
    if (int rc = a->ensure_state(nxt, a->pend_total)) return rc;
    if (!a->bucket_off[nxt]) TFG_HIP(hipMalloc(&a->bucket_off[nxt], (B + 1) * 8));
    {
        ProfScope _ps(ctx, "agg.compact");
        hipLaunchKernelGGL(agg_compact_kernel, dim3(B), dim3(256), 0, ctx->stream, a->S, a->pend,
                           (const uint64_t *)nullptr, (const uint64_t *)nullptr, (const uint64_t *)a->pend_off(),
                           a->st[nxt], (const uint64_t *)a->pend_base());
    }
    TFG_LAUNCH_CHECK();
    TFG_HIP(hipMemcpyAsync(a->bucket_off[nxt], a->pend_off(), (B + 1) * 8, hipMemcpyDeviceToDevice, ctx->stream));
    a->cur = nxt;
    a->n_groups = a->pend_total;
    a->pending = false;
    return TFG_OK;
}

// The fast signatures run over a tile-sorted partition: partition -> agg_bucket_tiled_kernel,
// whose groups stay pending (result() reads them in place; other calls compact them first);
// the histogram + scatter partition serves the other signatures.

int consume_fast_tiled(tfg_agg *a, int fast, const RowPred &pred, const void *keys, const void *const *vals,
                       int64_t n, bool &done) {
    done = false;
    Ctx *ctx = a->ctx;
    const AggSpec &S = a->S;
    const uint32_t B = a->B;
    const size_t n_old = a->n_groups;
    int rec_words = 1;
    for (int c = fast; c > 0; c /= 10) rec_words += (c % 10) >= 2;
    PCols pc{};
    pc.in[0] = keys;
    pc.width[0] = 8;
    pc.ncols = 1;
    pc.key0 = 1;
    pc.aos = 1;
    for (int i = 0, c = fast; i < S.n_aggs; ++i) {
        const int op = (i == 0 ? c / 100 : i == 1 ? c / 10 : c) % 10;
        if (op < 2) continue;
        pc.in[pc.ncols] = vals[i];
        pc.width[pc.ncols++] = 8;
    }
    TFG_CHECK(pc.ncols == rec_words, TFG_ERR_LOGICAL, "record layout mismatch");
    TiledGeom tg{};
    if (!make_tiled_geom(ctx, n, B, pc, tg)) return TFG_OK; // not applicable: caller takes the general path
    Carver cv;
    const size_t o_rec = cv.take<uint64_t>((size_t)tg.out_rows * rec_words);
    const size_t o_sp0 = cv.take<uint64_t>((size_t)n * rec_words), o_sp1 = cv.take<uint64_t>((size_t)n * rec_words);
    const size_t o_hist = cv.take<uint32_t>((size_t)B * tg.sg.T);
    const size_t o_flags = cv.take<uint8_t>((size_t)tg.sg.T); // the sparse variant's tile flags
    if (int rc = a->ensure_pend(n_old + (size_t)n)) return rc; // the groups stay there (pending)
    void *sp;
    if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
    char *sb = (char *)sp;
    pc.out[0] = sb + o_rec;
    SelBucket8 sel{(const uint64_t *)keys, fib_shift(B)};
    // the previous consume kept fewer rows than this one has tiles (e.g. a filter that keeps
    // nothing): the partition checks all-false tiles with vector loads.  kept_rows was read with
    // the previous consume's group count: a heuristic, a stale value only picks the other
    // (equally exact) kernel
    const bool sparse = a->kept_n > 0 && a->kept_rows * (uint64_t)tg.sg.TR < (uint64_t)a->kept_n;
    tg.sg.zero2 = a->pend_cursor(); // the bucket kernel's cursors, zeroed by the partition
    if (int rc = run_partition_tiled(ctx, sel, pred, tg, pc, (uint32_t *)(sb + o_hist), "agg.part.tiled", sparse,
                                     (uint8_t *)(sb + o_flags)))
        return rc;
    TiledIn tin{};
    tin.rec = (const uint64_t *)(sb + o_rec);
    tin.tile_hist = (const uint32_t *)(sb + o_hist);
    tin.T = tg.sg.T;
    tin.TR = tg.sg.TRS; // tile slot stride
    tin.spill[0] = (uint64_t *)(sb + o_sp0);
    tin.spill[1] = (uint64_t *)(sb + o_sp1);
    tin.cursor = a->pend_cursor();
    tin.xcd_remap = 1; // neighbouring runs read by one XCD: FETCH 1.95 -> 1.2 GB per C2 step (r03b)
    const bool has_old = n_old > 0;
    const GroupsIO old = a->st[a->cur];
    const uint64_t *ooff = has_old ? a->bucket_off[a->cur] : (const uint64_t *)nullptr;
    {
        ProfScope _ps(ctx, "agg.bucket");
        if (!launch_bucket_fast_tiled(fast, B, S, ctx->stream, tin, MODE_RAW, old, ooff, a->pend, a->pend_cnt(),
                                      a->pend_base()))
            return TFG_OK; // not reached: fast_signature returns the specialised codes only
    }
    TFG_LAUNCH_CHECK();
    // this consume's kept rows (the bucket kernels' cursor) are read with the group count, for the
    // next consume's all-false tile choice (no read-back of their own)
    a->consumed_n = n;
    a->kept_n = 0;
    a->pending = true; // groups stay bucket-strided in a->pend until a call needs them dense
    a->pend_known = false;
    done = true;
    return TFG_OK;
}

int consume_keyed(tfg_agg *a, int mode, const RowPred &pred, const void *keys, int key_width, const uint8_t *key_null,
                  const void *const *vals, const uint8_t *const *val_nulls, const uint64_t *const *val_cnts,
                  const uint64_t *given_off, int64_t n);

// op-code signature of the wide tiled path: the FastOps codes with at most one summed argument
// (records of 2-3 words: key lo, key hi, value), raw rows without NULL values
int wide_fast_signature(const AggSpec &S, const uint8_t *const *val_nulls) {
    if (S.key_width != 16 || S.n_aggs > 3) return 0;
    int code = 0, sums = 0;
    for (int i = 0; i < 3; ++i) {
        int op = 0;
        if (i < S.n_aggs) {
            if (val_nulls && val_nulls[i]) return 0;
            const int k = S.kind[i], t = S.src_type[i];
            if (k == TFG_AGG_COUNT_ALL || k == TFG_AGG_COUNT) op = 1;
            else if (S.acc[i] == ACC_I64 && (t == TFG_INT64 || t == TFG_UINT64)) op = 2;
            else if (S.acc[i] == ACC_F64 && t == TFG_FLOAT64) op = 3;
            else if (S.acc[i] == ACC_I128 && t == TFG_DECIMAL64) op = 4;
            else return 0;
            if (S.has_cnt[i] && op != 1) return 0;
            sums += op >= 2;
        }
        code = code * 10 + op;
    }
    switch (sums <= 1 ? code : 0) { // the WideFastOps specialisations (launch_bucket_wide_tiled)
    case 410: case 310: case 210: case 140: case 130: case 120: case 400: case 300: case 200: case 100: return code;
    default: return 0;
    }
}

// Wide keys (packed keys128 / key_string) of a wide fast signature over a tiled partition:
// one level (B <= 256 buckets) as consume_fast_tiled, or two levels (coarse = B / 64 buckets in
// pass 1, regroup_tiled_kernel into 64 fine buckets each); then the tiled bucket kernel with
// WideFastOps, scan and compaction.  `sel` produces the 16-byte keys (SelWide2 over packed keys,
// SelWideStr straight from the String column).  done = false: not applicable (general path).
// narrow 20-byte wide-key tiles (partition.h WNARROW): TFG_WIDE_NARROW=0 none, 1 pass-1 tiles
// only (the regroup writes 24-byte tiles), 2 pass-1 and regrouped tiles (A/B knob)
static int wide_narrow_mode() {
    static const int m = [] {
        const char *v = getenv("TFG_WIDE_NARROW");
        return v && *v ? atoi(v) : 2;
    }();
    return m;
}

template <typename Sel>
int consume_wide_tiled(tfg_agg *a, int code, Sel sel, const void *const *vals, int64_t n, unsigned *err, bool &done) {
    done = false;
    if (int rc = pend_compact(a)) return rc;
    Ctx *ctx = a->ctx;
    const AggSpec &S = a->S;
    const uint32_t B = a->B;
    const size_t n_old = a->n_groups;
    if (n <= 0 || n >= (int64_t)0xFFFFFFFFll) return TFG_OK;
    int ncol = 2;
    PCols pc{};
    pc.ncols = 2;
    pc.width[0] = pc.width[1] = 8;
    pc.key0 = 1;
    pc.aos = 1;
    for (int i = 0, c = code; i < S.n_aggs; ++i) {
        const int op = (i == 0 ? c / 100 : i == 1 ? c / 10 : c) % 10;
        if (op < 2) continue;
        pc.in[pc.ncols] = vals[i];
        pc.width[pc.ncols++] = 8;
        ++ncol;
    }
    const uint32_t bbits = fib_shift(1) - fib_shift(B); // log2(B)
    const bool two = bbits > 8;
    const uint32_t B1 = two ? B >> RG_FINE_BITS : B;
    TiledGeom tg{};
    if (!make_tiled_geom(ctx, n, B1, pc, tg)) return TFG_OK;
    const int T1 = tg.sg.T;
    const int64_t T2 = two ? (n + RG_TR - 1) / RG_TR + B1 : 0;
    Carver cv;
    const size_t o_rec1 = cv.take<uint64_t>((size_t)tg.out_rows * ncol);
    const size_t o_rec2 = cv.take<uint64_t>(two ? (size_t)T2 * RG_TR * ncol : 0);
    const size_t o_sp1 = cv.take<uint64_t>((size_t)n * ncol); // spill arena 0 = pass-1 records (two levels)
    const size_t o_sp0 = cv.take<uint64_t>(two ? 0 : (size_t)n * ncol);
    const size_t o_hist1 = cv.take<uint32_t>((size_t)B1 * T1);
    const size_t o_pref = cv.take<uint32_t>(two ? (size_t)B1 * (T1 + 1) : 0);
    const size_t o_tbase = cv.take<uint32_t>(B1 + 1);
    const size_t o_hist2 = cv.take<uint32_t>(two ? (size_t)RG_FINE * T2 : 0);
    const size_t o_desc = cv.take<RgDesc>(two ? (size_t)T2 : 0);
    if (int rc = a->ensure_pend(n_old + (size_t)n)) return rc; // the groups stay there (pending)
    void *sp;
    if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
    char *sb = (char *)sp;
    pc.out[0] = sb + o_rec1;
    sel.shift = fib_shift(B1);
    if (err) TFG_HIP(hipMemsetAsync(err, 0, sizeof(unsigned), ctx->stream));
    tg.sg.zero2 = a->pend_cursor(); // the bucket kernel's cursors, zeroed by the partition
    tg.sg.allow_narrow = wide_narrow_mode() >= 1;
    if (int rc = run_partition_tiled(ctx, sel, RowPred{}, tg, pc, (uint32_t *)(sb + o_hist1), "agg.part.tiled"))
        return rc;
    if (err) { // a String key longer than 15 bytes: the serialized method, not this one
        uint64_t e = 0;
        if (int rc = read_back_u64(ctx, (const uint64_t *)err, &e, 1)) return rc; // pinned: no staging copy
        if ((unsigned)e) {
            a->long_key = true;
            return fail(TFG_ERR_NOT_IMPLEMENTED, "String GROUP BY key longer than 15 bytes (serialized method)");
        }
    }
    TiledIn tin{};
    tin.rec = (const uint64_t *)(sb + o_rec1);
    tin.tile_hist = (const uint32_t *)(sb + o_hist1);
    tin.T = T1;
    tin.TR = tg.sg.TRS; // tile slot stride
    tin.spill[0] = (uint64_t *)(sb + (two ? o_rec1 : o_sp0));
    tin.spill[1] = (uint64_t *)(sb + o_sp1);
    if (two) {
        uint32_t *pref = (uint32_t *)(sb + o_pref), *tbase = (uint32_t *)(sb + o_tbase);
        uint32_t *hist2 = (uint32_t *)(sb + o_hist2);
        ProfScope _ps(ctx, "agg.part.regroup");
        hipLaunchKernelGGL(regroup_prefix_kernel, dim3(B1), dim3(1024), 0, ctx->stream, tin.tile_hist, T1, pref);
        hipLaunchKernelGGL(regroup_tile_base_kernel, dim3(1), dim3(1024), 0, ctx->stream, pref, T1, (int)B1, tbase);
        RgDesc *desc = (RgDesc *)(sb + o_desc);
        hipLaunchKernelGGL(regroup_desc_kernel, dim3((unsigned)((T2 + 255) / 256)), dim3(256), 0, ctx->stream,
                           (const uint32_t *)pref, T1, (const uint32_t *)tbase, (int)B1, (int)T2, desc);
        const uint32_t fine_shift = fib_shift(B);
        if (ncol == 3)
            hipLaunchKernelGGL(regroup_tiled_kernel<3>, dim3((unsigned)T2), dim3(RG_T), 0, ctx->stream, tin.rec,
                               tin.tile_hist, T1, tin.TR, pref, (const RgDesc *)desc, fine_shift,
                               (uint64_t *)(sb + o_rec2), hist2, (int)T2, wide_narrow_mode() >= 2);
        else
            hipLaunchKernelGGL(regroup_tiled_kernel<2>, dim3((unsigned)T2), dim3(RG_T), 0, ctx->stream, tin.rec,
                               tin.tile_hist, T1, tin.TR, pref, (const RgDesc *)desc, fine_shift,
                               (uint64_t *)(sb + o_rec2), hist2, (int)T2, wide_narrow_mode() >= 2);
        TFG_LAUNCH_CHECK();
        tin.rec = (const uint64_t *)(sb + o_rec2);
        tin.tile_hist = hist2;
        tin.T = (int)T2;
        tin.TR = RG_TR;
        tin.tile_base = tbase;
        tin.fine_bits = RG_FINE_BITS;
    }
    tin.cursor = a->pend_cursor();
    tin.xcd_remap = 0; // two-level wide tiles: measured slower with the remap (r03b)
    const bool has_old = n_old > 0;
    const GroupsIO old = a->st[a->cur];
    const uint64_t *ooff = has_old ? a->bucket_off[a->cur] : (const uint64_t *)nullptr;
    {
        ProfScope _ps(ctx, "agg.bucket");
        if (!launch_bucket_wide_tiled(code, B, S, ctx->stream, tin, MODE_RAW, old, ooff, a->pend, a->pend_cnt(),
                                      a->pend_base()))
            return TFG_OK; // other signatures: the general path (nothing enqueued that matters)
    }
    TFG_LAUNCH_CHECK();
    // this consume's kept rows (the bucket kernels' cursor) are read with the group count, for the
    // next consume's all-false tile choice (no read-back of their own)
    a->consumed_n = n;
    a->kept_n = 0;
    a->pending = true; // groups stay bucket-strided in a->pend until a call needs them dense
    a->pend_known = false;
    done = true;
    return TFG_OK;
}

int consume_keyed(tfg_agg *a, int mode, const RowPred &pred, const void *keys, int key_width, const uint8_t *key_null,
                  const void *const *vals, const uint8_t *const *val_nulls, const uint64_t *const *val_cnts,
                  const uint64_t *given_off, int64_t n) {
    Ctx *ctx = a->ctx;
    const AggSpec &S = a->S;
    const uint32_t B = a->B;
    const size_t n_old = a->n_groups;
    // fast signature: rows staged as interleaved records (key + summed arguments, 8 B each)
    const int fast = given_off ? 0 : fast_signature(S, mode, key_width, key_null, val_nulls);
    if (fast) {
        bool done = false;
        if (int rc = consume_fast_tiled(a, fast, pred, keys, vals, n, done)) return rc;
        if (done) return TFG_OK;
    }
    int rec_words = 1;
    for (int c = fast; c > 0; c /= 10) rec_words += (c % 10) >= 2;
    // ---- scratch layout
    Carver cv;
    const size_t o_key = cv.take<uint64_t>(n * (fast ? rec_words : key_width == 16 ? 2 : 1)), o_knull = cv.take<uint8_t>(n);
    size_t o_val[AGG_MAX] = {}, o_vnull[AGG_MAX] = {}, o_vcnt[AGG_MAX] = {};
    int vw[AGG_MAX] = {};
    for (int i = 0; i < S.n_aggs && !fast; ++i) {
        if (val_nulls && val_nulls[i]) o_vnull[i] = cv.take<uint8_t>(n);
        if (val_cnts && val_cnts[i]) o_vcnt[i] = cv.take<uint64_t>(n);
        if (!vals[i]) continue;
        if (S.acc[i] == ACC_REF) vw[i] = 8; // candidate references
        else if (mode == MODE_RAW || (mode == MODE_PARTIAL && S.acc[i] == ACC_ORD)) vw[i] = (int)type_width(S.src_type[i]);
        else vw[i] = 8 * std::max(1, acc_words(S.acc[i]));
        o_val[i] = cv.take<uint4>((n * vw[i] + 15) / 16);
    }
    const size_t staging_bytes = cv.off; // key/value columns above; a second copy holds spills
    const size_t o_spill = cv.take<uint8_t>(staging_bytes);
    const size_t o_stage_off = cv.take<uint64_t>(B + 1);
    const size_t o_new_cnt = cv.take<uint64_t>(B), o_new_off = cv.take<uint64_t>(B + 1);
    const size_t tmp_groups = n_old + (size_t)n;
    const size_t o_tmpg = cv.take<uint8_t>(a->carve_groups(nullptr, tmp_groups, a->st[0]) + 256);
    PartLayout L = make_layout(n, B);
    const size_t o_part =
        cv.take<uint8_t>(std::max(part_tmp_bytes(L, fast ? (size_t)rec_words * 8 : 0, false), scan_tmp_bytes(B + 1)));
    void *sp;
    if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
    char *sb = (char *)sp;
    // ---- stage rows (bucket-major)
    RowsIO rows{};
    rows.key_width = key_width;
    rows.key = sb + o_key;
    rows.key_null = key_null ? (uint8_t *)(sb + o_knull) : nullptr;
    uint64_t *stage_off = (uint64_t *)(sb + o_stage_off);
    if (given_off) {
        // rows already bucket-major (merge of a state with the same bucket function): copy
        TFG_HIP(hipMemcpyAsync(rows.key, keys, n * key_width, hipMemcpyDeviceToDevice, ctx->stream));
        if (key_null) TFG_HIP(hipMemcpyAsync(rows.key_null, key_null, n, hipMemcpyDeviceToDevice, ctx->stream));
        for (int i = 0; i < S.n_aggs; ++i) {
            if (vals[i]) {
                rows.val[i] = sb + o_val[i];
                TFG_HIP(hipMemcpyAsync(rows.val[i], vals[i], n * vw[i], hipMemcpyDeviceToDevice, ctx->stream));
            }
            if (val_cnts && val_cnts[i]) {
                rows.val_cnt[i] = (uint64_t *)(sb + o_vcnt[i]);
                TFG_HIP(hipMemcpyAsync(rows.val_cnt[i], val_cnts[i], n * 8, hipMemcpyDeviceToDevice, ctx->stream));
            }
        }
        TFG_HIP(hipMemcpyAsync(stage_off, given_off, (B + 1) * 8, hipMemcpyDeviceToDevice, ctx->stream));
    } else if (fast) {
        PCols pc{};
        pc.in[0] = keys;
        pc.out[0] = rows.key;
        pc.width[0] = 8;
        pc.ncols = 1;
        pc.key0 = 1;
        pc.aos = 1;
        pc.two_pass = 1;
        for (int i = 0, c = fast; i < S.n_aggs; ++i) {
            const int op = (i == 0 ? c / 100 : i == 1 ? c / 10 : c) % 10;
            if (op < 2) continue;
            pc.in[pc.ncols] = vals[i];
            pc.width[pc.ncols++] = 8;
        }
        TFG_CHECK(pc.ncols == rec_words, TFG_ERR_LOGICAL, "record layout mismatch");
        pc.aos = rec_words >= 2; // keys alone (count() only): one plain column
        SelBucket8 sel{(const uint64_t *)keys, fib_shift(B)};
        if (int rc = run_partition<SelBucket8, false>(ctx, sel, pred, L, pc, nullptr, nullptr, stage_off, sb + o_part,
                                                      "agg.part.hist", "agg.part.scatter"))
            return rc;
    } else {
        PCols pc{};
        pc.in[pc.ncols] = keys;
        pc.out[pc.ncols] = rows.key;
        pc.width[pc.ncols++] = key_width;
        pc.key0 = key_width == 8;
        if (key_null) {
            pc.in[pc.ncols] = key_null;
            pc.out[pc.ncols] = rows.key_null;
            pc.width[pc.ncols++] = 1;
        }
        for (int i = 0; i < S.n_aggs; ++i) {
            if (vals[i]) {
                rows.val[i] = sb + o_val[i];
                pc.in[pc.ncols] = vals[i];
                pc.out[pc.ncols] = rows.val[i];
                pc.width[pc.ncols++] = vw[i];
            }
            if (val_nulls && val_nulls[i]) {
                rows.val_null[i] = (uint8_t *)(sb + o_vnull[i]);
                pc.in[pc.ncols] = val_nulls[i];
                pc.out[pc.ncols] = rows.val_null[i];
                pc.width[pc.ncols++] = 1;
            }
        }
        TFG_CHECK(pc.ncols <= PCOLS, TFG_ERR_NOT_IMPLEMENTED, "too many aggregate columns");
        if (key_width == 16) {
            SelWide sel{(const uint4 *)keys, fib_shift(B)};
            if (int rc = run_partition<SelWide, false>(ctx, sel, pred, L, pc, nullptr, nullptr, stage_off, sb + o_part,
                                                        "agg.part.hist", "agg.part.scatter"))
                return rc;
        } else {
            SelBucket sel{keys, key_null, key_width, fib_shift(B)};
            if (int rc = run_partition<SelBucket, false>(ctx, sel, pred, L, pc, nullptr, nullptr, stage_off,
                                                          sb + o_part, "agg.part.hist", "agg.part.scatter"))
                return rc;
        }
    }
    // ---- bucket kernel
    GroupsIO tmp{};
    a->carve_groups(sb + o_tmpg, tmp_groups, tmp);
    uint64_t *new_cnt = (uint64_t *)(sb + o_new_cnt), *new_off = (uint64_t *)(sb + o_new_off);
    const bool has_old = n_old > 0;
    GroupsIO old = a->st[a->cur];
    RowsIO rows1 = rows; // same layout, shifted into the spill copy
    auto shift = [&](auto *p) { return p ? (decltype(p))((char *)p + o_spill) : p; };
    rows1.key = shift(rows.key);
    rows1.key_null = shift(rows.key_null);
    for (int i = 0; i < AGG_MAX; ++i) {
        rows1.val[i] = shift(rows.val[i]);
        rows1.val_null[i] = shift(rows.val_null[i]);
        rows1.val_cnt[i] = shift(rows.val_cnt[i]);
    }
    const uint64_t *ooff = has_old ? a->bucket_off[a->cur] : (const uint64_t *)nullptr;
    {
        ProfScope _ps(ctx, "agg.bucket");
        if (!launch_bucket_fast(fast, B, S, ctx->stream, rows, rows1, mode, stage_off, old, ooff, tmp, new_cnt)) {
            bool w256 = false; // a Decimal256 sum: rows carry 4-limb values
            for (int i = 0; i < S.n_aggs; ++i) w256 = w256 || S.acc[i] == ACC_I256;
#ifdef TFG_EXP_POOL
            if (getenv("TFG_POOLDBG"))
                for (int i = 0; i < S.n_aggs; ++i)
                    if (S.acc[i] == ACC_REF)
                        fprintf(stderr, "POOL launch agg %p ref[%d] v %p %p o %p %p n0 %llu n1 %llu nb %llu %llu\n",
                                (void *)a, i, (const void *)S.ref[i].v[0], (const void *)S.ref[i].v[1],
                                (const void *)S.ref[i].o[0], (const void *)S.ref[i].o[1],
                                (unsigned long long)S.ref[i].n0, (unsigned long long)S.ref[i].n1,
                                (unsigned long long)S.ref[i].nb[0], (unsigned long long)S.ref[i].nb[1]);
#endif
            launch_bucket_generic(key_width == 16, w256, B, S, ctx->stream, rows, rows1, mode, stage_off, old, ooff, tmp,
                                  new_cnt);
        }
    }
    TFG_LAUNCH_CHECK();
    if (int rc = exclusive_scan_u64(ctx, new_cnt, new_off, B, sb + o_part)) return rc;
    uint64_t total = 0;
    if (int rc = read_back_u64(ctx, new_off + B, &total, 1)) return rc;
    const int nxt = a->cur ^ 1;
    if (int rc = a->ensure_state(nxt, total)) return rc;
    if (!a->bucket_off[nxt]) TFG_HIP(hipMalloc(&a->bucket_off[nxt], (B + 1) * 8));
    { ProfScope _ps(ctx, "agg.compact");
    hipLaunchKernelGGL(agg_compact_kernel, dim3(B), dim3(256), 0, ctx->stream, S, tmp, stage_off,
                       has_old ? a->bucket_off[a->cur] : (const uint64_t *)nullptr, new_off, a->st[nxt],
                       (const uint64_t *)nullptr);
    }
    TFG_LAUNCH_CHECK();
    TFG_HIP(hipMemcpyAsync(a->bucket_off[nxt], new_off, (B + 1) * 8, hipMemcpyDeviceToDevice, ctx->stream));
    a->cur = nxt;
    a->n_groups = total;
    return TFG_OK;
}

int consume_nokey(tfg_agg *a, int mode, const RowPred &pred, const void *const *vals, const uint8_t *const *val_nulls,
                  int64_t n) {
    Ctx *ctx = a->ctx;
    RowsIO rows{};
    for (int i = 0; i < a->S.n_aggs; ++i) {
        rows.val[i] = (void *)vals[i];
        rows.val_null[i] = val_nulls ? (uint8_t *)val_nulls[i] : nullptr;
    }
    const unsigned grid = stream_grid(n, NK_T * 16, 1024);
    void *sp;
    if (int rc = scratch_get(ctx, grid * sizeof(NoKeyPartial), &sp)) return rc;
    { ProfScope _ps(ctx, "agg.nokey");
    hipLaunchKernelGGL(agg_nokey_kernel, dim3(grid), dim3(NK_T), 0, ctx->stream, a->S, rows, mode, pred, n,
                       (NoKeyPartial *)sp);
    }
    hipLaunchKernelGGL(agg_nokey_fold_kernel, dim3(1), dim3(64), 0, ctx->stream, a->S, (const NoKeyPartial *)sp,
                       (int)grid, a->st[a->cur]);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

// sum state of an argument type word (tfg_type | TFG_ARG_PREC(p)): Float64, Int64 / UInt64, or the
// Decimal result of SumDecimalInferer (Common/Decimal.h:156-163), Decimal(min(p + 22, 65), s):
// Decimal128 up to 38 digits, Decimal256 above (AggregateFunctionSum.cpp:57-85)
int sum_acc_kind(int word) {
    const int t = TFG_ARG_TYPE(word);
    if (t == TFG_FLOAT32 || t == TFG_FLOAT64) return ACC_F64;
    if (is_decimal_type(t) || t == TFG_DECIMAL256) {
        int p = TFG_ARG_PREC_OF(word);
        if (p == 0) p = t == TFG_DECIMAL32 ? 9 : t == TFG_DECIMAL64 ? 18 : t == TFG_DECIMAL128 ? 38 : 65;
        return std::min(p + 22, 65) > 38 ? ACC_I256 : ACC_I128;
    }
    return ACC_I64;
}

// A Decimal256 sum that left Int256 during the last call (the device flag S.ovf): the reference's
// checked_int256_t throws (libs/libcommon/include/common/types.h:35) -> TFG_ERR_OVERFLOW
int check_overflow(tfg_agg *a) {
    if (!a->S.ovf) return TFG_OK;
    unsigned f = 0;
    TFG_HIP(hipMemcpyAsync(&f, a->S.ovf, sizeof f, hipMemcpyDeviceToHost, a->ctx->stream));
    TFG_HIP(hipStreamSynchronize(a->ctx->stream));
    if (!f) return TFG_OK;
    TFG_HIP(hipMemsetAsync(a->S.ovf, 0, sizeof f, a->ctx->stream));
    if (f & 2) // RefSrc::err: a row reference outside its candidates (never dereferenced)
        return fail(TFG_ERR_LOGICAL, "row-reference aggregate state out of range (internal error)");
    if (f & 4) // RefSrc::err: a candidate's String bytes past its buffer (never dereferenced)
        return fail(TFG_ERR_LOGICAL, "row-reference String candidate past its buffer (internal error)");
    return fail(TFG_ERR_OVERFLOW, "Decimal256 sum overflow (DECIMAL_OVERFLOW: the sum left Int256)");
}

// ---- row-reference aggregates (ACC_REF, agg_dev.h): candidates, reference columns, store rebuild
struct RefIn { // source 1 of an ACC_REF aggregate's candidates: the consumed column (or a merge's source store)
    const uint8_t *val = nullptr; // fixed-width values, or String chars
    const uint64_t *off = nullptr; // String: end offsets
    const uint8_t *nul = nullptr;
    uint64_t n = 0;
    uint64_t bytes = ~0ull; // String chars bytes when known (a merge's source store)
};
struct RefCall { // the collated candidates of one call (String min / max under a case-insensitive collator)
    tfg_agg *a;
    CollatedStrings cs[AGG_MAX][2];
    explicit RefCall(tfg_agg *agg) : a(agg) {}
    // the candidates named in S.ref die with the call: no later launch may carry their pointers
    ~RefCall() {
#ifdef TFG_EXP_POOL // the fault analysis: TFG_REF_NOCLEAR=1 keeps round 5's dangling pointers
        static const bool keep = getenv("TFG_REF_NOCLEAR") && *getenv("TFG_REF_NOCLEAR") == '1';
        if (keep) return;
#endif
        for (auto &r : a->S.ref) r = RefSrc{};
    }
    RefCall(const RefCall &) = delete;
    RefCall &operator=(const RefCall &) = delete;
};

// the stream is synchronized before (the buffers' last users may still run)
void ref_store_free(RefStore &st) {
    if (st.val) (void)hipFree(st.val);
    if (st.scan) (void)hipFree(st.scan);
    if (st.nul) (void)hipFree(st.nul);
    st = RefStore{};
}

// S.ref[i] of every ACC_REF aggregate for one call: its store, then `in`.  String min / max under a
// case-insensitive collator compare sort keys of the whole rows ('\0' included, no trim)
int ref_setup(tfg_agg *a, const RefIn *in, RefCall &rc) {
    for (int i = 0; i < a->S.n_aggs; ++i) {
        if (a->S.acc[i] != ACC_REF) continue;
        RefSrc &R = a->S.ref[i];
        R = RefSrc{};
        const RefStore &st = a->store[i];
        R.n0 = st.n;
        R.n1 = in[i].n;
        R.err = a->S.ovf;
        const int t = a->S.src_type[i];
        R.v[0] = st.val;
        R.v[1] = in[i].val;
        R.nb[0] = st.bytes;
        R.nb[1] = in[i].bytes; // a consumed column's chars: size not passed (~0)
        if (t != TFG_STRING) {
            R.width = (int)type_width(t);
            continue;
        }
        R.o[0] = st.scan ? st.scan + 1 : nullptr;
        R.o[1] = in[i].off;
        const int coll = a->ref_coll[i];
        if (a->S.kind[i] == TFG_AGG_FIRST_ROW || !collator_transforms(coll)) continue;
        if (int r = collate_strings(a->ctx, coll, st.val, R.o[0], nullptr, nullptr, nullptr, (int64_t)st.n, rc.cs[i][0], true))
            return r;
        if (int r = collate_strings(a->ctx, coll, in[i].val, in[i].off, in[i].nul, nullptr, nullptr, (int64_t)in[i].n,
                                    rc.cs[i][1], true))
            return r;
        R.v[0] = rc.cs[i][0].chars;
        R.o[0] = rc.cs[i][0].offsets();
        R.nb[0] = rc.cs[i][0].bytes;
        R.v[1] = rc.cs[i][1].chars;
        R.o[1] = rc.cs[i][1].offsets();
        R.nb[1] = rc.cs[i][1].bytes;
    }
    return TFG_OK;
}

// after a call: each group's winning candidate copied into a new store in group order, the group's
// reference set to g + 1 (0 stays: no value)
int ref_rebuild(tfg_agg *a, const RefIn *in) {
    Ctx *ctx = a->ctx;
    const uint64_t G = a->n_groups;
    const GroupsIO &st = a->st[a->cur];
    const unsigned grid = stream_grid((int64_t)std::max<uint64_t>(G, 1), 256, 4096);
    for (int i = 0; i < a->S.n_aggs; ++i) {
        if (a->S.acc[i] != ACC_REF) continue;
        RefStore &old = a->store[i];
        RefStore &nw = a->spare[i]; // its buffers: free since the previous rebuild
        const RefCol s0{old.val, old.scan ? old.scan + 1 : nullptr, old.nul}, s1{in[i].val, in[i].off, in[i].nul};
        uint64_t *acc = (uint64_t *)st.acc[i];
        if (int rc = grow_buf(ctx, (void **)&nw.nul, &nw.nul_cap, G)) return rc;
        const int t = a->S.src_type[i];
        uint64_t total = 0;
        if (t != TFG_STRING) {
            const int w = (int)type_width(t);
            if (int rc = grow_buf(ctx, (void **)&nw.val, &nw.val_cap, G * w)) return rc;
            if (G) {
                ProfScope _ps(ctx, "agg.ref_store");
                hipLaunchKernelGGL(ref_store_fixed_kernel, dim3(grid), dim3(256), 0, ctx->stream, acc, G, old.n, in[i].n,
                                   a->S.ovf, w, s0, s1, nw.val, nw.nul);
                TFG_LAUNCH_CHECK();
            }
        } else {
            if (int rc = grow_buf(ctx, (void **)&nw.scan, &nw.scan_cap, (G + 1) * 8)) return rc;
            if (G) {
                if (int rc = grow_buf(ctx, &a->ref_tmp[0], &a->ref_tmp_cap[0], G * 8)) return rc;
                if (int rc = grow_buf(ctx, &a->ref_tmp[1], &a->ref_tmp_cap[1], scan_tmp_bytes((int64_t)G) + 256)) return rc;
                hipLaunchKernelGGL(ref_store_len_kernel, dim3(grid), dim3(256), 0, ctx->stream, (const uint64_t *)acc, G,
                                   old.n, in[i].n, a->S.ovf, s0, s1, (uint64_t *)a->ref_tmp[0]);
                TFG_LAUNCH_CHECK();
                if (int rc = exclusive_scan_u64(ctx, (const uint64_t *)a->ref_tmp[0], nw.scan, (int64_t)G, a->ref_tmp[1]))
                    return rc;
                if (int rc = read_back_u64(ctx, nw.scan + G, &total, 1)) return rc;
            } else {
                TFG_HIP(hipMemsetAsync(nw.scan, 0, 8, ctx->stream));
            }
            if (int rc = grow_buf(ctx, (void **)&nw.val, &nw.val_cap, total)) return rc;
            if (G) {
                ProfScope _ps(ctx, "agg.ref_store");
                hipLaunchKernelGGL(ref_store_str_kernel, dim3(grid), dim3(256), 0, ctx->stream, acc, G, old.n, in[i].n, s0,
                                   s1, (const uint64_t *)nw.scan, nw.val, nw.nul);
                TFG_LAUNCH_CHECK();
            }
        }
        nw.n = G;
        nw.bytes = total;
        std::swap(old, nw); // the old store's buffers become the spare ones
        nw.n = nw.bytes = 0;
    }
    return TFG_OK;
}

// the stores after create / reset: empty, or (without key) the one group's "no value"
int ref_reset(tfg_agg *a) {
    if (!a->has_ref) return TFG_OK;
    for (int i = 0; i < a->S.n_aggs; ++i) a->store[i].n = a->store[i].bytes = 0; // buffers kept
    if (!a->nokey) return TFG_OK;
    RefIn none[AGG_MAX];
    return ref_rebuild(a, none); // the group's references are 0 (zeroed state)
}

int consume_common(tfg_agg *a, int mode, const RowPred &pred, const void *keys, const uint8_t *key_nullmap,
                   const void *const *args, const uint8_t *const *arg_nullmaps, int64_t n) {
    TFG_CHECK(a, TFG_ERR_INVALID_ARG, "agg is null");
    TFG_CHECK(n >= 0 && n < (int64_t)0xFFFFFFFFll, TFG_ERR_INVALID_ARG, "row count out of range");
    if (failpoint("agg_consume")) return fail(TFG_ERR_FAULT_INJECTED, "failpoint agg_consume");
    if (n == 0) return TFG_OK;
    if (int rc = set_device(a->ctx)) return rc;
    if (int rc = pend_compact(a)) return rc; // this call folds into the dense state
    const void *vals[AGG_MAX] = {};
    const uint8_t *vnull[AGG_MAX] = {};
    RefIn rin[AGG_MAX];
    for (int i = 0; i < a->S.n_aggs; ++i) {
        if (mode == MODE_RAW && a->S.kind[i] == TFG_AGG_COUNT_ALL) continue;
        TFG_CHECK(args && args[i], TFG_ERR_INVALID_ARG, "argument %d is null", i);
        vals[i] = args[i];
        vnull[i] = arg_nullmaps ? arg_nullmaps[i] : nullptr;
        const int acc = a->S.acc[i];
        if (vnull[i] && mode == MODE_RAW && (a->S.kind[i] == TFG_AGG_SUM || acc == ACC_ORD || acc == ACC_REF) &&
            !a->arg_nullable[i])
            return fail(TFG_ERR_ILLEGAL_TYPE, "argument %d has a null map but was declared not nullable", i);
        if (acc != ACC_REF) continue;
        if (a->S.src_type[i] == TFG_STRING) { // a host tfg_str_col
            const tfg_str_col *sc = static_cast<const tfg_str_col *>(args[i]);
            TFG_CHECK(sc->chars && sc->offsets, TFG_ERR_INVALID_ARG, "String argument %d needs chars and offsets", i);
            rin[i] = RefIn{sc->chars, sc->offsets, vnull[i], (uint64_t)n};
        } else {
            rin[i] = RefIn{static_cast<const uint8_t *>(args[i]), nullptr, vnull[i], (uint64_t)n};
        }
    }
    RefCall rc(a);
    if (a->has_ref) {
        if (int r = ref_setup(a, rin, rc)) return r;
        if (!a->nokey) { // keyed: every row carries its candidate reference through the partition
            uint64_t n0 = 0;
            for (int i = 0; i < a->S.n_aggs; ++i)
                if (a->S.acc[i] == ACC_REF) n0 = a->store[i].n;
            if (int r = grow_buf(a->ctx, &a->ref_rows[0], &a->ref_rows_cap[0], (size_t)n * 8)) return r;
            void *refs = a->ref_rows[0];
            hipLaunchKernelGGL(ref_iota_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, a->ctx->stream,
                               (uint64_t *)refs, n0, n);
            TFG_LAUNCH_CHECK();
            for (int i = 0; i < a->S.n_aggs; ++i) {
                if (a->S.acc[i] != ACC_REF) continue;
                vals[i] = refs;
                if (a->S.kind[i] == TFG_AGG_FIRST_ROW) vnull[i] = nullptr; // a NULL first row counts
            }
        }
    }
    if (a->nokey) {
        if (int r = consume_nokey(a, mode, pred, vals, vnull, n)) return r;
    } else {
        TFG_CHECK(keys, TFG_ERR_INVALID_ARG, "keys are null");
        if (a->S.key_width == 16) TFG_CHECK(!key_nullmap, TFG_ERR_INVALID_ARG, "packed keys carry their NULL bits");
        if (int r = consume_keyed(a, mode, pred, keys, a->S.key_width, key_nullmap, vals, vnull, nullptr, nullptr, n))
            return r;
    }
    if (a->has_ref)
        if (int r = ref_rebuild(a, rin)) return r;
    return check_overflow(a);
}

} // namespace

// ---------------------------------------------------------------- the serialized method (serial.h)
// Key columns + states of an aggregator's groups in temporary device buffers (tfg_agg_result_keys).
struct AggExtract {
    uint64_t G = 0;
    int nkeys = 0, n_aggs = 0;
    void *kc[8] = {};
    uint64_t *ko[8] = {};
    uint8_t *kn[8] = {};
    void *st[AGG_MAX] = {};    // result entries: a device column, or (String) &so[i]
    void *st_in[AGG_MAX] = {}; // the same states as consume arguments: the column, or (String) &sc[i]
    uint8_t *sn[AGG_MAX] = {};
    tfg_str_out so[AGG_MAX] = {};
    tfg_str_col sc[AGG_MAX] = {};
    Ctx *ctx = nullptr;  // the buffers live in its call arena (no allocation in steady state) ...
    Ctx *user = nullptr; // ... and are read by this context's stream too (a merge's destination)
    ~AggExtract() {
        if (!ctx) return;
        if (user && user != ctx && user->stream != ctx->stream) (void)hipStreamSynchronize(user->stream);
        arena_drop(ctx);
    }
    int alloc(size_t bytes, void **p) { return arena_alloc(ctx, std::max<size_t>(bytes, 8), p); }
};

static int agg_extract(tfg_agg *a, AggExtract &e) {
    TFG_CHECK(!e.ctx, TFG_ERR_LOGICAL, "extract reused");
    arena_hold(a->ctx); // dropped by e's destructor
    e.ctx = a->ctx;
    uint64_t G = 0;
    if (int rc = tfg_agg_size(a, &G)) return rc;
    e.G = G;
    e.nkeys = a->kp.nkeys;
    e.n_aggs = a->sdict ? a->inner->S.n_aggs : a->S.n_aggs;
    if (G == 0) return TFG_OK;
    uint64_t chars = 0;
    bool has_str = false;
    for (int j = 0; j < e.nkeys; ++j) has_str |= a->key_types[j] == TFG_STRING;
    if (has_str) { // the chars size first (TFG_ERR_CAPACITY reports it)
        void *dummy;
        if (int rc = e.alloc(8, &dummy)) return rc;
        void *pc[8];
        uint64_t *po[8];
        for (int j = 0; j < 8; ++j) {
            pc[j] = dummy;
            po[j] = (uint64_t *)dummy;
        }
        const int rc = tfg_agg_result_keys(a, pc, po, nullptr, nullptr, nullptr, G, 0, nullptr, &chars);
        if (rc && rc != TFG_ERR_CAPACITY) return rc;
    }
    for (int j = 0; j < e.nkeys; ++j) {
        void *p;
        const bool str = a->key_types[j] == TFG_STRING;
        if (int rc = e.alloc(str ? chars : G * type_width(a->key_types[j]), &p)) return rc;
        e.kc[j] = p;
        if (str) {
            if (int rc = e.alloc(G * 8, &p)) return rc;
            e.ko[j] = (uint64_t *)p;
        }
        if (int rc = e.alloc(G, &p)) return rc;
        e.kn[j] = (uint8_t *)p;
    }
    for (int i = 0; i < e.n_aggs; ++i) {
        int t = 0, w = 0;
        if (int rc = tfg_agg_result_type(a, i, &t, &w)) return rc;
        void *p;
        if (int rc = e.alloc(G * (size_t)w, &p)) return rc;
        e.st[i] = e.st_in[i] = p;
        if (t == TFG_STRING) { // min / max / first_row of a String: offsets, then the chars
            uint64_t bytes = 0;
            if (int rc = tfg_agg_result_chars(a, i, &bytes)) return rc;
            void *c;
            if (int rc = e.alloc(bytes, &c)) return rc;
            e.so[i] = tfg_str_out{(uint8_t *)c, (uint64_t *)p, bytes};
            e.sc[i] = tfg_str_col{(const uint8_t *)c, (const uint64_t *)p};
            e.st[i] = &e.so[i];
            e.st_in[i] = &e.sc[i];
        }
        if (int rc = e.alloc(G, &p)) return rc;
        e.sn[i] = (uint8_t *)p;
    }
    return tfg_agg_result_keys(a, e.kc, e.ko, e.kn, e.st, e.sn, G, chars, nullptr, nullptr);
}

// rows -> dictionary group ids (in pack_buf) -> the inner aggregator
static int serial_consume(tfg_agg *a, const void *const *key_cols, const uint64_t *const *key_offsets,
                          const uint8_t *const *key_nullmaps, const void *const *vals, const uint8_t *const *val_nullmaps,
                          const uint8_t *mask, int64_t n, bool partial) {
    if (n <= 0) return n == 0 ? TFG_OK : fail(TFG_ERR_INVALID_ARG, "negative row count");
    if (int rc = set_device(a->ctx)) return rc;
    if (int rc = a->ensure_pack((size_t)n)) return rc;
    uint32_t *gid = (uint32_t *)a->pack_buf;
    if (int rc = serial_dict_assign(a->sdict, key_cols, key_offsets, key_nullmaps, mask, n, gid)) return rc;
    if (partial) return tfg_agg_consume_partial(a->inner, gid, nullptr, vals, val_nullmaps, n);
    return tfg_agg_consume(a->inner, gid, nullptr, vals, val_nullmaps, mask, n);
}

// Moves an aggregator to the serialized method: a dictionary over its key columns, an inner
// aggregator over UInt32 group ids, and (for a packed-key aggregator that already holds groups)
// its groups merged in as partial states.
static int serial_adopt(tfg_agg *a) {
    SerialDict *d = nullptr;
    if (int rc = serial_dict_create(a->ctx, a->kp.nkeys, a->key_types, a->key_collators, &d)) return rc;
    tfg_agg *in = nullptr;
    if (int rc = tfg_agg_create(static_cast<tfg_ctx *>(a->ctx), TFG_UINT32, a->S.n_aggs, a->c_kinds, a->c_types, a->c_scales, &a->c_params, &in)) {
        serial_dict_destroy(d);
        return rc;
    }
    AggExtract e;
    uint64_t held = 0;
    if (int rc = tfg_agg_size(a, &held)) {
        serial_dict_destroy(d);
        tfg_agg_destroy(in);
        return rc;
    }
    if (held) {
        if (int rc = agg_extract(a, e)) {
            serial_dict_destroy(d);
            tfg_agg_destroy(in);
            return rc;
        }
    }
    a->sdict = d;
    a->inner = in;
    a->long_key = false;
    if (e.G) return serial_consume(a, e.kc, e.ko, e.kn, e.st_in, e.sn, nullptr, (int64_t)e.G, true);
    return TFG_OK;
}

// tfg_agg_merge when either side uses the serialized method: src's groups as key columns + states
static int merge_through_keys(tfg_agg *dst, tfg_agg *src) {
    TFG_CHECK(dst->kp.nkeys == src->kp.nkeys, TFG_ERR_LOGICAL, "merging aggregators of different signatures");
    for (int j = 0; j < dst->kp.nkeys; ++j)
        TFG_CHECK(dst->key_types[j] == src->key_types[j], TFG_ERR_LOGICAL, "merging aggregators of different signatures");
    TFG_HIP(hipStreamSynchronize(src->ctx->stream));
    AggExtract e;
    e.user = dst->ctx;
    if (int rc = agg_extract(src, e)) return rc;
    if (e.G == 0) return TFG_OK;
    TFG_HIP(hipStreamSynchronize(src->ctx->stream));
    return tfg_agg_consume_partial_keys(dst, e.kc, e.ko, e.kn, e.st_in, e.sn, (int64_t)e.G);
}

extern "C" {

int tfg_agg_create(tfg_ctx *ctx, int key_type, int n_aggs, const int *agg_kinds, const int *arg_types,
                   const int *arg_scales, const tfg_agg_params *params, tfg_agg **out) {
    TFG_CHECK(ctx && out && agg_kinds, TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(n_aggs >= 1 && n_aggs <= AGG_MAX, TFG_ERR_NOT_IMPLEMENTED, "n_aggs %d out of range [1,%d]", n_aggs, AGG_MAX);
    TFG_CHECK(key_type == 0 || key_type == TFG_KEYS128 || (type_width(key_type) > 0 && type_width(key_type) <= 8),
              TFG_ERR_ILLEGAL_TYPE, "unsupported GROUP BY key type %d", key_type);
    if (int rc = set_device(ctx)) return rc;
    tfg_agg *a = new tfg_agg();
    a->ctx = ctx;
    a->key_type = key_type;
    a->nokey = key_type == 0;
    AggSpec &S = a->S;
    const bool wide = key_type == TFG_KEYS128;
    S.key_width = wide ? 16 : (int)type_width(key_type);
    S.n_aggs = n_aggs;
    int cell = wide ? 24 : 8; // key (wide: tag + 16-byte key)
    for (int i = 0; i < n_aggs; ++i) {
        const int kind = agg_kinds[i];
        const int at = arg_types ? TFG_ARG_TYPE(arg_types[i]) : 0;
        const bool nullable = arg_types && (arg_types[i] & TFG_ARG_NULLABLE);
        if (arg_types && TFG_ARG_PREC_OF(arg_types[i]) > 65) {
            delete a;
            return fail(TFG_ERR_ILLEGAL_TYPE, "decimal precision %d of argument %d exceeds 65", TFG_ARG_PREC_OF(arg_types[i]), i);
        }
        if (kind < TFG_AGG_SUM || kind > TFG_AGG_FIRST_ROW) {
            delete a;
            return fail(TFG_ERR_NOT_IMPLEMENTED, "aggregate kind %d not supported", kind);
        }
        S.kind[i] = kind;
        S.src_type[i] = at;
        a->arg_types[i] = at;
        a->arg_nullable[i] = nullable;
        if (kind == TFG_AGG_SUM) {
            if (!(is_fixed_numeric(at) || is_decimal_type(at) || at == TFG_DECIMAL256)) {
                delete a;
                return fail(TFG_ERR_ILLEGAL_TYPE, "sum over type %d not supported", at);
            }
            S.acc[i] = sum_acc_kind(arg_types[i]);
            S.has_cnt[i] = nullable ? 1 : 0;
            a->result_type[i] = S.acc[i] == ACC_F64 ? TFG_FLOAT64
                                : S.acc[i] == ACC_I256 ? TFG_DECIMAL256
                                : S.acc[i] == ACC_I128 ? TFG_DECIMAL128
                                : is_unsigned_type(at) ? TFG_UINT64 : TFG_INT64;
            a->result_width[i] = 8 * acc_words(S.acc[i]);
            cell += 8 * lds_acc_words(S.acc[i]);
        } else if (kind == TFG_AGG_MIN || kind == TFG_AGG_MAX || kind == TFG_AGG_FIRST_ROW) {
            const bool numeric = is_fixed_numeric(at) || at == TFG_DECIMAL32 || at == TFG_DECIMAL64;
            const bool wide = at == TFG_DECIMAL128 || at == TFG_DECIMAL256 || at == TFG_STRING;
            const int coll = arg_types ? TFG_ARG_COLLATOR_OF(arg_types[i]) : 0;
            if (!numeric && !wide) {
                delete a;
                return fail(TFG_ERR_ILLEGAL_TYPE, "min / max / first_row over type %d not supported", at);
            }
            if (at == TFG_STRING && !collator_known(coll)) {
                delete a;
                return fail(TFG_ERR_NOT_IMPLEMENTED, "collator %d not supported", coll);
            }
            if (kind == TFG_AGG_FIRST_ROW || wide) { // the group keeps a reference to its winning row
                S.acc[i] = ACC_REF;
                S.has_cnt[i] = 0;
                a->has_ref = true;
                a->ref_coll[i] = at == TFG_STRING ? coll : 0;
            } else { // numeric min / max: an order key; the count tells "no value" (NULL, or 0 without key)
                S.acc[i] = ACC_ORD;
                S.has_cnt[i] = (nullable || a->nokey) ? 1 : 0;
            }
            a->result_type[i] = at;
            a->result_width[i] = at == TFG_STRING ? 8 : (int)type_width(at);
            cell += 8;
        } else {
            S.acc[i] = ACC_NONE;
            S.has_cnt[i] = 1;
            a->result_type[i] = TFG_UINT64;
            a->result_width[i] = 8;
        }
        if (S.has_cnt[i]) cell += 8;
        (void)arg_scales;
    }
    // buckets: as many groups per bucket as the largest LDS table holds with slack (~4K for
    // 8-byte keys with sum + count, the TwoLevelHashTable analogue): fewer buckets give the radix
    // scatter longer runs per destination (measured: 256 buckets with 6K-cell tables 53.6G rows/s
    // against 512 with 4K-cell tables 48.5G on C2); at least 256 buckets, one per CU
    const int64_t eg = (params && params->expected_groups > 0) ? params->expected_groups : (1 << 20);
    int bbits = params ? params->bucket_bits : 0;
    // largest-table fill: inserts reserve cells (Table::reserve), so no headroom for in-flight
    // inserts is needed; wide keys (48-byte cells with a Decimal128 sum) fill to 7/8
    const int fill_big = wide ? 7 : 6;
    // wide keys may use up to 2^14 buckets: their two-level partition (coarse B >> 6, fine 64)
    // stays within 256 coarse destinations.  Their probe (tag, then the 16-byte key) is
    // latency-bound and slows sharply with the load factor, so they aim at ~3/8 of the largest
    // table: C5's 10M groups -> 16384 buckets (wide bucket kernel 1.92 ms, against 2.67 ms at
    // 8192 buckets / ~60% and 3.72 ms at 4096 / ~80%, r03); the table itself is then sized for
    // two workgroups per CU (below)
    // TFG_WIDE_QUAD=1 (A/B): wide keys in 256-thread workgroups with ~38 KB of LDS, four per CU,
    // over up to 2^15 buckets (two levels: 512 coarse x 64 fine)
    static const bool quad_env = [] {
        const char *v = getenv("TFG_WIDE_QUAD");
        return v && *v == '1';
    }();
    const bool quad = wide && !a->nokey && quad_env;
    size_t wide_cell = 8 + 16; // tag + 16-byte key, then the accumulators (below)
    for (int i = 0; i < n_aggs; ++i) {
        if (S.acc[i] != ACC_NONE) wide_cell += 8 * (size_t)lds_acc_words(S.acc[i]);
        if (S.has_cnt[i]) wide_cell += 8;
    }
    // quad: the 256-thread kernel's static LDS (~6.5 KB) beside a table in a quarter of the CU
    const int quad_cells = (int)(((40 * 1024 - 6656 - sizeof(Ctrl) - 16) / wide_cell - 2) & ~(size_t)63);
    const int max_bits = wide ? (quad ? 15 : 14) : 12;
    if (bbits <= 0) {
        const int64_t cells_max = LDS_TABLE_MAX / cell;
        const int64_t fit = quad ? (int64_t)quad_cells * 42 / 100
                                 : wide ? cells_max * 3 / 8 : (cells_max * fill_big / 8) * 5 / 6;
        bbits = 8;
        while (bbits < max_bits && ((int64_t)1 << bbits) * fit < eg) ++bbits;
    }
    if (bbits > max_bits) bbits = max_bits;
    a->B = a->nokey ? 1 : (1u << bbits);
    // LDS table geometry: room for a bucket's expected groups with 25% slack and headroom for one
    // step of in-flight inserts.  Power-of-two tables up to LDS_TABLE_BYTES (fill <= 5/8; 2-3
    // workgroups share a CU); a bucket too large for that gets the largest table one workgroup per
    // CU can hold (any multiple of 256 cells, fill <= 3/4)
    const int64_t per_bucket = eg / (int64_t)a->B + 1;
    const int64_t need = per_bucket * 5 / 4;
    int cap = 256;
    while (cap < (1 << 16) && cap * 5 / 8 < need) cap *= 2;
    int fill_num = 5;
    if ((size_t)(cap + 2) * cell > (size_t)LDS_TABLE_BYTES) {
        int c2 = 256;
        while ((size_t)(c2 + 256 + 2) * cell <= (size_t)LDS_TABLE_MAX && c2 * fill_big / 8 < need) c2 += 256;
        cap = c2;
        fill_num = fill_big;
    }
    if (quad && per_bucket * 100 <= (int64_t)quad_cells * 45 && quad_cells * fill_big / 8 >= need) {
        cap = quad_cells;
        fill_num = fill_big;
    } else if (wide && !a->nokey) {
        // wide keys: the probe is latency-bound, so two 8-wave workgroups per CU (the 512-thread
        // kernel at 128 VGPRs) beat one 16-wave workgroup with a larger, emptier table: C5 1472
        // cells at ~42 % load 4.37 ms vs 2048 at ~30 % 4.66 ms (r05z).  The largest table (64-cell
        // steps) whose LDS plus that kernel's ~8.5 KB of static LDS fits half a CU, if the bucket
        // fills at most 45 % of it
        size_t per_cell = 8 + 16; // tag + 16-byte key
        for (int i = 0; i < n_aggs; ++i) {
            if (S.acc[i] != ACC_NONE) per_cell += 8 * (size_t)lds_acc_words(S.acc[i]);
            if (S.has_cnt[i]) per_cell += 8;
        }
        const size_t dyn = 80 * 1024 - 8704 - sizeof(Ctrl) - 16;
        const int c2 = (int)((dyn / per_cell - 2) & ~(size_t)63);
        if (c2 >= 256 && per_bucket * 100 <= (int64_t)c2 * 45 && c2 * fill_big / 8 >= need) {
            cap = c2;
            fill_num = fill_big;
        }
    }
    if (const char *tc = getenv("TFG_AGG_TABLE_CELLS")) { // tuning experiments: cells a bucket table
        // bounded by what a CU's 160 KB leaves beside the largest bucket kernel's static LDS
        // (the tiled 1024-thread kernel's run records and sampled run index: ~12.5 KB)
        const int c = atoi(tc) & ~63;
        if (c >= 256 && (size_t)(c + 2) * cell + sizeof(Ctrl) + 16 <= (size_t)(LDS_CU_BYTES - BUCKET_STATIC_LDS_MAX)) {
            cap = c;
            fill_num = fill_big;
        }
    }
    S.cap = cap;
    S.bbits = a->nokey ? 0 : bbits;
    S.ngroups = (unsigned)(cap / 4); // GS = 4
    int off = (cap + 2) * 8;
    if (wide) {
        S.wkey_off = off;
        off += cap * 16;
    }
    for (int i = 0; i < n_aggs; ++i) {
        if (S.acc[i] != ACC_NONE) {
            S.acc_off[i] = off;
            off += (cap + 2) * 8 * lds_acc_words(S.acc[i]);
        }
        if (S.has_cnt[i]) {
            S.cnt_off[i] = off;
            off += (cap + 2) * 8;
        }
    }
    S.ctrl_off = off;
    S.lds_bytes = off + (int)sizeof(Ctrl) + 16;
    S.ovf = nullptr;
    for (int i = 0; i < n_aggs; ++i)
        if ((S.acc[i] == ACC_I256 || S.acc[i] == ACC_REF) && !S.ovf) { // Decimal256 overflow / bad reference flags
            if (hipMalloc((void **)&S.ovf, sizeof(unsigned)) != hipSuccess ||
                hipMemsetAsync(S.ovf, 0, sizeof(unsigned), ctx->stream) != hipSuccess) {
                if (S.ovf) (void)hipFree(S.ovf);
                delete a;
                return fail(TFG_ERR_OOM, "overflow flag allocation failed");
            }
        }
    // one workgroup per CU anyway (LDS): make it 16 waves, and keep the in-flight insert headroom
    S.bt = S.lds_bytes > 80 * 1024 ? BT_BIG : BT;
    if (quad && S.lds_bytes <= 40 * 1024 - 6656) S.bt = BT_QUAD; // the wide tiled kernel only (agg_bucket_wide.hip)
    S.maxfill = std::max(1, std::min(cap * fill_num / 8, cap - 8));
    if (a->nokey) {
        if (int rc = a->ensure_state(0, 1)) {
            delete a;
            return rc;
        }
        size_t bytes = a->carve_groups(nullptr, a->cap[0], a->st[0]);
        TFG_HIP(hipMemsetAsync(a->blk[0], 0, bytes, ctx->stream));
        a->n_groups = 1;
    }
    if (int rc = ref_reset(a)) {
        tfg_agg_destroy(a);
        return rc;
    }
    *out = a;
    return TFG_OK;
}

int tfg_agg_destroy(tfg_agg *a) {
    if (!a) return TFG_OK;
    (void)hipSetDevice(a->ctx->device);
    (void)hipStreamSynchronize(a->ctx->stream);
    for (int i = 0; i < 2; ++i) {
        if (a->blk[i]) (void)hipFree(a->blk[i]);
        if (a->bucket_off[i]) (void)hipFree(a->bucket_off[i]);
    }
    for (int i = 0; i < AGG_MAX; ++i) {
        ref_store_free(a->store[i]);
        ref_store_free(a->spare[i]);
        if (a->ref_rows[i]) (void)hipFree(a->ref_rows[i]);
    }
    for (int i = 0; i < 2; ++i)
        if (a->ref_tmp[i]) (void)hipFree(a->ref_tmp[i]);
    if (a->pack_buf) (void)hipFree(a->pack_buf);
    if (a->pack_err) (void)hipFree(a->pack_err);
    if (a->pend_blk) (void)hipFree(a->pend_blk);
    if (a->pend_dev) (void)hipFree(a->pend_dev);
    if (a->pend_ch) (void)hipFree(a->pend_ch);
    if (a->S.ovf) (void)hipFree(a->S.ovf);
    if (a->sdict) serial_dict_destroy(a->sdict);
    if (a->inner) tfg_agg_destroy(a->inner);
    delete a;
    return TFG_OK;
}

int tfg_agg_reset(tfg_agg *a) {
    TFG_CHECK(a, TFG_ERR_INVALID_ARG, "agg is null");
    a->pending = false; // the pending groups are dropped with the rest
    if (a->sdict) {
        if (int rc = set_device(a->ctx)) return rc;
        serial_dict_reset(a->sdict);
        return tfg_agg_reset(a->inner);
    }
    if (a->nokey) {
        if (int rc = set_device(a->ctx)) return rc;
        size_t bytes = a->carve_groups(nullptr, a->cap[a->cur], a->st[a->cur]);
        TFG_HIP(hipMemsetAsync(a->blk[a->cur], 0, bytes, a->ctx->stream));
        a->n_groups = 1;
    } else {
        a->n_groups = 0;
    }
    if (a->has_ref) {
        if (int rc = set_device(a->ctx)) return rc;
        return ref_reset(a);
    }
    return TFG_OK;
}

int tfg_agg_consume(tfg_agg *a, const void *keys, const uint8_t *key_nullmap, const void *const *args,
                    const uint8_t *const *arg_nullmaps, const uint8_t *mask, int64_t n) {
    TFG_CHECK(a, TFG_ERR_INVALID_ARG, "agg is null");
    TFG_CHECK(!a->sdict, TFG_ERR_NOT_IMPLEMENTED, "serialized GROUP BY keys: consume through tfg_agg_consume_keys");
    RowPred pred{};
    if (mask) {
        pred.kind = 1;
        pred.col = mask;
    }
    return consume_common(a, MODE_RAW, pred, keys, key_nullmap, args, arg_nullmaps, n);
}

int tfg_agg_consume_filtered(tfg_agg *a, int pred_type, const void *pred_col, const uint8_t *pred_nullmap, int op,
                             int scalar_type, const void *scalar_host, const void *keys, const uint8_t *key_nullmap,
                             const void *const *args, const uint8_t *const *arg_nullmaps, int64_t n) {
    TFG_CHECK(a && pred_col && scalar_host, TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(!a->sdict, TFG_ERR_NOT_IMPLEMENTED, "serialized GROUP BY keys: consume through tfg_agg_consume_keys");
    TFG_CHECK(is_fixed_numeric(pred_type) && is_fixed_numeric(scalar_type), TFG_ERR_ILLEGAL_TYPE,
              "unsupported predicate types %d / %d", pred_type, scalar_type);
    TFG_CHECK(op >= TFG_EQ && op <= TFG_GE, TFG_ERR_INVALID_ARG, "bad comparison op %d", op);
    RowPred pred{};
    pred.kind = 2;
    pred.type = pred_type;
    pred.col = pred_col;
    pred.nullmap = pred_nullmap;
    pred.b = host_num(scalar_type, scalar_host);
    pred.op = op;
    return consume_common(a, MODE_RAW, pred, keys, key_nullmap, args, arg_nullmaps, n);
}

int tfg_agg_consume_partial(tfg_agg *a, const void *keys, const uint8_t *key_nullmap, const void *const *states,
                            const uint8_t *const *state_nullmaps, int64_t n) {
    TFG_CHECK(a, TFG_ERR_INVALID_ARG, "agg is null");
    TFG_CHECK(!a->sdict, TFG_ERR_NOT_IMPLEMENTED,
              "serialized GROUP BY keys have no packed form: merge through tfg_agg_consume_partial_keys");
    RowPred pred{};
    return consume_common(a, MODE_PARTIAL, pred, keys, key_nullmap, states, state_nullmaps, n);
}

int tfg_agg_merge(tfg_agg *dst, tfg_agg *src) {
    TFG_CHECK(dst && src, TFG_ERR_INVALID_ARG, "null agg");
    if (dst->sdict || src->sdict) return merge_through_keys(dst, src);
    TFG_CHECK(dst->key_type == src->key_type && dst->S.n_aggs == src->S.n_aggs && dst->B == src->B,
              TFG_ERR_LOGICAL, "merging aggregators of different signatures");
    for (int i = 0; i < dst->S.n_aggs; ++i)
        TFG_CHECK(dst->S.kind[i] == src->S.kind[i] && dst->S.acc[i] == src->S.acc[i] &&
                      dst->S.has_cnt[i] == src->S.has_cnt[i] &&
                      (dst->S.acc[i] != ACC_REF ||
                       (dst->S.src_type[i] == src->S.src_type[i] && dst->ref_coll[i] == src->ref_coll[i])),
                  TFG_ERR_LOGICAL, "merging aggregators of different signatures");
    if (int rc = set_device(dst->ctx)) return rc;
    if (int rc = pend_compact(dst)) return rc;
    if (int rc = set_device(src->ctx)) return rc;
    if (int rc = pend_compact(src)) return rc;
    if (int rc = set_device(dst->ctx)) return rc;
    TFG_HIP(hipStreamSynchronize(src->ctx->stream));
    // row-reference aggregates: the candidates are dst's store, then src's (changeFirstTime(to) /
    // changeIfLess(to) keep dst's value on ties: Aggregator::mergeDataImpl folds src into dst)
    RefIn rin[AGG_MAX];
    RefCall rc(dst);
    if (dst->has_ref) {
        for (int i = 0; i < dst->S.n_aggs; ++i) {
            if (dst->S.acc[i] != ACC_REF) continue;
            const RefStore &ss = src->store[i];
            TFG_CHECK(ss.n == src->n_groups, TFG_ERR_LOGICAL, "value store out of step with the groups");
            rin[i] = RefIn{ss.val, ss.scan ? ss.scan + 1 : nullptr, ss.nul, ss.n, ss.bytes};
        }
        if (int r = ref_setup(dst, rin, rc)) return r;
    }
    if (dst->nokey) {
        hipLaunchKernelGGL(agg_state_add_kernel, dim3(1), dim3(64), 0, dst->ctx->stream, dst->S, dst->st[dst->cur],
                           src->st[src->cur]);
        TFG_LAUNCH_CHECK();
        if (dst->has_ref)
            if (int r = ref_rebuild(dst, rin)) return r;
        return check_overflow(dst);
    }
    if (src->n_groups == 0) return TFG_OK;
    const GroupsIO &g = src->st[src->cur];
    const void *vals[AGG_MAX] = {};
    const uint64_t *cnts[AGG_MAX] = {};
    for (int i = 0; i < src->S.n_aggs; ++i) {
        vals[i] = g.acc[i];
        cnts[i] = g.cnt[i];
        if (src->S.acc[i] != ACC_REF) continue;
        // src's references, moved past dst's store
        if (int r = grow_buf(dst->ctx, &dst->ref_rows[i], &dst->ref_rows_cap[i], src->n_groups * 8)) return r;
        void *sh = dst->ref_rows[i];
        hipLaunchKernelGGL(ref_shift_kernel, dim3(stream_grid((int64_t)src->n_groups, 256, 4096)), dim3(256), 0,
                           dst->ctx->stream, (const uint64_t *)g.acc[i], dst->store[i].n, (int64_t)src->n_groups,
                           (uint64_t *)sh);
        TFG_LAUNCH_CHECK();
        vals[i] = sh;
    }
    RowPred pred{};
    if (int r = consume_keyed(dst, MODE_STATE, pred, g.key, dst->S.key_width == 16 ? 16 : 8, g.key_null, vals, nullptr,
                              cnts, src->bucket_off[src->cur], (int64_t)src->n_groups))
        return r;
    if (dst->has_ref)
        if (int r = ref_rebuild(dst, rin)) return r;
    return check_overflow(dst);
}

int tfg_agg_size(tfg_agg *a, uint64_t *out_groups) {
    TFG_CHECK(a && out_groups, TFG_ERR_INVALID_ARG, "null argument");
    if (a->sdict) return tfg_agg_size(a->inner, out_groups);
    if (a->pending) {
        if (int rc = set_device(a->ctx)) return rc;
        if (int rc = pend_counts(a)) return rc;
        *out_groups = a->pend_total;
        return TFG_OK;
    }
    *out_groups = a->n_groups;
    return TFG_OK;
}

int tfg_agg_result_type(tfg_agg *a, int i, int *out_type, int *out_width) {
    TFG_CHECK(a, TFG_ERR_INVALID_ARG, "agg is null");
    if (a->sdict) return tfg_agg_result_type(a->inner, i, out_type, out_width);
    TFG_CHECK(i >= 0 && i < a->S.n_aggs, TFG_ERR_INVALID_ARG, "bad aggregate index");
    if (out_type) *out_type = a->result_type[i];
    if (out_width) *out_width = a->result_width[i];
    return TFG_OK;
}

// a result call that may run before the group count is read: a tiled consume's pending groups,
// count unknown, no value stores (their rebuild needs the count), room for some groups
static bool result_early(const tfg_agg *a, uint64_t capacity) {
    return a->pending && !a->pend_known && !a->has_ref && capacity > 0;
}

// the pending groups' result rows into `capacity` slots (rows past it dropped); the count stays on
// the device at pend_off()[B]
static int result_pending_launch(tfg_agg *a, void *out_keys, uint8_t *out_key_nullmap, void *const *out_states,
                                 uint8_t *const *out_state_nullmaps, uint64_t capacity) {
    ResultPtrs rp{};
    for (int i = 0; i < a->S.n_aggs; ++i) {
        rp.state[i] = out_states ? out_states[i] : nullptr;
        rp.state_null[i] = out_state_nullmaps ? out_state_nullmaps[i] : nullptr;
        rp.nullable[i] = a->arg_nullable[i] || a->S.kind[i] == TFG_AGG_FIRST_ROW;
    }
    if (a->B <= (uint32_t)RSCAN_MAXB) { // the offsets computed by the result kernel itself
        ProfScope _ps(a->ctx, "agg.result");
        hipLaunchKernelGGL(agg_result_buckets_scan_kernel, dim3(a->B * RSCAN_SPLIT), dim3(256), 0, a->ctx->stream,
                           a->S, a->pend, (const uint64_t *)a->pend_cnt(), (const uint64_t *)a->pend_base(),
                           a->pend_off(), (int)a->B, a->S.key_width, out_keys, out_key_nullmap, rp, capacity);
        TFG_LAUNCH_CHECK();
        return TFG_OK;
    }
    if (int rc = pend_scan(a)) return rc;
    {
        ProfScope _ps(a->ctx, "agg.result");
        hipLaunchKernelGGL(agg_result_buckets_kernel, dim3(a->B), dim3(256), 0, a->ctx->stream, a->S, a->pend,
                           (const uint64_t *)a->pend_cnt(), (const uint64_t *)a->pend_base(),
                           (const uint64_t *)a->pend_off(), a->S.key_width, out_keys, out_key_nullmap, rp, capacity);
    }
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_agg_result(tfg_agg *a, void *out_keys, uint8_t *out_key_nullmap, void *const *out_states,
                   uint8_t *const *out_state_nullmaps, uint64_t capacity, uint64_t *out_groups_host) {
    TFG_CHECK(a, TFG_ERR_INVALID_ARG, "agg is null");
    TFG_CHECK(!a->sdict, TFG_ERR_NOT_IMPLEMENTED,
              "serialized GROUP BY keys have no packed form: read them with tfg_agg_result_keys");
    if (result_early(a, capacity)) {
        // groups of a tiled consume, count not read yet: the result is written first (groups
        // past `capacity` dropped) and the count read after it, so no host round trip idles the
        // device between the consume and the result
        if (int rc = set_device(a->ctx)) return rc;
        if (int rc = result_pending_launch(a, out_keys, out_key_nullmap, out_states, out_state_nullmaps, capacity))
            return rc;
        if (int rc = pend_read_total(a)) return rc;
        if (out_groups_host) *out_groups_host = a->pend_total;
        if (a->pend_total > capacity)
            return fail(TFG_ERR_CAPACITY, "result needs %llu groups, capacity %llu (the first %llu written)",
                        (unsigned long long)a->pend_total, (unsigned long long)capacity,
                        (unsigned long long)capacity);
        return TFG_OK;
    }
    uint64_t G = 0;
    if (int rc = tfg_agg_size(a, &G)) return rc;
    if (out_groups_host) *out_groups_host = G;
    if (G > capacity) return fail(TFG_ERR_CAPACITY, "result needs %llu groups, capacity %llu",
                                  (unsigned long long)G, (unsigned long long)capacity);
    if (G == 0) return TFG_OK;
    ResultPtrs rp{};
    for (int i = 0; i < a->S.n_aggs; ++i) {
        rp.state[i] = out_states ? out_states[i] : nullptr;
        rp.state_null[i] = out_state_nullmaps ? out_state_nullmaps[i] : nullptr;
        // sum / min / max of a Nullable argument and every first_row are Nullable
        // (AggregateFunctionNullUnary / AggregateFunctionFirstRowNull)
        rp.nullable[i] = a->arg_nullable[i] || a->S.kind[i] == TFG_AGG_FIRST_ROW;
    }
    for (int i = 0; i < a->S.n_aggs; ++i) { // a String result must fit before anything is written
        if (a->S.acc[i] != ACC_REF || a->S.src_type[i] != TFG_STRING || !rp.state[i]) continue;
        const tfg_str_out *so = static_cast<const tfg_str_out *>(rp.state[i]);
        TFG_CHECK(so->offsets && (so->chars || a->store[i].bytes == 0), TFG_ERR_INVALID_ARG,
                  "String result %d needs chars and offsets", i);
        if (a->store[i].bytes > so->chars_capacity)
            return fail(TFG_ERR_CAPACITY, "String result %d needs %llu chars bytes, capacity %llu", i,
                        (unsigned long long)a->store[i].bytes, (unsigned long long)so->chars_capacity);
    }
    if (int rc = set_device(a->ctx)) return rc;
    { ProfScope _ps(a->ctx, "agg.result");
    if (a->pending) // straight from the tiled consume's buckets
        hipLaunchKernelGGL(agg_result_buckets_kernel, dim3(a->B), dim3(256), 0, a->ctx->stream, a->S, a->pend,
                           (const uint64_t *)a->pend_cnt(), (const uint64_t *)a->pend_base(),
                           (const uint64_t *)a->pend_off(), a->S.key_width, out_keys, out_key_nullmap, rp, G);
    else
        hipLaunchKernelGGL(agg_result_kernel, dim3(stream_grid((int64_t)G, 256, 4096)), dim3(256), 0, a->ctx->stream,
                           a->S, a->st[a->cur], G, a->S.key_width, a->nokey ? nullptr : out_keys, out_key_nullmap, rp);
    }
    TFG_LAUNCH_CHECK();
    for (int i = 0; i < a->S.n_aggs; ++i) { // row-reference aggregates: their stores are the result
        if (a->S.acc[i] != ACC_REF) continue;
        const RefStore &st = a->store[i];
        TFG_CHECK(st.n == G, TFG_ERR_LOGICAL, "value store out of step with the groups");
        hipStream_t sm = a->ctx->stream;
        if (rp.state_null[i]) {
            if (rp.nullable[i]) TFG_HIP(hipMemcpyAsync(rp.state_null[i], st.nul, G, hipMemcpyDeviceToDevice, sm));
            else TFG_HIP(hipMemsetAsync(rp.state_null[i], 0, G, sm)); // the type's default, never NULL
        }
        if (!rp.state[i]) continue;
        if (a->S.src_type[i] == TFG_STRING) {
            const tfg_str_out *so = static_cast<const tfg_str_out *>(rp.state[i]);
            TFG_HIP(hipMemcpyAsync(so->offsets, st.scan + 1, G * 8, hipMemcpyDeviceToDevice, sm));
            if (st.bytes) TFG_HIP(hipMemcpyAsync(so->chars, st.val, st.bytes, hipMemcpyDeviceToDevice, sm));
        } else {
            TFG_HIP(hipMemcpyAsync(rp.state[i], st.val, G * type_width(a->S.src_type[i]), hipMemcpyDeviceToDevice, sm));
        }
    }
    return TFG_OK;
}

int tfg_agg_weak_hash_packed(tfg_agg *a, const void *packed_keys, int64_t n, uint32_t *h) {
    TFG_CHECK(a, TFG_ERR_INVALID_ARG, "agg is null");
    TFG_CHECK(!a->sdict && a->kp.kind, TFG_ERR_NOT_IMPLEMENTED, "the aggregator holds no packed keys");
    if (n <= 0) return TFG_OK; // n = 0: does the aggregator hold packed keys?
    TFG_CHECK(packed_keys && h, TFG_ERR_INVALID_ARG, "null argument");
    if (int rc = set_device(a->ctx)) return rc;
    PackTypes pt{};
    for (int j = 0; j < a->kp.nkeys && j < 4; ++j) pt.type[j] = a->key_types[j];
    hipLaunchKernelGGL(weak_hash_packed_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, a->ctx->stream, a->kp, pt,
                       (const uint4 *)packed_keys, n, h);
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

int tfg_agg_result_chars(tfg_agg *a, int i, uint64_t *out_bytes) {
    TFG_CHECK(a && out_bytes, TFG_ERR_INVALID_ARG, "null argument");
    if (a->sdict) return tfg_agg_result_chars(a->inner, i, out_bytes);
    TFG_CHECK(i >= 0 && i < a->S.n_aggs, TFG_ERR_INVALID_ARG, "bad aggregate index");
    *out_bytes = (a->S.acc[i] == ACC_REF && a->S.src_type[i] == TFG_STRING) ? a->store[i].bytes : 0;
    return TFG_OK;
}


// ---------------------------------------------------------------- wide keys: keys128 / key_string
static int pack_keys(tfg_agg *a, const void *const *key_cols, const uint64_t *const *key_offsets,
                     const uint8_t *const *key_nullmaps, int64_t n) {
    TFG_CHECK(key_cols, TFG_ERR_INVALID_ARG, "key columns are null");
    KeyPack kp = a->kp;
    for (int j = 0; j < kp.nkeys; ++j) {
        TFG_CHECK(key_cols[j], TFG_ERR_INVALID_ARG, "key column %d is null", j);
        kp.col[j] = key_cols[j];
        kp.nullmap[j] = key_nullmaps ? key_nullmaps[j] : nullptr;
        if (kp.nullmap[j] && kp.kind == WK_FIXED && kp.off[kp.nkeys - 1] + kp.width[kp.nkeys - 1] > 15) {
            a->long_key = true; // nullable_keys256's tuples: the serialized method takes them
            return fail(TFG_ERR_NOT_IMPLEMENTED, "nullable keys of 16 bytes: no spare byte in the packed key");
        }
    }
    if (kp.kind == WK_STRING) {
        TFG_CHECK(key_offsets && key_offsets[0], TFG_ERR_INVALID_ARG, "String key needs its offsets");
        kp.offsets = key_offsets[0];
    }
    if (int rc = a->ensure_pack((size_t)n)) return rc;
    if (!a->pack_err) TFG_HIP(hipMalloc(&a->pack_err, 8));
    TFG_HIP(hipMemsetAsync(a->pack_err, 0, 8, a->ctx->stream));
    {
        ProfScope _ps(a->ctx, "agg.pack_keys");
        hipLaunchKernelGGL(pack_keys_kernel, dim3(stream_grid(n, 256 * 4, 8192)), dim3(256), 0, a->ctx->stream, kp, n,
                           (uint4 *)a->pack_buf, a->pack_err);
    }
    TFG_LAUNCH_CHECK();
    if (kp.kind == WK_STRING) {
        uint64_t err = 0;
        if (int rc = read_back_u64(a->ctx, (const uint64_t *)a->pack_err, &err, 1)) return rc;
        if ((unsigned)err) {
            a->long_key = true; // key_string past 15 bytes: the serialized method takes them
            return fail(TFG_ERR_NOT_IMPLEMENTED, "String GROUP BY key longer than 15 bytes");
        }
    }
    return TFG_OK;
}

int tfg_agg_create_keys(tfg_ctx *ctx, int nkeys, const int *key_types, const int *key_collators, int n_aggs,
                        const int *agg_kinds, const int *arg_types, const int *arg_scales, const tfg_agg_params *params,
                        tfg_agg **out) {
    TFG_CHECK(ctx && out && key_types && agg_kinds, TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(nkeys >= 1 && nkeys <= 8, TFG_ERR_NOT_IMPLEMENTED, "%d GROUP BY keys: 1-8 supported", nkeys);
    TFG_CHECK(n_aggs >= 1 && n_aggs <= AGG_MAX, TFG_ERR_NOT_IMPLEMENTED, "n_aggs %d out of range [1,%d]", n_aggs, AGG_MAX);
    if (nkeys == 1 && key_types[0] != TFG_STRING && type_width(key_types[0]) <= 8)
        return tfg_agg_create(ctx, key_types[0], n_aggs, agg_kinds, arg_types, arg_scales, params, out);
    // chooseAggregationMethod: one String key -> key_string; fixed keys within 16 bytes -> keys128;
    // anything else (String with other keys, wider fixed tuples, more than 4 keys) -> serialized
    KeyPack kp{};
    kp.nkeys = nkeys;
    bool serialized = nkeys > 4;
    int off = 0;
    for (int j = 0; j < nkeys; ++j) {
        const int t = key_types[j];
        const int c = key_collators ? key_collators[j] : TFG_COLLATOR_NONE;
        if (t == TFG_STRING) {
            TFG_CHECK(collator_known(c), TFG_ERR_NOT_IMPLEMENTED, "collator %d not supported", c);
            serialized |= nkeys > 1;
            continue;
        }
        const size_t w = type_width(t);
        TFG_CHECK(w > 0 && w <= 32, TFG_ERR_ILLEGAL_TYPE, "GROUP BY key %d of type %d cannot be packed", j, t);
        if (j < 4) {
            kp.width[j] = (int)w; // floats: raw bits, like packFixed
            kp.off[j] = off;
        }
        off += (int)w;
        serialized |= w > 8 && nkeys > 1; // a Decimal128 key with other keys
    }
    serialized |= off > 16;
    tfg_agg_params p{};
    if (params) p = *params;
    tfg_agg *a = nullptr;
    if (serialized) {
        a = new tfg_agg();
        a->ctx = ctx;
        a->key_type = TFG_KEYS128;
        a->S.n_aggs = n_aggs;
    } else {
        kp.kind = key_types[0] == TFG_STRING ? WK_STRING : WK_FIXED;
        kp.collator = key_collators ? key_collators[0] : TFG_COLLATOR_NONE;
        if (collator_transforms(kp.collator)) kp.collator = TFG_COLLATOR_NONE; // the consume collates first
        if (int rc = tfg_agg_create(ctx, TFG_KEYS128, n_aggs, agg_kinds, arg_types, arg_scales, &p, &a)) return rc;
    }
    a->kp = kp;
    if (serialized) a->kp.nkeys = nkeys;
    for (int j = 0; j < nkeys; ++j) {
        a->key_types[j] = key_types[j];
        const int c = key_collators ? key_collators[j] : TFG_COLLATOR_NONE;
        const bool tr = key_types[j] == TFG_STRING && collator_transforms(c);
        a->key_collators[j] = tr ? TFG_COLLATOR_NONE : c;
        a->key_transform[j] = tr ? c : 0;
    }
    for (int i = 0; i < n_aggs; ++i) {
        a->c_kinds[i] = agg_kinds[i];
        a->c_types[i] = arg_types ? arg_types[i] : 0;
        a->c_scales[i] = arg_scales ? arg_scales[i] : 0;
    }
    a->c_params = p;
    if (serialized) {
        if (int rc = serial_adopt(a)) {
            tfg_agg_destroy(a);
            return rc;
        }
    }
    *out = a;
    return TFG_OK;
}

static int consume_keys_packed(tfg_agg *a, const void *const *key_cols, const uint64_t *const *key_offsets,
                               const uint8_t *const *key_nullmaps, const void *const *args,
                               const uint8_t *const *arg_nullmaps, const uint8_t *mask, int64_t n);

int tfg_agg_consume_keys(tfg_agg *a, const void *const *key_cols, const uint64_t *const *key_offsets,
                         const uint8_t *const *key_nullmaps, const void *const *args, const uint8_t *const *arg_nullmaps,
                         const uint8_t *mask, int64_t n) {
    TFG_CHECK(a, TFG_ERR_INVALID_ARG, "agg is null");
    // String keys under a case-insensitive collator: HashMethodString / serializeValueIntoArena
    // take the collator's sort key (ColumnsHashing.h:233, AggregationCommon.h:202), so the rows
    // are collated into sort-key columns first (the result's key column holds the sort keys, as
    // the reference Aggregator's does)
    bool any = false;
    for (int j = 0; j < (a->kp.nkeys ? a->kp.nkeys : 1); ++j) any = any || a->key_transform[j];
    if (any && n > 0) {
        TFG_CHECK(key_cols && key_offsets, TFG_ERR_INVALID_ARG, "String keys need chars and offsets");
        if (int rc = set_device(a->ctx)) return rc;
        CollatedStrings cs[8];
        const void *kc[8] = {};
        const uint64_t *ko[8] = {};
        for (int j = 0; j < a->kp.nkeys; ++j) {
            kc[j] = key_cols[j];
            ko[j] = key_offsets[j];
            if (!a->key_transform[j]) continue;
            if (int rc = collate_strings(a->ctx, a->key_transform[j], (const uint8_t *)key_cols[j], key_offsets[j],
                                         key_nullmaps ? key_nullmaps[j] : nullptr, nullptr, nullptr, n, cs[j]))
                return rc;
            kc[j] = cs[j].chars;
            ko[j] = cs[j].offsets();
        }
        const int transforms[8] = {a->key_transform[0], a->key_transform[1], a->key_transform[2], a->key_transform[3],
                                   a->key_transform[4], a->key_transform[5], a->key_transform[6], a->key_transform[7]};
        for (int j = 0; j < 8; ++j) a->key_transform[j] = 0;
        const int rc = tfg_agg_consume_keys(a, kc, ko, key_nullmaps, args, arg_nullmaps, mask, n);
        for (int j = 0; j < 8; ++j) a->key_transform[j] = transforms[j];
        return rc;
    }
    if (a->sdict) return serial_consume(a, key_cols, key_offsets, key_nullmaps, args, arg_nullmaps, mask, n, false);
    a->long_key = false;
    int rc = consume_keys_packed(a, key_cols, key_offsets, key_nullmaps, args, arg_nullmaps, mask, n);
    if (rc == TFG_ERR_NOT_IMPLEMENTED && a->long_key) { // nothing was folded in: move, then take the block
        if ((rc = serial_adopt(a))) return rc;
        return serial_consume(a, key_cols, key_offsets, key_nullmaps, args, arg_nullmaps, mask, n, false);
    }
    return rc;
}

static int consume_keys_packed(tfg_agg *a, const void *const *key_cols, const uint64_t *const *key_offsets,
                               const uint8_t *const *key_nullmaps, const void *const *args,
                               const uint8_t *const *arg_nullmaps, const uint8_t *mask, int64_t n) {
    if (!a->kp.kind)
        return tfg_agg_consume(a, key_cols ? key_cols[0] : nullptr, key_nullmaps ? key_nullmaps[0] : nullptr, args,
                               arg_nullmaps, mask, n);
    if (n <= 0) return n == 0 ? TFG_OK : fail(TFG_ERR_INVALID_ARG, "negative row count");
    if (int rc = set_device(a->ctx)) return rc;
    // wide fast signatures: tiled partition of 16-byte keys (a String key packed as it is read)
    const int code = mask ? 0 : wide_fast_signature(a->S, arg_nullmaps);
    if (code && a->kp.kind == WK_STRING) {
        TFG_CHECK(key_cols && key_cols[0] && key_offsets && key_offsets[0], TFG_ERR_INVALID_ARG,
                  "String key needs its chars and offsets");
        if (!a->pack_err) TFG_HIP(hipMalloc(&a->pack_err, 8));
        SelWideStr sel{(const uint8_t *)key_cols[0], key_offsets[0], key_nullmaps ? key_nullmaps[0] : nullptr,
                       a->kp.collator, a->pack_err, 0};
        bool done = false;
        if (int rc = consume_wide_tiled(a, code, sel, args, n, a->pack_err, done)) return rc;
        if (done) return TFG_OK;
    }
    if (int rc = pack_keys(a, key_cols, key_offsets, key_nullmaps, n)) return rc;
    if (code) {
        bool done = false;
        if (int rc = consume_wide_tiled(a, code, SelWide2{(const uint4 *)a->pack_buf, 0}, args, n, nullptr, done)) return rc;
        if (done) return TFG_OK;
    }
    return tfg_agg_consume(a, a->pack_buf, nullptr, args, arg_nullmaps, mask, n);
}

int tfg_agg_consume_partial_keys(tfg_agg *a, const void *const *key_cols, const uint64_t *const *key_offsets,
                                 const uint8_t *const *key_nullmaps, const void *const *states,
                                 const uint8_t *const *state_nullmaps, int64_t n) {
    TFG_CHECK(a, TFG_ERR_INVALID_ARG, "agg is null");
    if (a->sdict) return serial_consume(a, key_cols, key_offsets, key_nullmaps, states, state_nullmaps, nullptr, n, true);
    if (!a->kp.kind)
        return tfg_agg_consume_partial(a, key_cols ? key_cols[0] : nullptr, key_nullmaps ? key_nullmaps[0] : nullptr,
                                       states, state_nullmaps, n);
    if (n <= 0) return n == 0 ? TFG_OK : fail(TFG_ERR_INVALID_ARG, "negative row count");
    if (int rc = set_device(a->ctx)) return rc;
    a->long_key = false;
    if (int rc = pack_keys(a, key_cols, key_offsets, key_nullmaps, n)) {
        if (rc != TFG_ERR_NOT_IMPLEMENTED || !a->long_key) return rc;
        if ((rc = serial_adopt(a))) return rc;
        return serial_consume(a, key_cols, key_offsets, key_nullmaps, states, state_nullmaps, nullptr, n, true);
    }
    return tfg_agg_consume_partial(a, a->pack_buf, nullptr, states, state_nullmaps, n);
}

// tfg_agg_result_keys for one String key whose groups are still in their buckets (a tiled consume,
// no value stores): agg_result_str_keys_kernel.  With chars_capacity >= 16 * capacity every key
// fits and nothing is read before the write (one round trip at the end for the count and chars);
// otherwise the totals are read first and checked.
static int result_str_keys_fused(tfg_agg *a, uint8_t *out_chars, uint64_t *out_offsets, uint8_t *out_null,
                                 void *const *out_states, uint8_t *const *out_state_nullmaps, uint64_t capacity,
                                 uint64_t chars_capacity, uint64_t *out_groups_host, uint64_t *out_chars_host) {
    Ctx *ctx = a->ctx;
    const uint32_t B = a->B;
    if (int rc = set_device(ctx)) return rc;
    if (!a->pend_ch) TFG_HIP(hipMalloc(&a->pend_ch, (2 * (size_t)B + 1) * 8));
    if (out_groups_host) *out_groups_host = 0;
    if (out_chars_host) *out_chars_host = 0;
    if (a->pend_known && a->pend_total > capacity) {
        if (out_groups_host) *out_groups_host = a->pend_total;
        return fail(TFG_ERR_CAPACITY, "result needs %llu groups, capacity %llu", (unsigned long long)a->pend_total,
                    (unsigned long long)capacity);
    }
    if (!a->pend_known)
        if (int rc = pend_scan(a)) return rc;
    hipLaunchKernelGGL(pend_key_chars_kernel, dim3(B), dim3(RSK_T), 0, ctx->stream, (const uint4 *)a->pend.key,
                       (const uint64_t *)a->pend_cnt(), (const uint64_t *)a->pend_base(), a->pend_ch);
    TFG_LAUNCH_CHECK();
    void *sp;
    if (int rc = scratch_get(ctx, scan_tmp_bytes((int64_t)B + 1), &sp)) return rc;
    if (int rc = exclusive_scan_u64(ctx, a->pend_ch, a->pend_ch + B, (int64_t)B, sp)) return rc;
    const uint64_t *g_dev = a->pend_off() + B, *c_dev = a->pend_ch + 2 * (size_t)B;
    auto read_totals = [&](uint64_t &g, uint64_t &ch) -> int { // pinned words: one sync, no staging
        uint64_t *hp = ctx->host_pinned;
        TFG_HIP(hipMemcpyAsync(hp, g_dev, 16, hipMemcpyDeviceToHost, ctx->stream)); // count, kept rows
        TFG_HIP(hipMemcpyAsync(hp + 2, c_dev, 8, hipMemcpyDeviceToHost, ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
        g = hp[0];
        ch = hp[2];
        a->pend_total = g;
        a->kept_rows = hp[1];
        a->kept_n = a->consumed_n;
        a->pend_known = true;
        return TFG_OK;
    };
    uint64_t G = 0, chars = 0;
    if (chars_capacity < 16 * capacity) { // not every key fits for sure: the totals first
        if (int rc = read_totals(G, chars)) return rc;
        if (out_groups_host) *out_groups_host = G;
        if (out_chars_host) *out_chars_host = chars;
        if (G > capacity)
            return fail(TFG_ERR_CAPACITY, "result needs %llu groups, capacity %llu", (unsigned long long)G,
                        (unsigned long long)capacity);
        if (chars > chars_capacity)
            return fail(TFG_ERR_CAPACITY, "String keys need %llu bytes, capacity %llu", (unsigned long long)chars,
                        (unsigned long long)chars_capacity);
    }
    ResultPtrs rp{};
    for (int i = 0; i < a->S.n_aggs; ++i) {
        rp.state[i] = out_states ? out_states[i] : nullptr;
        rp.state_null[i] = out_state_nullmaps ? out_state_nullmaps[i] : nullptr;
        rp.nullable[i] = a->arg_nullable[i] || a->S.kind[i] == TFG_AGG_FIRST_ROW;
    }
    {
        ProfScope _ps(ctx, "agg.result");
        hipLaunchKernelGGL(agg_result_str_keys_kernel, dim3(B), dim3(RSK_T), 0, ctx->stream, a->S, a->pend,
                           (const uint64_t *)a->pend_cnt(), (const uint64_t *)a->pend_base(),
                           (const uint64_t *)a->pend_off(), (const uint64_t *)a->pend_ch + B, capacity, chars_capacity,
                           out_chars, out_offsets, out_null, rp);
    }
    TFG_LAUNCH_CHECK();
    if (int rc = read_totals(G, chars)) return rc; // the count and the chars in one round trip
    if (out_groups_host) *out_groups_host = G;
    if (out_chars_host) *out_chars_host = chars;
    if (G > capacity)
        return fail(TFG_ERR_CAPACITY, "result needs %llu groups, capacity %llu (the first %llu written)",
                    (unsigned long long)G, (unsigned long long)capacity, (unsigned long long)capacity);
    return TFG_OK;
}

int tfg_agg_result_keys(tfg_agg *a, void *const *out_key_cols, uint64_t *const *out_key_offsets,
                        uint8_t *const *out_key_nullmaps, void *const *out_states, uint8_t *const *out_state_nullmaps,
                        uint64_t capacity, uint64_t chars_capacity, uint64_t *out_groups_host, uint64_t *out_chars_host) {
    TFG_CHECK(a, TFG_ERR_INVALID_ARG, "agg is null");
    if (a->sdict) { // group ids from the inner aggregator, then their key tuples from the dictionary
        const uint64_t G = a->inner->n_groups;
        if (out_groups_host) *out_groups_host = G;
        if (out_chars_host) *out_chars_host = 0;
        if (G > capacity)
            return fail(TFG_ERR_CAPACITY, "result needs %llu groups, capacity %llu", (unsigned long long)G,
                        (unsigned long long)capacity);
        if (G == 0) return TFG_OK;
        if (int rc = set_device(a->ctx)) return rc;
        if (int rc = a->ensure_pack(G)) return rc;
        if (int rc = tfg_agg_result(a->inner, a->pack_buf, nullptr, out_states, out_state_nullmaps, capacity, nullptr))
            return rc;
        return serial_dict_unpack(a->sdict, (const uint32_t *)a->pack_buf, G, out_key_cols, out_key_offsets,
                                  out_key_nullmaps, chars_capacity, out_chars_host);
    }
    if (!a->kp.kind) {
        if (out_chars_host) *out_chars_host = 0;
        return tfg_agg_result(a, out_key_cols ? out_key_cols[0] : nullptr, out_key_nullmaps ? out_key_nullmaps[0] : nullptr,
                              out_states, out_state_nullmaps, capacity, out_groups_host);
    }
    if (a->pending && !a->has_ref && a->kp.kind == WK_STRING && capacity > 0) {
        TFG_CHECK(out_key_cols && out_key_cols[0] && out_key_offsets && out_key_offsets[0], TFG_ERR_INVALID_ARG,
                  "String result needs chars and offsets");
        return result_str_keys_fused(a, (uint8_t *)out_key_cols[0], out_key_offsets[0],
                                     out_key_nullmaps ? out_key_nullmaps[0] : nullptr, out_states, out_state_nullmaps,
                                     capacity, chars_capacity, out_groups_host, out_chars_host);
    }
    Ctx *ctx = a->ctx;
    // before the group count is read (tfg_agg_result's early path): packed keys, key lengths,
    // their scan and the unpack run over `capacity` slots with the count read on the device, and
    // one host round trip at the end reads the count and the chars total.  String keys need
    // 16 bytes of chars a slot for it (a packed String key holds <= 15 bytes + '\0')
    const bool early = result_early(a, capacity) && (a->kp.kind != WK_STRING || chars_capacity >= 16 * capacity);
    uint64_t G = 0;
    const uint64_t *g_dev = nullptr;
    if (early) {
        // the pending buffer holds at most pend_cap groups: a generous hint sizes nothing past it
        const uint64_t ecap = std::min<uint64_t>(capacity, a->pend_cap);
        if (int rc = set_device(ctx)) return rc;
        if (int rc = a->ensure_pack(ecap)) return rc;
        if (int rc = result_pending_launch(a, a->pack_buf, nullptr, out_states, out_state_nullmaps, ecap)) return rc;
        G = ecap;
        g_dev = a->pend_off() + a->B;
    } else {
        if (int rc = tfg_agg_size(a, &G)) return rc;
        if (out_groups_host) *out_groups_host = G;
        if (out_chars_host) *out_chars_host = 0;
        if (G > capacity)
            return fail(TFG_ERR_CAPACITY, "result needs %llu groups, capacity %llu", (unsigned long long)G,
                        (unsigned long long)capacity);
        if (G == 0) return TFG_OK;
        if (int rc = set_device(ctx)) return rc;
        if (int rc = a->ensure_pack(G)) return rc;
        if (int rc = tfg_agg_result(a, a->pack_buf, nullptr, out_states, out_state_nullmaps, capacity, nullptr))
            return rc;
    }
    KeyOut ko{};
    uint64_t *start = nullptr;
    bool chars_known = true;
    const unsigned grid = stream_grid((int64_t)G, 256, 4096);
    if (a->kp.kind == WK_STRING) {
        TFG_CHECK(out_key_cols && out_key_cols[0] && out_key_offsets && out_key_offsets[0], TFG_ERR_INVALID_ARG,
                  "String result needs chars and offsets");
        Carver cv;
        const size_t o_len = cv.take<uint64_t>(G), o_start = cv.take<uint64_t>(G + 1), o_tmp = cv.take<uint8_t>(scan_tmp_bytes(G));
        void *sp;
        if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
        uint64_t *len1 = (uint64_t *)((char *)sp + o_len);
        start = (uint64_t *)((char *)sp + o_start);
        hipLaunchKernelGGL(wide_str_len_kernel, dim3(grid), dim3(256), 0, ctx->stream, (const uint4 *)a->pack_buf, G, len1,
                           g_dev);
        TFG_LAUNCH_CHECK();
        if (int rc = exclusive_scan_u64(ctx, len1, start, (int64_t)G, (char *)sp + o_tmp)) return rc;
        // a packed String key holds <= 15 bytes + '\0': with room for 16 a group the capacity needs
        // no check, and the total is read after the unpack is queued (no idle gap before it)
        chars_known = !early && chars_capacity < 16 * G;
        if (chars_known) {
            uint64_t chars = 0;
            if (int rc = read_back_u64(ctx, start + G, &chars, 1)) return rc;
            if (out_chars_host) *out_chars_host = chars;
            if (chars > chars_capacity)
                return fail(TFG_ERR_CAPACITY, "String keys need %llu bytes, capacity %llu", (unsigned long long)chars,
                            (unsigned long long)chars_capacity);
        }
        ko.offsets = out_key_offsets[0];
    }
    for (int j = 0; j < a->kp.nkeys; ++j) {
        ko.col[j] = out_key_cols ? out_key_cols[j] : nullptr;
        ko.nullmap[j] = out_key_nullmaps ? out_key_nullmaps[j] : nullptr;
    }
    {
        ProfScope _ps(ctx, "agg.unpack_keys");
        hipLaunchKernelGGL(unpack_keys_kernel, dim3(grid), dim3(256), 0, ctx->stream, a->kp,
                           (const uint4 *)a->pack_buf, (const uint64_t *)start, G, ko, g_dev);
    }
    TFG_LAUNCH_CHECK();
    if (early) { // the count and the chars total in one round trip
        uint64_t *hp = ctx->host_pinned; // pinned words: one sync, no staging
        TFG_HIP(hipMemcpyAsync(hp, g_dev, 16, hipMemcpyDeviceToHost, ctx->stream)); // count, kept rows
        hp[2] = 0;
        if (start) TFG_HIP(hipMemcpyAsync(hp + 2, start + G, 8, hipMemcpyDeviceToHost, ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
        const uint64_t cnt = hp[0], chars = hp[2];
        a->pend_total = cnt;
        a->kept_rows = hp[1];
        a->kept_n = a->consumed_n;
        a->pend_known = true;
        if (out_groups_host) *out_groups_host = cnt;
        if (out_chars_host) *out_chars_host = chars;
        if (cnt > capacity)
            return fail(TFG_ERR_CAPACITY, "result needs %llu groups, capacity %llu (the first %llu written)",
                        (unsigned long long)cnt, (unsigned long long)capacity, (unsigned long long)capacity);
        return TFG_OK;
    }
    if (!chars_known && out_chars_host)
        if (int rc = read_back_u64(ctx, start + G, out_chars_host, 1)) return rc;
    return TFG_OK;
}

} // extern "C"
