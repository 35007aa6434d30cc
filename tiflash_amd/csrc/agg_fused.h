// agg_fused.h — the fused filter -> GROUP BY kernel (agg_fused.hip) as seen by agg.hip.
#pragma once
#include "partition.h"

namespace tfg {

// Device outputs of one fused consume: every bucket's groups (u64 key, key-null flag, the sum
// state, the count state) at tmp_base[b] .. + out_cnt[b] of the tmp arrays, and the rows that
// found their bucket's LDS table full (spill keys / values, *spill_count_host of them).
struct FusedIO {
    uint64_t *tmp_key;
    uint8_t *tmp_key_null;
    uint64_t *tmp_sum;  // sum state (Int64 / UInt64 / Float64 bits); null when the signature has none
    uint64_t *tmp_cnt;  // count state; null when the signature has none
    uint64_t *out_cnt;  // [buckets]
    uint64_t *tmp_base; // [buckets]
    uint64_t *spill_key;
    uint64_t *spill_val;
};

constexpr int FUSED_BUCKETS = 256;    // one bucket (and one workgroup) per CU
constexpr int FUSED_TABLE_CAP = 5632; // LDS table cells per bucket
constexpr int FUSED_MAXFILL = FUSED_TABLE_CAP * 4 / 5;
constexpr int64_t FUSED_MIN_ROWS = (int64_t)1 << 22;

// Scratch bytes the fused consume of n rows needs beyond the FusedIO arrays.
size_t fused_scratch_bytes();
// Runs the fused kernel for the fast signatures (one 8-byte key without NULLs, one sum over
// Int64 / UInt64 / Float64 and / or count, codes 310 210 300 200 130 120 of fast_signature) when
// the device can hold one 1024-thread workgroup per CU on FUSED_BUCKETS CUs.  *launched = false
// (and nothing enqueued) when it does not apply.  scratch: fused_scratch_bytes() bytes.
int agg_fused_consume(Ctx *ctx, int code, const RowPred &pred, const void *keys, const void *vals, int64_t n,
                      const FusedIO &io, void *scratch, uint64_t *spill_count_host, bool &launched);

} // namespace tfg
