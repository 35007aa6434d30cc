/*
 * tiflash_amd.h — C-ABI drop-in boundary of the MI355X (gfx950) execution layer for
 * TiFlash's Block/Column hot path: filter / compare, arithmetic, hash GROUP BY (Aggregator),
 * hash join build + probe, and the ExchangeSender hash repartition.
 *
 * Conventions (plain C, no exceptions across the ABI, no torch types):
 *   - Every entry point returns an int status: TFG_OK (0) or a negative TFG_ERR_* code.
 *     tfg_last_error() returns a thread-local message for the last failure.  The codes mirror
 *     the reference's DB::ErrorCodes used on this path (SIZES_OF_COLUMNS_DOESNT_MATCH,
 *     ILLEGAL_TYPE_OF_COLUMN_FOR_FILTER, LOGICAL_ERROR, ...).
 *   - Column pointers are DEVICE pointers (HBM) laid out like the reference's PaddedPODArray
 *     payload: `n` contiguous values of the column's native width.  Null maps are UInt8,
 *     nonzero = NULL (ColumnNullable, dbms/src/Columns/ColumnNullable.h:37).  Filters are UInt8,
 *     nonzero = keep (dbms/src/Columns/ColumnUtil.cpp:32-79).
 *   - Work is enqueued on the context's HIP stream.  Functions that return a count to the host
 *     (out_*_host arguments) synchronise that stream; the device-side count is always written
 *     too, so callers that stay on the device never block.
 *   - Inputs are never modified (COW ColumnPtr semantics of IColumn::filter et al.,
 *     dbms/src/Columns/IColumn.h:426); every operation writes caller-provided outputs.
 *
 * Each entry point names the reference interface it replaces (paths relative to
 * /root/reference/dbms/src).
 */
#ifndef TIFLASH_AMD_H
#define TIFLASH_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- status codes */
#define TFG_OK 0
#define TFG_ERR_INVALID_ARG (-1)        /* BAD_ARGUMENTS */
#define TFG_ERR_HIP (-2)                /* runtime failure reported by HIP */
#define TFG_ERR_OOM (-3)                /* device allocation failed */
#define TFG_ERR_NOT_IMPLEMENTED (-4)    /* type / op combination not supported */
#define TFG_ERR_SIZE_MISMATCH (-5)      /* SIZES_OF_COLUMNS_DOESNT_MATCH */
#define TFG_ERR_ILLEGAL_TYPE (-6)       /* ILLEGAL_TYPE_OF_ARGUMENT / ..._FOR_FILTER */
#define TFG_ERR_LOGICAL (-7)            /* LOGICAL_ERROR */
#define TFG_ERR_CAPACITY (-8)           /* output buffer too small (caller retries larger) */
#define TFG_ERR_NO_DEVICE (-9)          /* no HIP device visible */
#define TFG_ERR_FAULT_INJECTED (-10)    /* test-only failpoint (TFG_FAILPOINT env var) */
#define TFG_ERR_OVERFLOW (-11)          /* DECIMAL_OVERFLOW ("Decimal math overflow") */

/* ---------------------------------------------------------------- column types */
/* Native fixed-width column payloads (ColumnVector<T> / ColumnDecimal<T>). Decimal columns
 * carry their scale separately; values are the scaled integers (Decimal<T>{T value},
 * dbms/src/Common/Decimal.h:209). */
typedef enum tfg_type {
    TFG_INT8 = 1,
    TFG_INT16 = 2,
    TFG_INT32 = 3,
    TFG_INT64 = 4,
    TFG_UINT8 = 5,
    TFG_UINT16 = 6,
    TFG_UINT32 = 7,
    TFG_UINT64 = 8,
    TFG_FLOAT32 = 9,
    TFG_FLOAT64 = 10,
    TFG_DECIMAL32 = 11,  /* Int32 payload  (precision <= 9)  */
    TFG_DECIMAL64 = 12,  /* Int64 payload  (precision <= 18) */
    TFG_DECIMAL128 = 13, /* Int128 payload (precision <= 38), little-endian two's complement */
    TFG_DECIMAL256 = 14, /* 256-bit payload (precision <= 65), four little-endian 64-bit limbs, two's
                          * complement: the reference's Decimal256 (boost checked_int256_t,
                          * libs/libcommon/include/common/types.h:35) as a fixed-width value; sum
                          * results, sum / min / max / first_row arguments */
    TFG_STRING = 20,     /* ColumnString: chars (every row ends with '\0') + UInt64 end offsets
                          * (Columns/ColumnString.h:50-54); GROUP BY keys and min / max / first_row
                          * arguments */
    TFG_KEYS128 = 21,    /* a packed 16-byte GROUP BY key (see tfg_agg_create_keys): the device
                          * form the keys128 / key_string methods aggregate on, and the form
                          * partial results travel in between the two phases of an aggregation */
} tfg_type;

/* Comparison ops (dbms/src/Functions/FunctionsComparison.h, accurate:: semantics of
 * dbms/src/Core/AccurateComparison.h:33-159). */
typedef enum tfg_cmp_op {
    TFG_EQ = 0,
    TFG_NE = 1,
    TFG_LT = 2,
    TFG_LE = 3,
    TFG_GT = 4,
    TFG_GE = 5,
} tfg_cmp_op;

/* Binary arithmetic (dbms/src/Functions/FunctionBinaryArithmetic.h). */
typedef enum tfg_arith_op {
    TFG_PLUS = 0,
    TFG_MINUS = 1,
    TFG_MULTIPLY = 2,
} tfg_arith_op;

/* Logical combination of UInt8 masks (dbms/src/Functions/FunctionsLogical.cpp). */
typedef enum tfg_logic_op {
    TFG_AND = 0,
    TFG_OR = 1,
    TFG_NOT = 2, /* unary: b ignored */
} tfg_logic_op;

/* Aggregate functions on the path (dbms/src/AggregateFunctions/AggregateFunctionSum.h,
 * AggregateFunctionCount.h).  Result types follow the reference factory
 * (AggregateFunctionSum.cpp:31-120): sum(Int*) -> Int64, sum(UInt*) -> UInt64,
 * sum(Float*) -> Float64, sum(Decimal(p,s)) -> Decimal(min(p+22,65), s) (SumDecimalInferer,
 * Common/Decimal.h:156-163): Decimal128 when p+22 <= 38 (Decimal32 / Decimal64 with p <= 16),
 * else Decimal256 (Decimal64 with p >= 17, every Decimal128 / Decimal256 argument);
 * count -> UInt64.
 *
 * An aggregate argument type word is the tfg_type, optionally or-ed with TFG_ARG_NULLABLE (the
 * argument carries a null map) and, for Decimal arguments, TFG_ARG_PREC(p): the column's
 * DataTypeDecimal precision (0 = the type's maximum, 9 / 18 / 38 / 65).  Decimal256 sums are
 * exact and checked like the reference's checked_int256_t (libs/libcommon/include/common/types.h:35):
 * the device keeps a fifth limb, and a consume or merge whose exact sum leaves Int256 returns
 * TFG_ERR_OVERFLOW. */
#define TFG_ARG_NULLABLE 0x100
#define TFG_ARG_PREC(p) ((int)(p) << 16)
#define TFG_ARG_TYPE(w) ((w) & 0xFF)
#define TFG_ARG_PREC_OF(w) (((w) >> 16) & 0xFF)
/* the collator of a String min / max argument (SingleValueDataString::setCollators,
 * AggregateFunctionMinMaxAny.h:272-275): a tfg_collator */
#define TFG_ARG_COLLATOR(c) ((int)(c) << 24)
#define TFG_ARG_COLLATOR_OF(w) (((w) >> 24) & 0x7F)
typedef enum tfg_agg_kind {
    TFG_AGG_SUM = 0,
    TFG_AGG_COUNT = 1,     /* count(arg): non-NULL rows of arg */
    TFG_AGG_COUNT_ALL = 2, /* count(*) / count(1): arg ignored */
    /* min / max / first_row (AggregateFunctionMinMaxAny.cpp:39-46,85-98,155-159; SingleValueDataFixed /
     * SingleValueDataString, AggregateFunctionMinMaxAny.h:40-456): every argument type on the path —
     * Int*, UInt*, Float*, Decimal32..Decimal256 and String; the result has the argument's type.
     *   min / max: NULL arguments are skipped (AggregateFunctionNullUnary); a group whose argument is
     *     NULL in every row yields NULL (Nullable result), without key and without rows the type's
     *     default (non-Nullable argument: SingleValueDataFixed::insertResultInto -> insertDefault).
     *     Numeric arguments keep an order key (Float order is IEEE total order: -0 < +0, NaN past
     *     +inf, where the reference's `<` leaves ties and NaN to row order).  Decimal128 / Decimal256
     *     compare as signed integers; String compares as SingleValueDataString::less / greater do:
     *     the collator's compareFastPath over the row INCLUDING its terminating '\0'
     *     (getDataAtWithTerminatingZero), so padding collators do not trim; without a collator, bytes.
     *     Of equal values (equal under the collator) the first row in input order is kept
     *     (changeIfLess / changeIfGreater are strict).
     *   first_row: the first row in input order (changeFirstTime), NULL included: a NULL first row
     *     makes the result NULL and later rows do not replace it (AggregateFunctionFirstRowNull,
     *     AggregateFunctionNull.h:193-330); without rows the result is NULL.
     *   "Input order" is the order of the rows of one consume, consumes in call order, and for
     *   tfg_agg_merge the destination's groups before the source's — the reference's answer with one
     *   thread (its multi-threaded answer depends on thread scheduling and merge order).
     * String arguments: the args[i] / states[i] entry of the consume calls is a HOST pointer to a
     * tfg_str_col, and the out_states[i] entry of the result calls a HOST pointer to a tfg_str_out
     * (tfg_agg_result_type reports TFG_STRING, width 8: the end offsets). */
    TFG_AGG_MIN = 3,
    TFG_AGG_MAX = 4,
    TFG_AGG_FIRST_ROW = 5,
} tfg_agg_kind;
/* A String column argument / partial state (ColumnString: chars, each row ending in '\0', and
 * UInt64 end offsets), DEVICE pointers in a host struct. */
typedef struct tfg_str_col {
    const uint8_t *chars;
    const uint64_t *offsets;
} tfg_str_col;
/* A String result column: DEVICE buffers for the end offsets (one per group) and the chars
 * (chars_capacity bytes; tfg_agg_result_chars gives the bytes needed). */
typedef struct tfg_str_out {
    uint8_t *chars;
    uint64_t *offsets;
    uint64_t chars_capacity;
} tfg_str_out;

/* Join kinds (ASTTableJoin::Kind, dbms/src/Interpreters/Join.h). Strictness ALL. */
typedef enum tfg_join_kind {
    TFG_JOIN_INNER = 0,
    TFG_JOIN_LEFT = 1,  /* unmatched probe rows emit build index -1 (default / NULL row) */
    TFG_JOIN_SEMI = 2,  /* probe rows with at least one match, once */
    TFG_JOIN_ANTI = 3,  /* probe rows with no match (NULL keys count as no match) */
} tfg_join_kind;

/* String collators relevant to partition hashing (dbms/src/TiDB/Collation/Collator.h). */
typedef enum tfg_collator {
    TFG_COLLATOR_NONE = 0,        /* raw bytes                                       */
    TFG_COLLATOR_BINARY = 1,      /* BinCollatorSortKey<false>: raw bytes            */
    TFG_COLLATOR_BIN_PADDING = 2, /* BinCollatorSortKey<true>: right-trim ' ' (utf8mb4_bin etc.) */
    TFG_COLLATOR_GENERAL_CI = 3,  /* GeneralCICollator (utf8_general_ci / utf8mb4_general_ci): right-trim ' ',
                                     then each UTF-8 character's 16-bit weight big-endian
                                     (TiDB/Collation/Collator.cpp:416-455) */
    TFG_COLLATOR_UNICODE_CI = 4,  /* UCACICollator<Unicode0400, padding> (utf8_unicode_ci / utf8mb4_unicode_ci):
                                     right-trim ' ', then each non-ignorable character's UCA 4.0.0
                                     weights as 16-bit big-endian chunks (Collator.cpp:580-629) */
    TFG_COLLATOR_UCA0900_AI_CI = 5, /* UCACICollator<Unicode0900, no padding> (utf8mb4_0900_ai_ci): the same with
                                       the UCA 9.0.0 weights and no trim */
} tfg_collator;

/* ---------------------------------------------------------------- context & memory */
typedef struct tfg_ctx tfg_ctx;

/* Creates a context bound to HIP device `device` and stream `stream` (a hipStream_t; NULL =
 * the null stream).  The context owns a growable device scratch arena. */
int tfg_ctx_create(int device, void *stream, tfg_ctx **out);
int tfg_ctx_destroy(tfg_ctx *ctx);
int tfg_ctx_set_stream(tfg_ctx *ctx, void *stream);
int tfg_ctx_sync(tfg_ctx *ctx);
/* Pre-sizes the scratch arena so later calls never allocate (and can be graph-captured). */
int tfg_ctx_reserve(tfg_ctx *ctx, size_t bytes);
const char *tfg_last_error(void);
const char *tfg_version(void);
int tfg_device_count(int *out);

/* Kernel profiler: when enabled, every kernel phase is bracketed by HIP events recorded on the
 * context stream (the stream the kernels run on); totals accumulate per phase name
 * (e.g. "agg.bucket", "part.scatter").  tfg_profile_read syncs the stream and returns phase
 * `index` (TFG_ERR_INVALID_ARG past the last one).  Replaces the reference's per-operator
 * stopwatches (DataStreams/BlockStreamProfileInfo.h:36-60, Operators/OperatorProfileInfo.h:27-59). */
int tfg_profile_enable(tfg_ctx *ctx, int on);
int tfg_profile_reset(tfg_ctx *ctx);
int tfg_profile_read(tfg_ctx *ctx, int index, char *name, size_t name_len, double *total_ms, uint64_t *count);

int tfg_buf_alloc(tfg_ctx *ctx, size_t bytes, void **out_dev);
int tfg_buf_free(tfg_ctx *ctx, void *dev);
int tfg_upload(tfg_ctx *ctx, void *dst_dev, const void *src_host, size_t bytes);
int tfg_download(tfg_ctx *ctx, void *dst_host, const void *src_dev, size_t bytes);
/* Device-to-device copy, asynchronous on the context's stream (column concatenation / COW copies). */
int tfg_copy(tfg_ctx *ctx, void *dst_dev, const void *src_dev, size_t bytes);
/* Device memset on the context's stream (asynchronous): `bytes` bytes of dst_dev set to `value`
 * (e.g. a received column's null map before the slices that carry one land in it). */
int tfg_memset(tfg_ctx *ctx, void *dst_dev, int value, size_t bytes);

/* Size in bytes of one value of `type`, 0 if unknown. */
size_t tfg_type_width(int type);

/* ---------------------------------------------------------------- a1/a2 comparison */
/* out_mask[i] = Op(col[i], scalar) as 0/1.  Replaces NumComparisonImpl::vectorConstant
 * (Functions/FunctionsComparison.h:101-114) reached from FunctionComparison::executeImpl
 * (:1388-1440).  `scalar_host` points to one host value of `scalar_type`.  A NULL input row
 * (col_nullmap[i] != 0) yields 0, i.e. the Nullable(UInt8) result already folded the way
 * FilterDescription does (Columns/FilterDescription.cpp:68-108). */
int tfg_cmp_const(tfg_ctx *ctx, int col_type, const void *col, const uint8_t *col_nullmap, int64_t n,
                  int op, int scalar_type, const void *scalar_host, uint8_t *out_mask);
/* Constant on the left: out[i] = Op(scalar, col[i]) (NumComparisonImpl::constantVector). */
int tfg_cmp_const_left(tfg_ctx *ctx, int scalar_type, const void *scalar_host, int op, int col_type,
                       const void *col, const uint8_t *col_nullmap, int64_t n, uint8_t *out_mask);
/* out_mask[i] = Op(a[i], b[i]) (NumComparisonImpl::vectorVector, :78-99). */
int tfg_cmp_vector(tfg_ctx *ctx, int a_type, const void *a, const uint8_t *a_nullmap, int op, int b_type,
                   const void *b, const uint8_t *b_nullmap, int64_t n, uint8_t *out_mask);
/* and / or / not over UInt8 masks (Functions/FunctionsLogical.cpp); any nonzero is true. */
int tfg_mask_logic(tfg_ctx *ctx, int op, const uint8_t *a, const uint8_t *b, int64_t n, uint8_t *out_mask);

/* ---------------------------------------------------------------- a3 arithmetic */
/* out[i] = a[i] op b[i] (FunctionBinaryArithmetic.h:761-1200, DecimalBinaryOperation :231-500).
 * Either side may be a constant (`*_is_const` != 0: the pointer is a HOST pointer to one value).
 * Decimal operands are aligned to the result scale for +/- (applyScaled) and multiplied raw for
 * * (result scale = a_scale + b_scale, MulDecimalInferer, Common/Decimal.h:109-163); a multiply
 * whose result scale is capped below a_scale + b_scale (decimal_max_scale 30) divides the product
 * by 10^(a_scale + b_scale - res_scale), truncating (DataTypeDecimal::getScales).
 * Integer results wrap like the reference's native ops; Decimal128 results are exact Int128.
 * Decimal256 results / operands: exact 256-bit values (computed in 512 bits, PromoteType<Int256>);
 * TFG_ERR_OVERFLOW when a value does not fit Int256, or when a Decimal256 operand's result
 * exceeds 10^65 - 1 (DecimalBinaryOperation::check_overflow, FunctionBinaryArithmetic.h:250-252). */
int tfg_arith(tfg_ctx *ctx, int op, int a_type, const void *a, int a_is_const, int a_scale, int b_type,
              const void *b, int b_is_const, int b_scale, int res_type, int res_scale, int64_t n, void *out);

/* ---------------------------------------------------------------- a5-a8 filter */
/* Number of nonzero bytes (countBytesInFilter, Columns/countBytesInFilter.cpp:32-124); with a
 * null map: rows with f != 0 && !null (countBytesInFilterWithNull). */
int tfg_count_mask(tfg_ctx *ctx, const uint8_t *mask, const uint8_t *nullmap, int64_t n,
                   uint64_t *out_count_dev, uint64_t *out_count_host);
/* Stable compaction of `ncols` fixed-width columns by one filter (ColumnVector<T>::filter ->
 * filterImpl, Columns/ColumnVector.cpp:659-683, Columns/filterColumn.cpp:174-305: output order =
 * input order).  widths[j] in {1,2,4,8,16}.  outs[j] must hold count values. */
int tfg_filter(tfg_ctx *ctx, const uint8_t *mask, int64_t n, int ncols, const void *const *cols,
               const int *widths, void *const *outs, uint64_t *out_count_dev, uint64_t *out_count_host);
/* Fused FilterTransformAction::transform (DataStreams/FilterTransformAction.cpp:72-173) for the
 * predicate `pred_col Op scalar`: the mask is never materialised. */
int tfg_filter_cmp_const(tfg_ctx *ctx, int pred_type, const void *pred_col, const uint8_t *pred_nullmap, int op,
                         int scalar_type, const void *scalar_host, int64_t n, int ncols, const void *const *cols,
                         const int *widths, void *const *outs, uint64_t *out_count_dev, uint64_t *out_count_host);
/* String column compaction (filterArraysImplGeneric, Columns/filterColumn.cpp:97-171):
 * ColumnString layout = chars (each row ends with '\0') + UInt64 end offsets
 * (Columns/ColumnString.h:50-54).  out_chars must hold the kept rows' bytes. */
int tfg_filter_string(tfg_ctx *ctx, const uint8_t *mask, int64_t n, const uint8_t *chars, const uint64_t *offsets,
                      uint8_t *out_chars, uint64_t *out_offsets, uint64_t *out_rows_host, uint64_t *out_bytes_host);

/* ---------------------------------------------------------------- a22-a24 hash / partition */
/* Seeds h[i] = 0xFFFFFFFF (WeakHash32::initial_hash = ~0u, Common/WeakHash.h:33). */
int tfg_weak_hash_init(tfg_ctx *ctx, uint32_t *h, int64_t n);
/* h[i] = CRC32-C(h[i], value_i) exactly like IColumn::updateWeakHash32 for fixed-width columns
 * (Columns/ColumnVector.cpp:499-535, ColumnDecimal.cpp:658, Common/HashTable/Hash.h:70-145):
 * integers are converted to UInt64 by C++ implicit conversion (signed types sign-extend),
 * Decimal128 hashes its two 64-bit limbs low then high.  NULL rows keep the previous h
 * (ColumnNullable.cpp:131-173).  Float32 / Float64 convert to UInt64 as the reference's x86-64
 * build does (clang, SSE4.2: cvttsd2si pair; NaN / out of range -> 0x8000000000000000, negative
 * values wrap), pinned by tests/golden/float_weak_hash.json. */
int tfg_weak_hash_update(tfg_ctx *ctx, int type, const void *col, const uint8_t *nullmap, int64_t n, uint32_t *h);
/* BlockInfo::selective (Core/BlockInfo.h:47-49; ColumnVector.cpp:500-535): h has n entries and
 * h[i] hashes row selective[i] (a DEVICE array of n UInt64 row ids); selective NULL = every row. */
int tfg_weak_hash_update_selective(tfg_ctx *ctx, int type, const void *col, const uint8_t *nullmap,
                                   const uint64_t *selective, int64_t n, uint32_t *h);
/* String keys (ColumnString::updateWeakHash32, Columns/ColumnString.cpp:1228-1327 with
 * ::updateWeakHash32(bytes), Common/HashTable/Hash.h:148-214). */
int tfg_weak_hash_update_string(tfg_ctx *ctx, const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                                int64_t n, int collator, uint32_t *h);
/* ColumnString::updateWeakHash32 over selective rows (ColumnString.cpp:1256-1294). */
int tfg_weak_hash_update_string_selective(tfg_ctx *ctx, const uint8_t *chars, const uint64_t *offsets,
                                          const uint8_t *nullmap, const uint64_t *selective, int64_t n, int collator,
                                          uint32_t *h);
/* out_perm[i] = selective[perm[i]] (perm NULL: selective[i]): a tfg_partition permutation of the
 * selective rows mapped back to block rows, for tfg_gather (IColumn::scatter with a selective,
 * IColumn.h:678-721). */
int tfg_selective_perm(tfg_ctx *ctx, const uint64_t *selective, const uint32_t *perm, int64_t n, uint32_t *out_perm);
/* selector[i] = (UInt64(h[i]) * part_num) >> 32 (fillSelector, Flash/Mpp/HashBaseWriterHelper.cpp:46-62);
 * with fine_grained_stream_count > 0: selector = part * S + h % S (fillSelectorForFineGrainedShuffle, :64-84). */
int tfg_fill_selector(tfg_ctx *ctx, const uint32_t *h, int64_t n, uint32_t part_num,
                      uint32_t fine_grained_stream_count, uint32_t *out_selector);
/* Stable counting partition of rows by selector (the permutation behind IColumn::scatter,
 * Columns/IColumn.h:655-721): out_perm lists row ids partition by partition, each partition
 * in input row order; out_offsets[p] = first slot of partition p, out_offsets[P] = n.
 * out_offsets is a DEVICE array of P+1 uint64; out_offsets_host (optional) receives a copy. */
int tfg_partition(tfg_ctx *ctx, const uint32_t *selector, int64_t n, uint32_t num_parts, uint32_t *out_perm,
                  uint64_t *out_offsets, uint64_t *out_offsets_host);
/* out_j[r] = col_j[perm[r]] for r < n (gather); used for scatter after tfg_partition and to
 * materialise join results.  perm entries of 0xFFFFFFFF (-1) write a zero / default value. */
int tfg_gather(tfg_ctx *ctx, const uint32_t *perm, int64_t n, int ncols, const void *const *cols, const int *widths,
               void *const *outs);
/* String gather (ColumnString::insertFrom per joined row, Interpreters/JoinPartition.cpp:1290-1378;
 * replicate of a String probe column): row r of the output is row perm[r] of (chars, offsets);
 * perm 0xFFFFFFFF writes the default (empty) String.  Writes the n end offsets, then the chars
 * when out_chars is non-NULL and they fit in chars_capacity (else TFG_ERR_CAPACITY);
 * *out_chars_host = the output chars bytes (terminators included).  Synchronises. */
int tfg_gather_string(tfg_ctx *ctx, const uint32_t *perm, int64_t n, const uint8_t *chars, const uint64_t *offsets,
                      uint64_t *out_offsets, uint8_t *out_chars, uint64_t chars_capacity, uint64_t *out_chars_host);
/* One-call HashBaseWriterHelper::scatterColumns (HashBaseWriterHelper.cpp:144-172) for
 * fixed-width key columns: weak hash over key_cols -> fillSelector(part_num) -> stable
 * partition -> gather of all `ncols` columns into outs (partition-major).  */
int tfg_hash_partition(tfg_ctx *ctx, int64_t n, int nkeys, const int *key_col_idx, int ncols, const int *types,
                       const void *const *cols, const uint8_t *const *nullmaps, uint32_t part_num,
                       void *const *outs, uint64_t *out_offsets, uint64_t *out_offsets_host);

/* ---------------------------------------------------------------- a9-a17 aggregation */
typedef struct tfg_agg tfg_agg;

typedef struct tfg_agg_params {
    /* log2 of the number of radix buckets rows are partitioned into before the LDS-table pass
     * (the GPU analogue of TwoLevelHashTable's 256 buckets, Common/HashTable/TwoLevelHashTable.h:47-71).
     * 0 = choose from expected_groups. */
    int bucket_bits;
    /* hint for the number of distinct keys (0 = unknown: 2^20 assumed). */
    int64_t expected_groups;
} tfg_agg_params;

/* Aggregator with one fixed-width GROUP BY key (method key8..key64 / nullable, Interpreters/
 * Aggregator.cpp:394-537) or no key (key_type = 0: a single group, without_key).
 * arg_types[i] / arg_scales[i] describe the argument of agg i (ignored for COUNT_ALL). */
int tfg_agg_create(tfg_ctx *ctx, int key_type, int n_aggs, const int *agg_kinds, const int *arg_types,
                   const int *arg_scales, const tfg_agg_params *params, tfg_agg **out);
int tfg_agg_destroy(tfg_agg *agg);
/* Drops every group but keeps the device allocations (a new query on the same signature). */
int tfg_agg_reset(tfg_agg *agg);
/* Aggregator::executeOnBlock (Interpreters/Aggregator.cpp:1127-1246): folds n rows into the
 * state.  `mask` (optional) is a UInt8 filter applied first (rows with 0 are skipped). */
int tfg_agg_consume(tfg_agg *agg, const void *keys, const uint8_t *key_nullmap, const void *const *args,
                    const uint8_t *const *arg_nullmaps, const uint8_t *mask, int64_t n);
/* Fused Filter -> Aggregator: rows with pred_col Op scalar are aggregated (mask never built). */
int tfg_agg_consume_filtered(tfg_agg *agg, int pred_type, const void *pred_col, const uint8_t *pred_nullmap, int op,
                             int scalar_type, const void *scalar_host, const void *keys, const uint8_t *key_nullmap,
                             const void *const *args, const uint8_t *const *arg_nullmaps, int64_t n);
/* Merge partial states (mergeDataImpl / two-phase final agg, Aggregator.cpp:2338-2505):
 * rows are (key, partial state) as produced by tfg_agg_result of the same agg signature. */
int tfg_agg_consume_partial(tfg_agg *agg, const void *keys, const uint8_t *key_nullmap, const void *const *states,
                            const uint8_t *const *state_nullmaps, int64_t n);
int tfg_agg_merge(tfg_agg *dst, tfg_agg *src);
/* Number of groups so far (syncs). */
int tfg_agg_size(tfg_agg *agg, uint64_t *out_groups);
/* convertToBlockImplFinal (Aggregator.cpp:1651-1780): writes every group.  out_keys: key type
 * width per group; out_key_nullmap (optional, nullable keys); out_states[i]: result type
 * width (8 B for Int64/UInt64/Float64 sums and counts, 16 B for Decimal128 sums, 32 B for
 * Decimal256 sums);
 * out_state_nullmaps[i] (optional): 1 when sum saw no non-NULL value (AggregateFunctionNull).
 * Order is the table's (compare unordered, as the reference tests do).
 * *out_groups_host = the group count; more than `capacity` -> TFG_ERR_CAPACITY.  When the count
 * is not known yet (the groups of a tiled consume, no tfg_agg_size since, no first_row / wide
 * min / max aggregate) the groups are written first and the count read after them: the first
 * `capacity` groups are written even when TFG_ERR_CAPACITY is returned, so a caller may pass a
 * capacity hint (e.g. the previous call's count) and retry with the reported count. */
int tfg_agg_result(tfg_agg *agg, void *out_keys, uint8_t *out_key_nullmap, void *const *out_states,
                   uint8_t *const *out_state_nullmaps, uint64_t capacity, uint64_t *out_groups_host);
/* Several GROUP BY keys, one String key or one 16-byte key (Aggregator::chooseAggregationMethod,
 * Interpreters/Aggregator.cpp:394-537):
 *   - fixed-width keys whose widths sum to <= 16 bytes take keys128 / nullable_keys128 (packFixed,
 *     Common/ColumnsHashing.h:324-480; nullable keys use byte 15 for their NULL bits);
 *   - one String key takes key_string (HashMethodString, ColumnsHashing.h:179-241): rows group by
 *     the collator's sort key (key_collators[j]: tfg_collator; BIN_PADDING right-trims spaces);
 *   - everything else takes the serialized method (HashMethodSerialized, ColumnsHashing.h:578-629):
 *     String keys with other keys, fixed tuples past 16 bytes (keys256), 5-8 keys.  Each row's key
 *     tuple is serialised (a NULL byte per key, the value bytes, a String's length + sort key) and
 *     a device dictionary maps equal byte strings to one group; fingerprint collisions are caught
 *     by a byte compare and retried with another seed, never merged.
 * keys128 / key_string aggregate on a packed 16-byte key (TFG_KEYS128).  A block whose keys do not
 * fit it (a String sort key over 15 bytes; nullable fixed keys of 16 bytes, nullable_keys256)
 * moves the aggregator to the serialized method, carrying the groups it holds; from then on it has
 * no packed form (tfg_agg_result / tfg_agg_consume_partial return TFG_ERR_NOT_IMPLEMENTED; use the
 * *_keys calls).  One fixed key of <= 8 bytes falls back to tfg_agg_create.  key_collators may
 * be NULL. */
int tfg_agg_create_keys(tfg_ctx *ctx, int nkeys, const int *key_types, const int *key_collators, int n_aggs,
                        const int *agg_kinds, const int *arg_types, const int *arg_scales, const tfg_agg_params *params,
                        tfg_agg **out);
/* executeOnBlock over the key columns of tfg_agg_create_keys: key_cols[j] is the data (String:
 * chars) of key j, key_offsets[j] the String key's end offsets (NULL for fixed keys),
 * key_nullmaps (optional) their null maps. */
int tfg_agg_consume_keys(tfg_agg *agg, const void *const *key_cols, const uint64_t *const *key_offsets,
                         const uint8_t *const *key_nullmaps, const void *const *args, const uint8_t *const *arg_nullmaps,
                         const uint8_t *mask, int64_t n);
/* Two-phase final aggregation over partial (key columns, states) rows (mergeOnBlock). */
int tfg_agg_consume_partial_keys(tfg_agg *agg, const void *const *key_cols, const uint64_t *const *key_offsets,
                                 const uint8_t *const *key_nullmaps, const void *const *states,
                                 const uint8_t *const *state_nullmaps, int64_t n);
/* convertToBlockImplFinal with the key columns restored (String: chars + end offsets).  Every
 * String key column gets chars_capacity bytes; *out_chars_host = the chars the largest String key
 * column needs (TFG_ERR_CAPACITY past chars_capacity, nothing written).  tfg_agg_result on a
 * packed-key agg writes the packed TFG_KEYS128 keys instead, which tfg_agg_consume_partial accepts.
 * As tfg_agg_result, groups whose count is not known yet are written before it is read when
 * chars_capacity >= 16 * capacity (packed String keys hold at most 16 bytes with the '\0'): one
 * host round trip at the end returns the count and the chars; a count above `capacity` returns
 * TFG_ERR_CAPACITY after writing the first `capacity` groups. */
int tfg_agg_result_keys(tfg_agg *agg, void *const *out_key_cols, uint64_t *const *out_key_offsets,
                        uint8_t *const *out_key_nullmaps, void *const *out_states, uint8_t *const *out_state_nullmaps,
                        uint64_t capacity, uint64_t chars_capacity, uint64_t *out_groups_host, uint64_t *out_chars_host);
/* IColumn::updateWeakHash32 of the aggregator's key columns (Columns/ColumnString.cpp:1228-1327,
 * ColumnVector.cpp:483-535, ColumnNullable.cpp:131-173) computed from the packed TFG_KEYS128 keys
 * tfg_agg_result writes for a packed-key aggregator: h[i] is updated as the unpacked key columns
 * would update it (the two-phase sender routes its partial groups without unpacking them,
 * HashBaseWriterHelper.cpp:46-62).  TFG_ERR_NOT_IMPLEMENTED for an aggregator without packed keys
 * (the serialized method). */
int tfg_agg_weak_hash_packed(tfg_agg *agg, const void *packed_keys, int64_t n, uint32_t *h);
/* Result type of agg i (tfg_type) and its width in bytes. */
int tfg_agg_result_type(tfg_agg *agg, int i, int *out_type, int *out_width);
/* Chars bytes (terminators included) of the String result of agg i (min / max / first_row over a
 * String argument) as tfg_agg_result / tfg_agg_result_keys would write them now; 0 for other
 * aggregates. */
int tfg_agg_result_chars(tfg_agg *agg, int i, uint64_t *out_bytes);

/* ---------------------------------------------------------------- a18-a21 hash join */
typedef struct tfg_join tfg_join;

/* Join::insertFromBlock + finishOneBuild for one fixed-width key (Interpreters/Join.cpp:532-735,
 * JoinPartition.cpp:584-728).  Rows with a NULL key are not inserted.  Build may be called
 * repeatedly (blocks); build row ids continue across calls.  `expected_build_rows` sizes
 * the partitioning (0 = size from the first block). */
int tfg_join_create(tfg_ctx *ctx, int key_type, int64_t expected_build_rows, tfg_join **out);
int tfg_join_build(tfg_join *join, const void *keys, const uint8_t *key_nullmap, int64_t n);
/* JoinV2 (Interpreters/JoinV2/HashJoinPointerTable.{h,cpp}, §8 f3): the same build / finalize /
 * probe / probe_rows / destroy calls over a pointer table instead of radix partitions:
 * 2^d chain heads, d from pointerTableCapacity = max(pow2ceil(2 * build rows), 1024), bucket =
 * top d bits of the key's 64-bit hash, rows pushed on their chain by exchange; with
 * TFG_JOIN_V2_TAGGED each head also carries the OR of its rows' low 16 hash bits (tagged
 * pointer) so a probe skips chains that cannot hold its key.  Probing needs no partition pass.
 * Same results as tfg_join_create (unordered). */
#define TFG_JOIN_V2_TAGGED 1
int tfg_join_create_v2(tfg_ctx *ctx, int key_type, int64_t expected_build_rows, int flags, tfg_join **out);
int tfg_join_finalize(tfg_join *join);
int tfg_join_destroy(tfg_join *join);
/* Join::joinBlock (Join.cpp:1977 -> probeBlockImplTypeCase, JoinPartition.cpp:1465-1644):
 * emits (probe row, build row) index pairs.  LEFT emits build = 0xFFFFFFFF for unmatched rows;
 * SEMI/ANTI emit the probe row only (out_build_idx may be NULL).  If the result exceeds
 * `capacity`, TFG_ERR_CAPACITY is returned and *out_count_host holds the needed size.
 * Pair order: grouped by radix partition (compare unordered, like the reference's tests). */
int tfg_join_probe(tfg_join *join, int kind, const void *keys, const uint8_t *key_nullmap, int64_t n,
                   uint32_t *out_probe_idx, uint32_t *out_build_idx, uint64_t capacity, uint64_t *out_count_dev,
                   uint64_t *out_count_host);
/* Build rows that carry `npay` (1-2) payload columns of 8 bytes (the build block's columns the
 * joined block needs).  A join is built either with tfg_join_build (index pairs) or with this
 * call for every block (materialising probe). */
int tfg_join_build_rows(tfg_join *join, const void *keys, const uint8_t *key_nullmap, int64_t n, int npay,
                        const void *const *pay);
/* Materialising probe (Join::joinBlock with Adder<KIND, All> + replicateRange, Join.cpp:1153-1358,
 * ColumnVector.cpp:706-738): output row i carries the probe row's `npay` (1-2) payload columns of
 * 8 bytes (out_probe[w]) and, for INNER / LEFT, the matched build row's payload columns
 * (out_build[w]; LEFT rows without a match get 0 and out_build_null[i] = 1).  SEMI / ANTI output
 * the probe payloads only.  Capacity handling as tfg_join_probe; row order grouped by partition. */
int tfg_join_probe_rows(tfg_join *join, int kind, const void *keys, const uint8_t *key_nullmap, int64_t n, int npay,
                        const void *const *probe_pay, void *const *out_probe, void *const *out_build,
                        uint8_t *out_build_null, uint64_t capacity, uint64_t *out_count_host);
/* Other conditions (Join::handleOtherConditions, Interpreters/Join.cpp:798-1150): after an
 * INNER probe and the condition evaluated over the joined pairs, flags[probe_idx[i]] = 1 for
 * every pair i with pass[i] != 0 (pass == NULL: every pair).  `flags` (one byte per probe row)
 * is zeroed by the caller; the LEFT / SEMI / ANTI / left-outer-semi results follow from it. */
int tfg_join_mark(tfg_ctx *ctx, const uint32_t *probe_idx, const uint8_t *pass, int64_t n_pairs, uint8_t *flags);
/* Build-side statistics: rows inserted, distinct keys, partitions. */
int tfg_join_stats(tfg_join *join, uint64_t *rows, uint64_t *partitions);
/* General join keys (chooseJoinMapMethod, Interpreters/JoinHashMap.cpp:33-116: keys128 / keys256
 * for several fixed keys, key_strbin / key_strbinpadding for one String key by collator,
 * serialized otherwise; HashMethodKeysFixed / HashMethodString / HashMethodSerialized,
 * Common/ColumnsHashing.h:179-629).  tfg_join_key_hash folds each row's key tuple (fixed keys of
 * 1-16 bytes as stored; String keys as the collator's sort key, any length) into a UInt64
 * fingerprint; out_nullmap[i] = 1 when any key column is NULL (the row is then a NULL key, as
 * extractNestedColumnsAndNullMap ORs the key null maps).  A join built and probed on the
 * fingerprints yields candidate pairs; tfg_join_keys_equal writes out_pass[i] = pass_in[i] (1
 * when pass_in is NULL) && the full key tuples of probe row probe_idx[i] and build row
 * build_idx[i] are equal, so the verified pairs are exactly the reference's key-equal pairs.
 * key_offsets[j] are String end offsets (NULL for fixed keys); out_pass may alias pass_in. */
int tfg_join_key_hash(tfg_ctx *ctx, int nkeys, const int *key_types, const int *key_collators,
                      const void *const *key_cols, const uint64_t *const *key_offsets,
                      const uint8_t *const *key_nullmaps, int64_t n, uint64_t *out_keys, uint8_t *out_nullmap);
int tfg_join_keys_equal(tfg_ctx *ctx, int nkeys, const int *key_types, const int *key_collators,
                        const void *const *probe_cols, const uint64_t *const *probe_offsets,
                        const void *const *build_cols, const uint64_t *const *build_offsets, const uint32_t *probe_idx,
                        const uint32_t *build_idx, const uint8_t *pass_in, int64_t n_pairs, uint8_t *out_pass);

/* ---------------------------------------------------------------- (e) exchange over RCCL */
/* MPP ExchangeSender -> ExchangeReceiver repartition inside one node (HashPartitionWriter::
 * partitionAndWriteBlocks, Flash/Mpp/HashPartitionWriter.cpp:139-204 -> MPPTunnelSet::write ->
 * ExchangeReceiver, Flash/Mpp/ExchangeReceiver.cpp:626-945): one process per GPU, one RCCL
 * communicator, all-to-all of the partition-major buffers tfg_hash_partition produces.
 * Rank 0 creates the id (tfg_comm_unique_id, 128 bytes) and distributes it out of band. */
typedef struct tfg_comm tfg_comm;
int tfg_comm_unique_id(uint8_t *out_id, size_t len);
int tfg_comm_init(tfg_ctx *ctx, int nranks, int rank, const uint8_t *id, size_t len, tfg_comm **out);
int tfg_comm_destroy(tfg_comm *comm);
int tfg_comm_info(tfg_comm *comm, int *nranks, int *rank);
/* recv_bytes_host[p] = send_bytes_host[this rank] of rank p (host arrays of nranks entries; syncs). */
int tfg_alltoall_counts(tfg_comm *comm, const uint64_t *send_bytes_host, uint64_t *recv_bytes_host);
/* Byte all-to-all on the context's stream: send slice p = [send_displs[p], +send_bytes[p]) to rank
 * p; rank p's slice lands at recv + recv_displs[p].  Counts / displacements are host arrays. */
int tfg_alltoallv(tfg_comm *comm, const void *send, const uint64_t *send_bytes, const uint64_t *send_displs,
                  void *recv, const uint64_t *recv_bytes, const uint64_t *recv_displs);

/* Zero-copy exchange (the product's exchange: tfa::MPPExchange and tiflash_amd/exchange.py): every
 * column plane's slice for a destination is sent from where it lies in the partitioned columns,
 * and every slice from a source is received straight into the output column at its row offset —
 * one RCCL group of ncclSend / ncclRecv per call (HashPartitionWriter::partitionAndWriteBlocks ->
 * MPPTunnelSetWriter, Flash/Mpp/HashPartitionWriter.cpp:139-204, MPPTunnelSetWriter.cpp:365-400;
 * no packet encode / decode and no pack / unpack copy on the device path).  A peer's k-th send
 * slice matches that peer's k-th receive slice from this rank: list each peer's slices in the same
 * (plane) order on both sides; zero-byte slices are skipped.  Asynchronous on the context stream. */
typedef struct tfg_slice {
    int peer;      /* destination (send) or source (recv) rank */
    void *ptr;     /* device memory (read for a send) */
    uint64_t bytes;
} tfg_slice;
int tfg_exchange_slices(tfg_comm *comm, int nsend, const tfg_slice *send, int nrecv, const tfg_slice *recv);
/* k counts per rank pair (row counts per plane): recv[p * k + i] = send[this rank * k + i] of rank
 * p (host arrays of nranks * k; syncs). */
int tfg_alltoall_counts_n(tfg_comm *comm, int k, const uint64_t *send_host, uint64_t *recv_host);
/* String columns received from nparts ranks: end offsets rows [row_start[p], row_start[p + 1])
 * came relative to rank p's chars; each gets add[p] (host arrays). */
int tfg_string_rebase_offsets(tfg_ctx *ctx, uint64_t *offsets, int nparts, const uint64_t *row_start,
                              const uint64_t *add);

/* ---------------------------------------------------------------- (f1) MPP packet codec */
/* The Block wire format of MPP packets, encoded from / decoded into device columns; the packet
 * itself is a device buffer (the tunnel moves its bytes).
 *   TFG_CODEC_CHBLOCK: CHBlockChunkCodecStream::encode / CHBlockChunkCodec::decode
 *                      (Flash/Coprocessor/CHBlockChunkCodec.cpp:134-258).
 *   TFG_CODEC_V1:      CHBlockChunkCodecV1::encode / decode with CompressionMethod::NONE
 *                      (Flash/Coprocessor/CHBlockChunkCodecV1.cpp:370-432, 567-583); decode accepts
 *                      packets of several parts (decodeColumnsByBlock, :97-142), and LZ4
 *                      packets (method byte 0x82: CompressedCHBlockChunkReadBuffer, :567-581)
 *                      and ZSTD packets (0x90, the HIGH_COMPRESSION mode) are decompressed on the
 *                      device first.
 * Type names as on the wire (IDataType::getName): Int8..Int64, UInt8..UInt64, Float32, Float64,
 * Decimal(P,S) with P <= 38, MyDate, MyDateTime(n), MyDuration(n), String (size-prefixed rows),
 * StringV2 (sizes, then chars), and Nullable(...) of each.  Column data follows the tfg_type
 * payloads above; String columns pass chars in `data` and end offsets in `offsets`. */
#define TFG_CODEC_CHBLOCK 0
#define TFG_CODEC_V1 1
typedef struct tfg_codec_column {
    const char *name;       /* host string */
    const char *type_name;  /* host string, e.g. "Nullable(Decimal(15,2))" */
    const void *data;       /* device: values, or String chars */
    const uint64_t *offsets; /* device: String end offsets */
    const uint8_t *nullmap; /* device: Nullable null map */
} tfg_codec_column;
/* Encodes n rows of ncols columns into `out` (device, `capacity` bytes).  out == NULL: returns
 * the exact packet size in *out_bytes_host only.  Synchronises the context stream. */
int tfg_codec_encode(tfg_ctx *ctx, int version, int ncols, const tfg_codec_column *cols, int64_t n, uint8_t *out,
                     size_t capacity, size_t *out_bytes_host);
/* Decoding: tfg_codec_decode parses the header and locates every column's data (String rows are
 * found on the device); then tfg_codec_column_info gives each column's name, type name, tfg_type,
 * nullability and decoded String chars bytes (terminators included), and tfg_codec_column_read
 * writes the column (values / chars + offsets / null map) into caller-provided device buffers.
 * The packet buffer must stay alive until the packet is destroyed. */
typedef struct tfg_codec_packet tfg_codec_packet;
int tfg_codec_decode(tfg_ctx *ctx, int version, const uint8_t *packet, size_t bytes, tfg_codec_packet **out);
int tfg_codec_packet_info(tfg_codec_packet *p, int *out_cols, int64_t *out_rows);
int tfg_codec_column_info(tfg_codec_packet *p, int i, char *name, size_t name_len, char *type_name, size_t type_len,
                          int *out_type, int *out_nullable, uint64_t *out_chars_bytes);
int tfg_codec_column_read(tfg_codec_packet *p, int i, void *out_data, uint64_t *out_offsets, uint8_t *out_nullmap);
int tfg_codec_packet_destroy(tfg_codec_packet *p);

/* LZ4 packets (CompressionMethod values of IO/Compression/CompressionMethod.h:21-29).
 * tfg_codec_compress replaces CHBlockChunkCodecV1::encode(std::string_view, method)
 * (CHBlockChunkCodecV1.cpp:555-565) as MPPTunnelSetHelper::ToCompressedPacket calls it
 * (Flash/Mpp/MPPTunnelSetHelper.cpp:170-185): the body of an uncompressed V1 `packet` (method
 * byte 0x02 first) becomes LZ4 frames `0x82 | UInt32 frame bytes | UInt32 raw bytes | LZ4 block`
 * (64 KB of body per frame), or with TFG_COMPRESSION_ZSTD ZSTD frames
 * `0x90 | UInt32 frame bytes | UInt32 raw bytes | ZSTD frame` (one RFC 8878 frame per 64 KB:
 * single-segment header with the content size, one block — Huffman, RLE or raw literals;
 * sequences with RLE, described (normalized counts) or predefined FSE tables; offsets coded with
 * repeat codes 1-3 — or a raw block when that is smaller; no checksum).  out == NULL:
 * *out_bytes_host = tfg_codec_compress_bound(bytes) (covers both); otherwise the exact size,
 * TFG_ERR_CAPACITY when it exceeds `capacity`.  LZ4HC writes the same format and is accepted as LZ4.
 * tfg_codec_decompress is CompressedCHBlockChunkReadBuffer over a whole packet: the frames of an
 * LZ4 packet (any frame sizes, as any LZ4 encoder wrote them) or of a ZSTD packet (frames
 * `0x90 | UInt32 frame bytes | UInt32 raw bytes | ZSTD frame`, CompressionCodecZSTD.cpp:38-65;
 * RFC 8878 frames without dictionaries, checksums verified) become the uncompressed V1 packet
 * (0x02 + body).  out == NULL: the size only.  Malformed frames: TFG_ERR_INVALID_ARG. */
#define TFG_COMPRESSION_LZ4 1
#define TFG_COMPRESSION_LZ4HC 2
#define TFG_COMPRESSION_ZSTD 3
#define TFG_COMPRESSION_NONE 5
size_t tfg_codec_compress_bound(size_t bytes);
int tfg_codec_compress(tfg_ctx *ctx, int method, const uint8_t *packet, size_t bytes, uint8_t *out, size_t capacity,
                       size_t *out_bytes_host);
int tfg_codec_decompress(tfg_ctx *ctx, const uint8_t *packet, size_t bytes, uint8_t *out, size_t capacity,
                         size_t *out_bytes_host);

#ifdef __cplusplus
}
#endif

#endif /* TIFLASH_AMD_H */
