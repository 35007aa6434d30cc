/*
 * oracle.h — CPU restatement of the reference's hot-path algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU baseline.
 * The product path (tiflash_amd/) never links or calls it.
 *
 * The reference (xfworld/tiflash) cannot be compiled here (its contrib/ submodules incl. boost
 * are empty — SURVEY.md §8c), so this is a from-scratch restatement of the cited reference
 * functions.  It is pinned by: (1) the hardware CRC32-C instruction the reference itself uses
 * (_mm_crc32_u64, Common/HashTable/Hash.h:70-95) on this host; (2) the known answers in the
 * reference's own gtests, transcribed as fixtures in tests/golden/ (see tests/golden/README.md).
 */
#ifndef TFG_ORACLE_H
#define TFG_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int orc_has_hw_crc(void);
uint32_t orc_crc32c_u64(uint32_t crc, uint64_t x);    /* SSE4.2 crc32q when available */
uint32_t orc_crc32c_u64_sw(uint32_t crc, uint64_t x); /* bitwise, reflected 0x82F63B78 */
uint32_t orc_update_weak_hash32_bytes(const uint8_t *pos, size_t size, uint32_t h);
/* utf8mb4_general_ci: weight of a code point; sort key of len bytes (right-trimmed first) into out
 * (>= 2 * len bytes), look-ahead bounded by row_end; returns the key's length */
uint32_t orc_general_ci_weight(uint32_t c);
size_t orc_general_ci_sort_key(const uint8_t *s, size_t len, size_t row_end, uint8_t *out);
/* utf8mb4_unicode_ci (v0900 = 0, UCA 4.0.0, padding) / utf8mb4_0900_ai_ci (v0900 = 1): a code
 * point's weight pair (0 = zero weight, skipped) and a row's sort key; orc_collate dispatches a
 * transforming collator's sort key (<= ORC_KEY_MULT bytes per input byte) */
#define ORC_KEY_MULT 8
int orc_uca_weight(int v0900, uint32_t r, uint64_t *first, uint64_t *second);
size_t orc_uca_sort_key(int v0900, const uint8_t *s, size_t len, size_t row_end, uint8_t *out);
int orc_collator_transforms(int collator);
size_t orc_collate(int collator, const uint8_t *s, size_t len, size_t row_end, uint8_t *out);

void orc_weak_hash_update(int type, const void *col, const uint8_t *nullmap, size_t n, uint32_t *h);
uint64_t orc_float64_to_u64(double x); /* the reference build's Float64 -> UInt64 (x86-64 clang) */
uint64_t orc_float32_to_u64(float x);
void orc_weak_hash_update_string(const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap, size_t n,
                                 int collator, uint32_t *h);
void orc_fill_selector(const uint32_t *h, size_t n, uint32_t part_num, uint32_t fgs, uint32_t *sel);
void orc_partition(const uint32_t *sel, size_t n, uint32_t parts, uint32_t *perm, uint64_t *offsets);

void orc_cmp(int a_type, const void *a, int a_const, int op, int b_type, const void *b, int b_const,
             const uint8_t *a_null, const uint8_t *b_null, size_t n, uint8_t *out);
size_t orc_count_bytes_in_filter(const uint8_t *f, const uint8_t *nullmap, size_t n);
size_t orc_filter(int width, const void *col, const uint8_t *f, size_t n, void *out);
size_t orc_filter_string(const uint8_t *chars, const uint64_t *offsets, const uint8_t *f, size_t n,
                         uint8_t *out_chars, uint64_t *out_offsets, size_t *out_bytes);
int orc_arith(int op, int a_type, const void *a, int a_const, int a_scale, int b_type, const void *b, int b_const,
              int b_scale, int res_type, int res_scale, size_t n, void *out);

typedef struct orc_agg orc_agg;
/* arg_types[i]: tfg_type | TFG_ARG_PREC(p) (include/tiflash_amd.h); sum(Decimal(p,s)) keeps a
 * Decimal256 state when min(p + 22, 65) > 38 (SumDecimalInferer). */
int orc_sum_result_prec(int arg_type_word);
orc_agg *orc_agg_create(int key_type, int n_aggs, const int *kinds, const int *arg_types);
void orc_agg_destroy(orc_agg *a);
void orc_agg_consume(orc_agg *a, const void *keys, const uint8_t *key_null, const void *const *args,
                     const uint8_t *const *arg_nulls, const uint8_t *mask, size_t n);
void orc_agg_merge(orc_agg *dst, const orc_agg *src);
size_t orc_agg_size(const orc_agg *a);
/* String min / max / first_row results: chars bytes; String arguments / results travel as host
 * structs {chars, offsets} (args / out_states entries), like the device ABI's tfg_str_col / _out */
size_t orc_agg_result_chars(const orc_agg *a, int i);
int orc_min_max_str_compare(int collator, const uint8_t *a, size_t la, const uint8_t *b, size_t lb);
/* out_keys: u64 key bits; out_key_null; out_states[i]: 8, 16 or 32 B per group; out_state_null[i]. */
void orc_agg_result(const orc_agg *a, uint64_t *out_keys, uint8_t *out_key_null, void *const *out_states,
                    uint8_t *const *out_state_null);

/* Several keys / one String key (Aggregator methods keys128, key_string, serialized). */
typedef struct orc_aggk orc_aggk;
orc_aggk *orc_aggk_create(int nkeys, const int *key_types, const int *collators, int n_aggs, const int *kinds,
                          const int *arg_types);
void orc_aggk_destroy(orc_aggk *a);
void orc_aggk_consume(orc_aggk *a, const void *const *key_cols, const uint64_t *const *key_offsets,
                      const uint8_t *const *key_nulls, const void *const *args, const uint8_t *const *arg_nulls,
                      const uint8_t *mask, size_t n);
size_t orc_aggk_size(const orc_aggk *a);
size_t orc_aggk_result_chars(const orc_aggk *a, int i);
size_t orc_aggk_result(const orc_aggk *a, uint8_t *out_keys, uint64_t *out_key_offsets, void *const *out_states,
                       uint8_t *const *out_state_null);

typedef struct orc_join orc_join;
orc_join *orc_join_create(int key_type);
void orc_join_build(orc_join *j, const void *keys, const uint8_t *key_null, size_t n);
void orc_join_destroy(orc_join *j);
size_t orc_join_probe(const orc_join *j, int kind, const void *keys, const uint8_t *key_null, size_t n,
                      uint32_t *out_probe, uint32_t *out_build, size_t capacity);

/* CPU baseline legs (threads = nthreads; per-thread tables merged after a barrier like
 * ParallelAggregatingBlockInputStream.cpp:77-159).  Return the number of groups / matches. */
size_t orc_bench_filter_agg(const int64_t *f, int64_t threshold, const int64_t *k, const double *v, size_t n,
                            int nthreads, size_t block_rows, double *checksum);
/* The C2 step with the reference's own data structures (cpu_baseline.c): per-thread key64 HashMap
 * with arena states, prefetch, two-level conversion at 100k keys, bucket-parallel merge and
 * result conversion.  bench.py's cpu_baseline leg. */
size_t orc_bench_filter_agg_ref(const int64_t *f, int64_t threshold, const int64_t *k, const double *v, size_t n,
                                int nthreads, size_t block_rows, double *checksum);
/* C3 join leg with the reference's structures (cpu_baseline.c): segment maps of RowRefList cells. */
typedef struct orc_join_ref orc_join_ref;
orc_join_ref *orc_join_ref_build(const int64_t *build_keys, const int64_t *build_pay, size_t nb, int nthreads);
size_t orc_join_ref_probe(const orc_join_ref *j, const int64_t *probe_keys, const int64_t *probe_pay, size_t np,
                          int nthreads, uint64_t *checksum);
void orc_join_ref_destroy(orc_join_ref *j);
/* C5 partial aggregation leg (cpu_baseline_str.c): StringHashMap StringKey16 sub-maps, arena
 * Decimal128 + count states, two-level at 100k keys, bucket-parallel merge + result conversion. */
size_t orc_bench_string_agg(const uint8_t *chars, const uint64_t *offsets, const int64_t *v, size_t n, int nthreads,
                            size_t block_rows, uint64_t *checksum);
size_t orc_bench_join(const int64_t *build_keys, size_t nb, const int64_t *probe_keys, size_t np, int nthreads,
                      uint64_t *checksum);

/* CHBlockChunkCodec / V1 (NONE) restated (codec.c): packet bytes of n rows (see codec.c). */
size_t orc_codec_encode(int version, int ncols, const char *const *names, const char *const *types,
                        const void *const *data, const uint64_t *const *offsets, const uint8_t *const *nullmaps,
                        int64_t n, int nparts, const int64_t *part_rows, uint8_t *out, size_t cap);

/* LZ4 block format and LZ4 MPP packets restated (lz4.c). */
int64_t orc_lz4_decompress_block(const uint8_t *src, size_t srclen, uint8_t *dst, size_t dstcap);
size_t orc_lz4_bound(size_t n);
size_t orc_lz4_compress_block(const uint8_t *src, size_t n, uint8_t *dst);
size_t orc_lz4_packet_compress(const uint8_t *pkt, size_t bytes, size_t frame_raw, uint8_t *out);
int64_t orc_lz4_packet_decompress(const uint8_t *pkt, size_t bytes, uint8_t *out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
