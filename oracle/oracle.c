/*
 * oracle.c — CPU restatement of the reference's hot path (xfworld/tiflash, dbms/src/...).
 *
 * TEST INFRASTRUCTURE ONLY (checker + timed CPU baseline).  Never linked by the product.
 * Every function cites the reference lines it restates; paths are relative to
 * /root/reference/dbms/src.  Written from scratch (the reference cannot be compiled here:
 * SURVEY.md §8c); pinned by the hardware CRC32-C instruction and the reference gtests'
 * known answers (tests/golden/).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#ifdef __SSE4_2__
#include <nmmintrin.h>
#endif

#include "../include/tiflash_amd.h"
#include "collation_data.h"
#include "uca_data.h"

/* ------------------------------------------------------------------ CRC32-C */
/* intHashCRC32(x, seed) = _mm_crc32_u64(seed, x)  (Common/HashTable/Hash.h:70-95). */
int orc_has_hw_crc(void)
{
#ifdef __SSE4_2__
    return 1;
#else
    return 0;
#endif
}

uint32_t orc_crc32c_u64_sw(uint32_t crc, uint64_t x)
{
    /* crc32q semantics: reflected CRC-32C (poly 0x1EDC6F41, reversed 0x82F63B78), no init/final
     * inversion inside the instruction. */
    for (int byte = 0; byte < 8; ++byte) {
        crc ^= (uint32_t)(x & 0xFF);
        x >>= 8;
        for (int b = 0; b < 8; ++b)
            crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
    }
    return crc;
}

uint32_t orc_crc32c_u64(uint32_t crc, uint64_t x)
{
#ifdef __SSE4_2__
    return (uint32_t)_mm_crc32_u64(crc, x);
#else
    return orc_crc32c_u64_sw(crc, x);
#endif
}

static inline uint32_t int_hash_crc32(uint64_t x) { return orc_crc32c_u64(0xFFFFFFFFu, x); }

/* ::updateWeakHash32(const UInt8 * pos, size_t size, UInt32) (Common/HashTable/Hash.h:148-214). */
uint32_t orc_update_weak_hash32_bytes(const uint8_t *pos, size_t size, uint32_t h)
{
    if (size < 8) {
        uint64_t value = 0;
        memcpy(&value, pos, size);
        ((unsigned char *)&value)[7] = (unsigned char)size;
        return orc_crc32c_u64(h, value);
    }
    const uint8_t *end = pos + size;
    while (pos + 8 <= end) {
        uint64_t word;
        memcpy(&word, pos, 8);
        h = orc_crc32c_u64(h, word);
        pos += 8;
    }
    if (pos < end) {
        uint8_t tail = (uint8_t)(end - pos);
        uint64_t word;
        memcpy(&word, end - 8, 8);
        word &= (~(uint64_t)0) << (8 * (8 - tail));
        word |= tail;
        h = orc_crc32c_u64(h, word);
    }
    return h;
}

/* ------------------------------------------------------------------ value access */
static size_t type_width(int t)
{
    switch (t) {
    case TFG_INT8: case TFG_UINT8: return 1;
    case TFG_INT16: case TFG_UINT16: return 2;
    case TFG_INT32: case TFG_UINT32: case TFG_FLOAT32: case TFG_DECIMAL32: return 4;
    case TFG_INT64: case TFG_UINT64: case TFG_FLOAT64: case TFG_DECIMAL64: return 8;
    case TFG_DECIMAL128: return 16;
    case TFG_DECIMAL256: return 32;
    default: return 0;
    }
}
static int is_float(int t) { return t == TFG_FLOAT32 || t == TFG_FLOAT64; }
static int is_unsigned(int t) { return t == TFG_UINT8 || t == TFG_UINT16 || t == TFG_UINT32 || t == TFG_UINT64; }

static int64_t load_s(int t, const void *p, size_t i)
{
    switch (t) {
    case TFG_INT8: return ((const int8_t *)p)[i];
    case TFG_INT16: return ((const int16_t *)p)[i];
    case TFG_INT32: case TFG_DECIMAL32: return ((const int32_t *)p)[i];
    case TFG_INT64: case TFG_DECIMAL64: return ((const int64_t *)p)[i];
    case TFG_UINT8: return ((const uint8_t *)p)[i];
    case TFG_UINT16: return ((const uint16_t *)p)[i];
    case TFG_UINT32: return ((const uint32_t *)p)[i];
    case TFG_UINT64: return (int64_t)((const uint64_t *)p)[i];
    default: return 0;
    }
}
static double load_f(int t, const void *p, size_t i)
{
    return t == TFG_FLOAT32 ? (double)((const float *)p)[i] : ((const double *)p)[i];
}
static __int128 load_i128(int t, const void *p, size_t i)
{
    if (t == TFG_DECIMAL128) {
        __int128 v;
        memcpy(&v, (const char *)p + 16 * i, 16);
        return v;
    }
    if (t == TFG_UINT64) return (__int128)((const uint64_t *)p)[i];
    return (__int128)load_s(t, p, i);
}
/* Raw bits of a key zero-extended to UInt64 (HashMethodOneNumber reads the raw FieldType,
 * Common/ColumnsHashing.h:43-90; key8..key64 methods). */
static uint64_t load_key_bits(int t, const void *p, size_t i)
{
    switch (type_width(t)) {
    case 1: return ((const uint8_t *)p)[i];
    case 2: return ((const uint16_t *)p)[i];
    case 4: return ((const uint32_t *)p)[i];
    default: return ((const uint64_t *)p)[i];
    }
}

/* ------------------------------------------------------------------ weak hash / partition */
/* ColumnVector<T>::updateWeakHash32Impl (Columns/ColumnVector.cpp:499-535): h = crc(h, UInt64(v));
 * ColumnDecimal (ColumnDecimal.cpp:658 -> wideIntHashCRC32, Hash.h:97-145);
 * ColumnNullable keeps the old hash for NULL rows (ColumnNullable.cpp:131-173). */
/* Float -> UInt64 as the reference's implicit conversion in intHashCRC32(UInt64, UInt32)
 * (Columns/ColumnVector.cpp:528, Common/HashTable/Hash.h:83-94) compiles on x86-64 with clang
 * (SSE4.2, no AVX-512): cvttsd2si(x) | (cvttsd2si(x - 2^63) & (cvttsd2si(x) >> 63)), where the
 * truncating convert gives INT64_MIN for NaN / out-of-range values.  Restated explicitly (a C
 * cast is undefined there); pinned by tests/golden/float_weak_hash.json. */
static int64_t cvtt_d(double x) { return (x >= -9223372036854775808.0 && x < 9223372036854775808.0) ? (int64_t)x : INT64_MIN; }
static int64_t cvtt_f(float x) { return (x >= -9223372036854775808.0f && x < 9223372036854775808.0f) ? (int64_t)x : INT64_MIN; }
uint64_t orc_float64_to_u64(double x)
{
    const int64_t a = cvtt_d(x), b = cvtt_d(x - 9223372036854775808.0);
    return (uint64_t)(a | (b & (a >> 63)));
}
uint64_t orc_float32_to_u64(float x)
{
    const float y = x - 9223372036854775808.0f; /* float arithmetic, as subss */
    const int64_t a = cvtt_f(x), b = cvtt_f(y);
    return (uint64_t)(a | (b & (a >> 63)));
}

void orc_weak_hash_update(int type, const void *col, const uint8_t *nullmap, size_t n, uint32_t *h)
{
    for (size_t i = 0; i < n; ++i) {
        if (nullmap && nullmap[i]) continue;
        if (type == TFG_FLOAT64 || type == TFG_FLOAT32) {
            const uint64_t v = type == TFG_FLOAT64 ? orc_float64_to_u64(((const double *)col)[i])
                                                   : orc_float32_to_u64(((const float *)col)[i]);
            h[i] = orc_crc32c_u64(h[i], v);
        } else if (type == TFG_DECIMAL128) {
            uint64_t limb[2];
            memcpy(limb, (const char *)col + 16 * i, 16);
            uint32_t x = orc_crc32c_u64(h[i], limb[0]);
            h[i] = orc_crc32c_u64(x, limb[1]);
        } else {
            /* implicit conversion to UInt64: signed types sign-extend, unsigned zero-extend */
            uint64_t v = is_unsigned(type) ? (uint64_t)load_s(type, col, i) : (uint64_t)load_s(type, col, i);
            h[i] = orc_crc32c_u64(h[i], v);
        }
    }
}

/* ---------------------------------------------------------------- utf8mb4_general_ci
 * GeneralCICollator::sortKey = convertImpl<false, true> (TiDB/Collation/Collator.cpp:416-455):
 * right-trim ' ' (RightTrim, CollatorCompare.h:56-61), decode UTF-8 (decodeUtf8Char,
 * Collator.cpp:43-74: the lead byte sets the length, continuation bytes unchecked), write each
 * character's weight big-endian; weight (Collator.h:403-407): 0xFFFD past the BMP, else the
 * GeneralCI::weight_lut entry (collation_data.h, re-encoded as runs).  `row_end` bounds the
 * decoder's look-ahead (a truncated sequence reads zeros past it). */
static const uint32_t orc_gci_runs[TFG_GCI_RUNS][3] = {TFG_GCI_RUNS_INIT};

uint32_t orc_general_ci_weight(uint32_t c)
{
    if (c > 0xFFFF) return 0xFFFD;
    int lo = 0, hi = TFG_GCI_RUNS - 1;
    while (lo <= hi) { /* the last run starting at or before c */
        const int mid = (lo + hi) / 2;
        if (orc_gci_runs[mid][0] <= c) lo = mid + 1;
        else hi = mid - 1;
    }
    if (hi < 0 || c > orc_gci_runs[hi][1]) return c;
    const uint32_t v = orc_gci_runs[hi][2];
    if (v >> 16) return v & 0xFFFF;
    return (uint32_t)(c + (int16_t)(v & 0xFFFF)) & 0xFFFF;
}

/* decodeUtf8Char (Collator.cpp:43-74): the lead byte sets the length, continuation bytes are not
 * checked; a sequence cut by the row's end reads zeros past row_end */
static uint32_t orc_utf8_next(const uint8_t *s, size_t row_end, size_t *off)
{
#define ORC_AT(k) ((size_t)(k) < row_end ? (uint32_t)s[k] : 0u)
    const size_t o = *off;
    const uint32_t b0 = s[o];
    uint32_t c;
    if (b0 < 0x80) {
        c = b0;
        *off = o + 1;
    } else if (b0 < 0xE0) {
        c = (b0 & 0x1F) << 6 | (ORC_AT(o + 1) & 0x3F);
        *off = o + 2;
    } else if (b0 < 0xF0) {
        c = (b0 & 0x0F) << 12 | (ORC_AT(o + 1) & 0x3F) << 6 | (ORC_AT(o + 2) & 0x3F);
        *off = o + 3;
    } else {
        c = (b0 & 0x07) << 18 | (ORC_AT(o + 1) & 0x3F) << 12 | (ORC_AT(o + 2) & 0x3F) << 6 | (ORC_AT(o + 3) & 0x3F);
        *off = o + 4;
    }
#undef ORC_AT
    return c;
}

size_t orc_general_ci_sort_key(const uint8_t *s, size_t len, size_t row_end, uint8_t *out)
{
    while (len > 0 && s[len - 1] == ' ') --len;
    size_t off = 0, o = 0;
    while (off < len) {
        const uint32_t w = orc_general_ci_weight(orc_utf8_next(s, row_end, &off));
        out[o++] = (uint8_t)(w >> 8);
        out[o++] = (uint8_t)w;
    }
    return o;
}

/* ---------------------------------------------------------------- UCA collators
 * utf8_unicode_ci / utf8mb4_unicode_ci = UCACICollator<Unicode0400, padding> and
 * utf8mb4_0900_ai_ci = UCACICollator<Unicode0900, no padding> (Collator.h:415-437).
 * sortKey = convertImpl<false, true> (Collator.cpp:580-629): right-trim ' ' when padding, then per
 * character (weight(), :639-667) skip zero-weight characters, take the LUT weight
 * (Unicode0400::weight :703-727: 0xFFFD past the BMP; Unicode0900::weight :791-816: an implicit
 * weight from the code point past the table) or, for the LUT value 0xFFFD, the character's long
 * weight pair (weightLutLongMap), and write `first` then `second` with writeResult (Collator.h:
 * 336-344): 16-bit chunks from the low end while the value is non-zero, each big-endian.
 * The LUTs (uca_data.h) are expanded from their runs on first use (single-threaded checker). */
typedef struct {
    uint32_t start, count;
    uint64_t base, delta;
} orc_uca_run;
typedef struct {
    uint32_t cp;
    uint64_t first, second;
} orc_uca_long;
static const orc_uca_run orc_uca0400_runs[TFG_UCA0400_NRUNS] = {TFG_UCA0400_RUNS_INIT};
static const orc_uca_run orc_uca0900_runs[TFG_UCA0900_NRUNS] = {TFG_UCA0900_RUNS_INIT};
static const orc_uca_long orc_uca0400_long[TFG_UCA0400_NLONG] = {TFG_UCA0400_LONG_INIT};
static const orc_uca_long orc_uca0900_long[TFG_UCA0900_NLONG] = {TFG_UCA0900_LONG_INIT};
static uint64_t *orc_uca_lut[2];

static const uint64_t *orc_uca_table(int v0900)
{
    if (!orc_uca_lut[v0900]) {
        const orc_uca_run *runs = v0900 ? orc_uca0900_runs : orc_uca0400_runs;
        const int nr = v0900 ? TFG_UCA0900_NRUNS : TFG_UCA0400_NRUNS;
        const size_t size = v0900 ? TFG_UCA0900_SIZE : TFG_UCA0400_SIZE;
        uint64_t *t = (uint64_t *)calloc(size, 8);
        for (int i = 0; i < nr; ++i)
            for (uint32_t k = 0; k < runs[i].count; ++k) t[runs[i].start + k] = runs[i].base + (uint64_t)k * runs[i].delta;
        orc_uca_lut[v0900] = t;
    }
    return orc_uca_lut[v0900];
}

/* T::weight: 0 = a zero-weight character (skipped), else first / second set */
int orc_uca_weight(int v0900, uint32_t r, uint64_t *first, uint64_t *second)
{
    *second = 0;
    if (!v0900 && r > 0xFFFF) {
        *first = 0xFFFD;
        return 1;
    }
    if (v0900 && r >= TFG_UCA0900_SIZE) { /* (the reference tests r > 0x2CEA1 and reads one past its LUT at r == 0x2CEA1) */
        *first = (uint64_t)(r >> 15) + 0xFBC0 + ((uint64_t)((r & 0x7FFF) | 0x8000) << 16);
        return 1;
    }
    const uint64_t w = orc_uca_table(v0900)[r];
    if (w == 0) return 0;
    if (w != 0xFFFD) {
        *first = w;
        return 1;
    }
    const orc_uca_long *lw = v0900 ? orc_uca0900_long : orc_uca0400_long;
    const int nl = v0900 ? TFG_UCA0900_NLONG : TFG_UCA0400_NLONG;
    *first = 0; /* weightLutLongMap's default entry: {0, 0} */
    for (int i = 0; i < nl; ++i)
        if (lw[i].cp == r) {
            *first = lw[i].first;
            *second = lw[i].second;
        }
    return 1;
}

size_t orc_uca_sort_key(int v0900, const uint8_t *s, size_t len, size_t row_end, uint8_t *out)
{
    if (!v0900)
        while (len > 0 && s[len - 1] == ' ') --len;
    size_t off = 0, o = 0;
    while (off < len) {
        uint64_t w[2];
        if (!orc_uca_weight(v0900, orc_utf8_next(s, row_end, &off), &w[0], &w[1])) continue;
        for (int h = 0; h < 2; ++h)
            for (uint64_t x = w[h]; x != 0; x >>= 16) {
                out[o++] = (uint8_t)(x >> 8);
                out[o++] = (uint8_t)x;
            }
    }
    return o;
}

int orc_collator_transforms(int collator)
{
    return collator == TFG_COLLATOR_GENERAL_CI || collator == TFG_COLLATOR_UNICODE_CI || collator == TFG_COLLATOR_UCA0900_AI_CI;
}

/* the sort key of a transforming collator (<= ORC_KEY_MULT bytes per input byte) */
size_t orc_collate(int collator, const uint8_t *s, size_t len, size_t row_end, uint8_t *out)
{
    if (collator == TFG_COLLATOR_GENERAL_CI) return orc_general_ci_sort_key(s, len, row_end, out);
    return orc_uca_sort_key(collator == TFG_COLLATOR_UCA0900_AI_CI, s, len, row_end, out);
}

/* the collator's sort key of a ColumnString row's bytes (len = size - 1, '\0' excluded) into buf
 * (>= ORC_KEY_MULT * len bytes); returns a pointer to the key and its length */
static const uint8_t *orc_sort_key(int collator, const uint8_t *s, size_t len, uint8_t *buf, size_t *klen)
{
    if (orc_collator_transforms(collator)) {
        *klen = orc_collate(collator, s, len, len + 1, buf);
        return buf;
    }
    if (collator == TFG_COLLATOR_BIN_PADDING)
        while (len > 0 && s[len - 1] == ' ') --len;
    *klen = len;
    return s;
}

/* ColumnString::updateWeakHash32 (Columns/ColumnString.cpp:1228-1327): hashes size-1 bytes (the
 * trailing '\0' excluded) after the collator's sort key; BIN padding collators right-trim ' '
 * (TiDB/Collation/CollatorCompare.h:49-95). */
void orc_weak_hash_update_string(const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap, size_t n,
                                 int collator, uint32_t *h)
{
    uint8_t *buf = NULL;
    size_t cap = 0;
    for (size_t i = 0; i < n; ++i) {
        if (nullmap && nullmap[i]) continue;
        uint64_t prev = i ? offsets[i - 1] : 0;
        size_t len = (size_t)(offsets[i] - prev - 1);
        if (ORC_KEY_MULT * len + 16 > cap) {
            cap = 2 * (ORC_KEY_MULT * len + 16);
            buf = (uint8_t *)realloc(buf, cap);
        }
        size_t klen;
        const uint8_t *k = orc_sort_key(collator, chars + prev, len, buf, &klen);
        h[i] = orc_update_weak_hash32_bytes(k, klen, h[i]);
    }
    free(buf);
}

/* fillSelector / fillSelectorForFineGrainedShuffle (Flash/Mpp/HashBaseWriterHelper.cpp:46-84). */
void orc_fill_selector(const uint32_t *h, size_t n, uint32_t part_num, uint32_t fgs, uint32_t *sel)
{
    for (size_t i = 0; i < n; ++i) {
        uint64_t s = h[i];
        s *= part_num;
        s >>= 32;
        if (fgs) s = s * fgs + h[i] % fgs;
        sel[i] = (uint32_t)s;
    }
}

/* Stable partition behind IColumn::scatterImpl (Columns/IColumn.h:655-721): each destination
 * receives rows in input order. */
void orc_partition(const uint32_t *sel, size_t n, uint32_t parts, uint32_t *perm, uint64_t *offsets)
{
    memset(offsets, 0, sizeof(uint64_t) * (parts + 1));
    for (size_t i = 0; i < n; ++i) offsets[sel[i] + 1]++;
    for (uint32_t p = 0; p < parts; ++p) offsets[p + 1] += offsets[p];
    uint64_t *cur = (uint64_t *)malloc(sizeof(uint64_t) * (parts ? parts : 1));
    memcpy(cur, offsets, sizeof(uint64_t) * parts);
    for (size_t i = 0; i < n; ++i) perm[cur[sel[i]]++] = (uint32_t)i;
    free(cur);
}

/* ------------------------------------------------------------------ comparison */
/* Exact comparison of two numbers of different classes; returns -1/0/1, or 2 if unordered (NaN).
 * Restates accurate::lessOp / equalsOp (Core/AccurateComparison.h:33-159): same-signedness ints
 * compare natively, mixed signedness exactly, int vs float exactly (DecomposedFloat for >32-bit
 * ints, double cast otherwise — both exact), anything vs NaN is false. */
typedef struct { int cls; int64_t s; uint64_t u; double d; } num; /* cls 0=signed 1=unsigned 2=float */

static num load_num(int t, const void *p, size_t i)
{
    num r = {0, 0, 0, 0.0};
    if (is_float(t)) { r.cls = 2; r.d = load_f(t, p, i); }
    else if (is_unsigned(t)) { r.cls = 1; r.u = (uint64_t)load_s(t, p, i); }
    else { r.cls = 0; r.s = load_s(t, p, i); }
    return r;
}

static int cmp_s_d(int64_t a, double d)
{
    if (d >= 9223372036854775808.0) return -1;
    if (d < -9223372036854775808.0) return 1;
    int64_t t = (int64_t)d;
    if (a < t) return -1;
    if (a > t) return 1;
    double frac = d - (double)t;
    return frac > 0 ? -1 : (frac < 0 ? 1 : 0);
}
static int cmp_u_d(uint64_t a, double d)
{
    if (d >= 18446744073709551616.0) return -1;
    if (d < 0) return 1;
    uint64_t t = (uint64_t)d;
    if (a < t) return -1;
    if (a > t) return 1;
    double frac = d - (double)t;
    return frac > 0 ? -1 : 0;
}
static int cmp_num(num a, num b)
{
    if (a.cls == 2 && isnan(a.d)) return 2;
    if (b.cls == 2 && isnan(b.d)) return 2;
    if (a.cls == 2 && b.cls == 2) return a.d < b.d ? -1 : (a.d > b.d ? 1 : 0);
    if (a.cls == 0 && b.cls == 0) return a.s < b.s ? -1 : (a.s > b.s ? 1 : 0);
    if (a.cls == 1 && b.cls == 1) return a.u < b.u ? -1 : (a.u > b.u ? 1 : 0);
    if (a.cls == 0 && b.cls == 1) return a.s < 0 ? -1 : ((uint64_t)a.s < b.u ? -1 : ((uint64_t)a.s > b.u ? 1 : 0));
    if (a.cls == 1 && b.cls == 0) return -cmp_num(b, a);
    if (a.cls == 0 && b.cls == 2) return cmp_s_d(a.s, b.d);
    if (a.cls == 1 && b.cls == 2) return cmp_u_d(a.u, b.d);
    /* a float, b int */
    return -cmp_num(b, a);
}

static uint8_t apply_op(int op, int c)
{
    if (c == 2) return op == TFG_NE; /* NaN: only notEquals is true (notEqualsOp = !equalsOp) */
    switch (op) {
    case TFG_EQ: return c == 0;
    case TFG_NE: return c != 0;
    case TFG_LT: return c < 0;
    case TFG_LE: return c <= 0;
    case TFG_GT: return c > 0;
    case TFG_GE: return c >= 0;
    }
    return 0;
}

/* NumComparisonImpl::vectorVector / vectorConstant / constantVector
 * (Functions/FunctionsComparison.h:74-122).  NULL rows -> 0 (FilterDescription folding). */
void orc_cmp(int a_type, const void *a, int a_const, int op, int b_type, const void *b, int b_const,
             const uint8_t *a_null, const uint8_t *b_null, size_t n, uint8_t *out)
{
    for (size_t i = 0; i < n; ++i) {
        if ((a_null && a_null[i]) || (b_null && b_null[i])) { out[i] = 0; continue; }
        num x = load_num(a_type, a, a_const ? 0 : i);
        num y = load_num(b_type, b, b_const ? 0 : i);
        out[i] = apply_op(op, cmp_num(x, y));
    }
}

/* countBytesInFilter / countBytesInFilterWithNull (Columns/countBytesInFilter.cpp:32-124). */
size_t orc_count_bytes_in_filter(const uint8_t *f, const uint8_t *nullmap, size_t n)
{
    size_t c = 0;
    for (size_t i = 0; i < n; ++i) c += (f[i] != 0) && !(nullmap && nullmap[i]);
    return c;
}

/* filterImpl (Columns/filterColumn.cpp:174-305): per 64 rows ToBits64 -> prefix / suffix run
 * or pop-bit loop; scalar tail.  Stable. */
size_t orc_filter(int width, const void *col, const uint8_t *f, size_t n, void *out)
{
    const char *src = (const char *)col;
    char *dst = (char *)out;
    size_t k = 0, i = 0;
    for (; i + 64 <= n; i += 64) {
        uint64_t mask = 0;
        for (int b = 0; b < 64; ++b) mask |= (uint64_t)(f[i + b] != 0) << b; /* ToBits64 */
        while (mask) {
            int idx = __builtin_ctzll(mask);
            memcpy(dst + (size_t)width * k++, src + (size_t)width * (i + idx), (size_t)width);
            mask &= mask - 1;
        }
    }
    for (; i < n; ++i)
        if (f[i]) memcpy(dst + (size_t)width * k++, src + (size_t)width * i, (size_t)width);
    return k;
}

/* filterArraysImplGeneric for ColumnString (Columns/filterColumn.cpp:97-171). */
size_t orc_filter_string(const uint8_t *chars, const uint64_t *offsets, const uint8_t *f, size_t n,
                         uint8_t *out_chars, uint64_t *out_offsets, size_t *out_bytes)
{
    size_t rows = 0, bytes = 0;
    for (size_t i = 0; i < n; ++i) {
        if (!f[i]) continue;
        uint64_t prev = i ? offsets[i - 1] : 0;
        size_t len = (size_t)(offsets[i] - prev);
        memcpy(out_chars + bytes, chars + prev, len);
        bytes += len;
        out_offsets[rows++] = bytes;
    }
    *out_bytes = bytes;
    return rows;
}

/* ------------------------------------------------------------------ arithmetic */
static __int128 pow10_i128(int e)
{
    __int128 r = 1;
    while (e-- > 0) r *= 10;
    return r;
}
static int is_decimal(int t) { return t == TFG_DECIMAL32 || t == TFG_DECIMAL64 || t == TFG_DECIMAL128; }

/* BinaryOperationImplBase / DecimalBinaryOperation (Functions/FunctionBinaryArithmetic.h:72-215,
 * 231-500): for +/- decimals are scaled to the result scale (applyScaled); * multiplies raw
 * values (result scale = sa + sb).  Integer ops wrap (two's complement). */
int orc_arith(int op, int a_type, const void *a, int a_const, int a_scale, int b_type, const void *b, int b_const,
              int b_scale, int res_type, int res_scale, size_t n, void *out)
{
    int dec = is_decimal(res_type);
    for (size_t i = 0; i < n; ++i) {
        size_t ia = a_const ? 0 : i, ib = b_const ? 0 : i;
        if (res_type == TFG_FLOAT64 || res_type == TFG_FLOAT32) {
            /* an integer operand converts to Float64 by value (UInt64 above 2^63 included) */
            double x = is_float(a_type) ? load_f(a_type, a, ia)
                       : a_type == TFG_UINT64 ? (double)((const uint64_t *)a)[ia] : (double)load_s(a_type, a, ia);
            double y = is_float(b_type) ? load_f(b_type, b, ib)
                       : b_type == TFG_UINT64 ? (double)((const uint64_t *)b)[ib] : (double)load_s(b_type, b, ib);
            double r = op == TFG_PLUS ? x + y : op == TFG_MINUS ? x - y : x * y;
            if (res_type == TFG_FLOAT64) ((double *)out)[i] = r;
            else ((float *)out)[i] = (float)r;
            continue;
        }
        __int128 x = load_i128(a_type, a, ia), y = load_i128(b_type, b, ib), r;
        if (dec && op != TFG_MULTIPLY) {
            x *= pow10_i128(res_scale - (is_decimal(a_type) ? a_scale : 0));
            y *= pow10_i128(res_scale - (is_decimal(b_type) ? b_scale : 0));
        }
        if (op == TFG_PLUS) r = (__int128)((unsigned __int128)x + (unsigned __int128)y);
        else if (op == TFG_MINUS) r = (__int128)((unsigned __int128)x - (unsigned __int128)y);
        else r = (__int128)((unsigned __int128)x * (unsigned __int128)y);
        switch (type_width(res_type)) {
        case 1: ((int8_t *)out)[i] = (int8_t)r; break;
        case 2: ((int16_t *)out)[i] = (int16_t)r; break;
        case 4: ((int32_t *)out)[i] = (int32_t)r; break;
        case 8: ((int64_t *)out)[i] = (int64_t)r; break;
        case 16: memcpy((char *)out + 16 * i, &r, 16); break;
        default: return -1;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ HashMap (key64) */
/* HashTable<UInt64, ..., HashCRC32<UInt64>, HashTableGrower<8>> restated:
 * linear probing place = hash & mask, next = +1 (Common/HashTable/HashTable.h:437, 254-296);
 * resize when size > maxFill = buf/2 (overflow), growing by 2 degrees below 2^23, then 1;
 * key 0 lives outside the buffer (ZeroValueStorage, :325-360). */
typedef struct {
    uint64_t *keys;
    int64_t *vals; /* mapped value: group / list index, -1 = empty */
    int degree;
    size_t size;
    int has_zero;
    int64_t zero_val;
} hmap;

static void hmap_init(hmap *m)
{
    m->degree = 8;
    size_t cap = (size_t)1 << m->degree;
    m->keys = (uint64_t *)calloc(cap, sizeof(uint64_t));
    m->vals = (int64_t *)malloc(cap * sizeof(int64_t));
    for (size_t i = 0; i < cap; ++i) m->vals[i] = -1;
    m->size = 0;
    m->has_zero = 0;
    m->zero_val = -1;
}
static void hmap_free(hmap *m)
{
    free(m->keys);
    free(m->vals);
}
static void hmap_resize(hmap *m)
{
    size_t old_cap = (size_t)1 << m->degree;
    uint64_t *ok = m->keys;
    int64_t *ov = m->vals;
    m->degree += m->degree >= 23 ? 1 : 2;
    size_t cap = (size_t)1 << m->degree, mask = cap - 1;
    m->keys = (uint64_t *)calloc(cap, sizeof(uint64_t));
    m->vals = (int64_t *)malloc(cap * sizeof(int64_t));
    for (size_t i = 0; i < cap; ++i) m->vals[i] = -1;
    for (size_t i = 0; i < old_cap; ++i) {
        if (ov[i] < 0) continue;
        size_t p = int_hash_crc32(ok[i]) & mask;
        while (m->vals[p] >= 0) p = (p + 1) & mask;
        m->keys[p] = ok[i];
        m->vals[p] = ov[i];
    }
    free(ok);
    free(ov);
}
/* emplace: returns pointer to mapped value; *inserted set when new. */
static int64_t *hmap_emplace(hmap *m, uint64_t key, int *inserted)
{
    *inserted = 0;
    if (key == 0) { /* emplaceIfZero */
        if (!m->has_zero) { m->has_zero = 1; *inserted = 1; }
        return &m->zero_val;
    }
    size_t mask = ((size_t)1 << m->degree) - 1;
    size_t p = int_hash_crc32(key) & mask;
    while (m->vals[p] >= 0 && m->keys[p] != key) p = (p + 1) & mask;
    if (m->vals[p] >= 0) return &m->vals[p];
    m->keys[p] = key;
    m->vals[p] = 0;
    m->size++;
    *inserted = 1;
    if (m->size > ((size_t)1 << (m->degree - 1))) { /* grower.overflow -> resize */
        hmap_resize(m);
        mask = ((size_t)1 << m->degree) - 1;
        p = int_hash_crc32(key) & mask;
        while (m->keys[p] != key || m->vals[p] < 0) p = (p + 1) & mask;
    }
    return &m->vals[p];
}
static const int64_t *hmap_find(const hmap *m, uint64_t key)
{
    if (key == 0) return m->has_zero ? &m->zero_val : NULL;
    size_t mask = ((size_t)1 << m->degree) - 1;
    size_t p = int_hash_crc32(key) & mask;
    while (m->vals[p] >= 0) {
        if (m->keys[p] == key) return &m->vals[p];
        p = (p + 1) & mask;
    }
    return NULL;
}

/* ------------------------------------------------------------------ Aggregator */
#define ORC_MAX_AGGS 8
struct orc_agg {
    int key_type; /* 0 = without_key */
    int n_aggs;
    int kinds[ORC_MAX_AGGS];
    int arg_types[ORC_MAX_AGGS];
    hmap map;
    size_t n_groups, cap_groups;
    uint64_t *gkeys;
    uint8_t *gkey_null;
    int prec[ORC_MAX_AGGS];       /* Decimal argument precision (0: the type's maximum) */
    int wide[ORC_MAX_AGGS];       /* sum result is Decimal256 (SumDecimalInferer: p + 22 > 38) */
    __int128 *acc_i[ORC_MAX_AGGS]; /* integer / decimal accumulators (wrap per result width) */
    uint64_t *acc_w[ORC_MAX_AGGS]; /* Decimal256 accumulators: 4 little-endian limbs per group */
    double *acc_f[ORC_MAX_AGGS];
    uint64_t *cnt[ORC_MAX_AGGS]; /* non-NULL rows seen */
    int coll[ORC_MAX_AGGS];       /* String min / max: the collator (TFG_ARG_COLLATOR) */
    uint8_t **sval[ORC_MAX_AGGS]; /* String min / max / first_row: the value's bytes with its '\0' */
    size_t *slen[ORC_MAX_AGGS];
    uint8_t *fnull[ORC_MAX_AGGS]; /* first_row: the first row was NULL (AggregateFunctionFirstRowNull flag 2) */
    int64_t null_group;           /* group index of the NULL key, -1 */
};

/* Result precision of sum(Decimal(p, s)): SumDecimalInferer::infer (Common/Decimal.h:156-163),
 * min(p + 22, 65); the result is Decimal256 above 38 digits (createDecimal, DataTypes/DataTypeDecimal.h). */
static int decimal_max_prec(int t)
{
    return t == TFG_DECIMAL32 ? 9 : t == TFG_DECIMAL64 ? 18 : t == TFG_DECIMAL128 ? 38 : 65;
}
static int is_decimal_t(int t)
{
    return t == TFG_DECIMAL32 || t == TFG_DECIMAL64 || t == TFG_DECIMAL128 || t == TFG_DECIMAL256;
}
int orc_sum_result_prec(int arg_type_word)
{
    const int t = arg_type_word & 0xFF;
    int p = (arg_type_word >> 16) & 0xFF;
    if (!is_decimal_t(t)) return 0;
    if (p == 0) p = decimal_max_prec(t);
    return p + 22 < 65 ? p + 22 : 65;
}

/* 256-bit two's complement add (boost checked_int256_t sums: exact below 2^255) */
static void add256(uint64_t *acc, const uint64_t *x)
{
    unsigned __int128 c = 0;
    for (int k = 0; k < 4; ++k) {
        c += (unsigned __int128)acc[k] + x[k];
        acc[k] = (uint64_t)c;
        c >>= 64;
    }
}
static void load_i256(int t, const void *p, size_t i, uint64_t *x)
{
    if (t == TFG_DECIMAL256) {
        memcpy(x, (const char *)p + 32 * i, 32);
        return;
    }
    __int128 v = load_i128(t, p, i);
    x[0] = (uint64_t)v;
    x[1] = (uint64_t)((unsigned __int128)v >> 64);
    x[2] = x[3] = v < 0 ? ~0ull : 0ull;
}

static int64_t agg_new_group(orc_agg *a, uint64_t key, uint8_t is_null);
orc_agg *orc_agg_create(int key_type, int n_aggs, const int *kinds, const int *arg_types)
{
    if (n_aggs > ORC_MAX_AGGS) return NULL;
    orc_agg *a = (orc_agg *)calloc(1, sizeof(orc_agg));
    a->key_type = key_type;
    a->n_aggs = n_aggs;
    for (int i = 0; i < n_aggs; ++i) {
        const int w = arg_types ? arg_types[i] : 0;
        a->kinds[i] = kinds[i];
        a->arg_types[i] = w & 0xFF;
        a->prec[i] = (w >> 16) & 0xFF;
        a->coll[i] = (w >> 24) & 0x7F;
        a->wide[i] = kinds[i] == TFG_AGG_SUM && orc_sum_result_prec(w) > 38;
    }
    hmap_init(&a->map);
    a->null_group = -1;
    /* without key the one group exists before any row (Aggregator::convertToBlocks emits it for an
     * empty input: without_key states are created up front, Aggregator.cpp:1132-1160) */
    if (key_type == 0) agg_new_group(a, 0, 0);
    return a;
}

void orc_agg_destroy(orc_agg *a)
{
    if (!a) return;
    hmap_free(&a->map);
    free(a->gkeys);
    free(a->gkey_null);
    for (int i = 0; i < a->n_aggs; ++i) {
        free(a->acc_i[i]);
        free(a->acc_w[i]);
        free(a->acc_f[i]);
        free(a->cnt[i]);
        if (a->sval[i])
            for (size_t g = 0; g < a->n_groups; ++g) free(a->sval[i][g]);
        free(a->sval[i]);
        free(a->slen[i]);
        free(a->fnull[i]);
    }
    free(a);
}

static int64_t agg_new_group(orc_agg *a, uint64_t key, uint8_t is_null)
{
    if (a->n_groups == a->cap_groups) {
        size_t nc = a->cap_groups ? a->cap_groups * 2 : 1024;
        a->gkeys = (uint64_t *)realloc(a->gkeys, nc * sizeof(uint64_t));
        a->gkey_null = (uint8_t *)realloc(a->gkey_null, nc);
        for (int i = 0; i < a->n_aggs; ++i) {
            a->acc_i[i] = (__int128 *)realloc(a->acc_i[i], nc * sizeof(__int128));
            a->acc_w[i] = (uint64_t *)realloc(a->acc_w[i], nc * 4 * sizeof(uint64_t));
            a->acc_f[i] = (double *)realloc(a->acc_f[i], nc * sizeof(double));
            a->cnt[i] = (uint64_t *)realloc(a->cnt[i], nc * sizeof(uint64_t));
            a->sval[i] = (uint8_t **)realloc(a->sval[i], nc * sizeof(uint8_t *));
            a->slen[i] = (size_t *)realloc(a->slen[i], nc * sizeof(size_t));
            a->fnull[i] = (uint8_t *)realloc(a->fnull[i], nc);
        }
        a->cap_groups = nc;
    }
    size_t g = a->n_groups++;
    a->gkeys[g] = key;
    a->gkey_null[g] = is_null;
    for (int i = 0; i < a->n_aggs; ++i) { /* createAggregateStates: zero-initialised sums */
        a->acc_i[i][g] = 0;
        memset(a->acc_w[i] + 4 * g, 0, 32);
        a->acc_f[i][g] = 0.0;
        a->cnt[i][g] = 0;
        a->sval[i][g] = NULL;
        a->slen[i][g] = 0;
        a->fnull[i][g] = 0;
    }
    return (int64_t)g;
}

static int64_t agg_lookup(orc_agg *a, uint64_t key, int is_null)
{
    if (a->key_type == 0) { /* without_key: one group */
        if (a->n_groups == 0) agg_new_group(a, 0, 0);
        return 0;
    }
    if (is_null) { /* nullable key: NULL is its own group */
        if (a->null_group < 0) a->null_group = agg_new_group(a, 0, 1);
        return a->null_group;
    }
    int ins;
    int64_t *slot = hmap_emplace(&a->map, key, &ins);
    if (ins) *slot = agg_new_group(a, key, 0);
    return *slot;
}

/* min / max / first_row (AggregateFunctionMinMaxAny.h: SingleValueDataFixed / SingleValueDataString
 * changeIfLess / changeIfGreater / changeFirstTime, :40-456; AggregateFunctionFirstRowData): the value
 * is kept in acc_i (integers and Decimal32..128, as __int128), acc_w (Decimal256, 4 limbs), acc_f
 * (floats) or sval / slen (String: the row's bytes with its terminating zero, as
 * getDataAtWithTerminatingZero hands them to the state); cnt counts the rows that set or offered a
 * value, and fnull records "the first row was NULL" for first_row (AggregateFunctionFirstRowNull,
 * flag 2: a NULL first row makes the result NULL and later rows do not replace it). */
static int is_ord_kind(int k) { return k == TFG_AGG_MIN || k == TFG_AGG_MAX || k == TFG_AGG_FIRST_ROW; }

/* A String argument or partial state: a host struct naming the chars and end offsets (tfg_str_col) */
typedef struct {
    const uint8_t *chars;
    const uint64_t *offsets;
} orc_str_col;
/* A String result: chars (orc_agg_result_chars bytes) and end offsets */
typedef struct {
    uint8_t *chars;
    uint64_t *offsets;
} orc_str_out;

/* GeneralCICollator::compare (TiDB/Collation/Collator.cpp:395-413): RightTrim both, then the
 * characters' weights pairwise; a proper prefix orders first */
static int gci_compare(const uint8_t *s1, size_t l1, const uint8_t *s2, size_t l2)
{
    while (l1 > 0 && s1[l1 - 1] == ' ') --l1;
    while (l2 > 0 && s2[l2 - 1] == ' ') --l2;
    size_t o1 = 0, o2 = 0;
    while (o1 < l1 && o2 < l2) {
        const int w1 = (int)orc_general_ci_weight(orc_utf8_next(s1, l1, &o1));
        const int w2 = (int)orc_general_ci_weight(orc_utf8_next(s2, l2, &o2));
        if (w1 != w2) return w1 < w2 ? -1 : 1;
    }
    return (o1 < l1) - (o2 < l2);
}
/* UCACICollator::weight (Collator.cpp:653-676): the next weight word, decoding characters only when
 * both words are spent (zero-weight characters skipped) */
static void uca_next(int v0900, uint64_t *first, uint64_t *second, size_t *off, size_t len, const uint8_t *s)
{
    if (*first != 0) return;
    if (*second != 0) {
        *first = *second;
        *second = 0;
        return;
    }
    while (*off < len)
        if (orc_uca_weight(v0900, orc_utf8_next(s, len, off), first, second)) break;
}
/* UCACICollator::compare (Collator.cpp:536-578): preprocess (RightTrim with padding), then the
 * weight words 16-bit chunk by chunk from the low end; an exhausted side (word 0) decides */
static int uca_compare(int v0900, const uint8_t *s1, size_t l1, const uint8_t *s2, size_t l2)
{
    if (!v0900) {
        while (l1 > 0 && s1[l1 - 1] == ' ') --l1;
        while (l2 > 0 && s2[l2 - 1] == ' ') --l2;
    }
    size_t o1 = 0, o2 = 0;
    uint64_t f1 = 0, x1 = 0, f2 = 0, x2 = 0;
    for (;;) {
        uca_next(v0900, &f1, &x1, &o1, l1, s1);
        uca_next(v0900, &f2, &x2, &o2, l2, s2);
        if (f1 == 0 || f2 == 0) return f1 < f2 ? -1 : f1 > f2 ? 1 : 0;
        if (f1 == f2) {
            f1 = f2 = 0;
            continue;
        }
        while (f1 != 0 && f2 != 0) {
            if (((f1 ^ f2) & 0xFFFF) == 0) {
                f1 >>= 16;
                f2 >>= 16;
            } else {
                return (int)(f1 & 0xFFFF) < (int)(f2 & 0xFFFF) ? -1 : 1;
            }
        }
    }
}
/* SingleValueDataString::less / greater (AggregateFunctionMinMaxAny.h:218-230) over two values WITH
 * their terminating zero: the collator's compareFastPath (Collator.h:91-98: padding binary
 * collators RtrimStrCompare, else compare()); without a collator StringRef operator< (memcmp of
 * the common prefix, then the size).  The '\0' ends every value, so the padding trims stop there. */
int orc_min_max_str_compare(int collator, const uint8_t *a, size_t la, const uint8_t *b, size_t lb)
{
    if (collator == TFG_COLLATOR_GENERAL_CI) return gci_compare(a, la, b, lb);
    if (collator == TFG_COLLATOR_UNICODE_CI || collator == TFG_COLLATOR_UCA0900_AI_CI)
        return uca_compare(collator == TFG_COLLATOR_UCA0900_AI_CI, a, la, b, lb);
    if (collator == TFG_COLLATOR_BIN_PADDING) {
        while (la > 0 && a[la - 1] == ' ') --la;
        while (lb > 0 && b[lb - 1] == ' ') --lb;
    }
    const size_t m = la < lb ? la : lb;
    const int c = m ? memcmp(a, b, m) : 0;
    if (c) return c < 0 ? -1 : 1;
    return la < lb ? -1 : la > lb ? 1 : 0;
}

static int cmp256(const uint64_t *x, const uint64_t *y)
{
    if ((int64_t)x[3] != (int64_t)y[3]) return (int64_t)x[3] < (int64_t)y[3] ? -1 : 1;
    for (int k = 2; k >= 0; --k)
        if (x[k] != y[k]) return x[k] < y[k] ? -1 : 1;
    return 0;
}
static void str_row(const void *p, size_t r, const uint8_t **s, size_t *len)
{
    const orc_str_col *c = (const orc_str_col *)p;
    const uint64_t b = r ? c->offsets[r - 1] : 0, e = c->offsets[r];
    *s = c->chars + b;
    *len = e - b; /* with the '\0' */
}
/* the state of group g takes row r of column p */
static void ord_set_row(orc_agg *a, int i, int64_t g, int t, const void *p, size_t r)
{
    if (t == TFG_STRING) {
        const uint8_t *v;
        size_t len;
        str_row(p, r, &v, &len);
        free(a->sval[i][g]);
        a->sval[i][g] = (uint8_t *)malloc(len ? len : 1);
        memcpy(a->sval[i][g], v, len);
        a->slen[i][g] = len;
    } else if (t == TFG_DECIMAL256) {
        memcpy(a->acc_w[i] + 4 * g, (const char *)p + 32 * r, 32);
    } else if (is_float(t)) {
        a->acc_f[i][g] = load_f(t, p, r);
    } else {
        a->acc_i[i][g] = is_unsigned(t) ? (__int128)(uint64_t)load_s(t, p, r) : load_i128(t, p, r);
    }
}
/* row r of column p against group g's value: -1 / 0 / 1 */
static int ord_cmp_row(const orc_agg *a, int i, int64_t g, int t, const void *p, size_t r)
{
    if (t == TFG_STRING) {
        const uint8_t *v;
        size_t len;
        str_row(p, r, &v, &len);
        return orc_min_max_str_compare(a->coll[i], v, len, a->sval[i][g], a->slen[i][g]);
    }
    if (t == TFG_DECIMAL256) return cmp256((const uint64_t *)((const char *)p + 32 * r), a->acc_w[i] + 4 * g);
    if (is_float(t)) {
        const double v = load_f(t, p, r), cur = a->acc_f[i][g];
        return v < cur ? -1 : v > cur ? 1 : 0;
    }
    const __int128 v = is_unsigned(t) ? (__int128)(uint64_t)load_s(t, p, r) : load_i128(t, p, r), cur = a->acc_i[i][g];
    return v < cur ? -1 : v > cur ? 1 : 0;
}
static void ord_offer(orc_agg *a, int i, int64_t g, int t, const void *p, size_t r, int is_null)
{
    const int k = a->kinds[i];
    if (k == TFG_AGG_FIRST_ROW) {
        if (a->cnt[i][g] || a->fnull[i][g]) return; /* changeFirstTime: only the first row */
        if (is_null) { a->fnull[i][g] = 1; return; }
        ord_set_row(a, i, g, t, p, r);
        a->cnt[i][g] = 1;
        return;
    }
    if (is_null) return; /* AggregateFunctionNullUnary skips NULL rows */
    const int c = a->cnt[i][g] ? ord_cmp_row(a, i, g, t, p, r) : 0;
    if (!a->cnt[i][g] || (k == TFG_AGG_MIN ? c < 0 : c > 0)) ord_set_row(a, i, g, t, p, r); /* strict */
    a->cnt[i][g]++;
}
/* dst group d takes src group g's value */
static void ord_copy(orc_agg *dst, int i, int64_t d, const orc_agg *src, int64_t g)
{
    dst->acc_i[i][d] = src->acc_i[i][g];
    dst->acc_f[i][d] = src->acc_f[i][g];
    memcpy(dst->acc_w[i] + 4 * d, src->acc_w[i] + 4 * g, 32);
    if (src->sval[i][g]) {
        free(dst->sval[i][d]);
        dst->sval[i][d] = (uint8_t *)malloc(src->slen[i][g] ? src->slen[i][g] : 1);
        memcpy(dst->sval[i][d], src->sval[i][g], src->slen[i][g]);
        dst->slen[i][d] = src->slen[i][g];
    }
}
/* merge of one group's state (changeIfLess(to) / changeIfGreater(to) / changeFirstTime(to)) */
static void ord_merge(orc_agg *dst, int i, int64_t d, const orc_agg *src, int64_t g)
{
    const int k = dst->kinds[i], t = dst->arg_types[i];
    const int dh = dst->cnt[i][d] != 0 || dst->fnull[i][d], sh = src->cnt[i][g] != 0 || src->fnull[i][g];
    if (!sh) return;
    if (k == TFG_AGG_FIRST_ROW) {
        if (dh) return;
        dst->cnt[i][d] = src->cnt[i][g];
        dst->fnull[i][d] = src->fnull[i][g];
        ord_copy(dst, i, d, src, g);
        return;
    }
    int take = !dst->cnt[i][d];
    if (!take) {
        int c;
        if (t == TFG_STRING)
            c = orc_min_max_str_compare(dst->coll[i], src->sval[i][g], src->slen[i][g], dst->sval[i][d], dst->slen[i][d]);
        else if (t == TFG_DECIMAL256)
            c = cmp256(src->acc_w[i] + 4 * g, dst->acc_w[i] + 4 * d);
        else if (is_float(t))
            c = src->acc_f[i][g] < dst->acc_f[i][d] ? -1 : src->acc_f[i][g] > dst->acc_f[i][d] ? 1 : 0;
        else
            c = src->acc_i[i][g] < dst->acc_i[i][d] ? -1 : src->acc_i[i][g] > dst->acc_i[i][d] ? 1 : 0;
        take = k == TFG_AGG_MIN ? c < 0 : c > 0;
    }
    if (take) ord_copy(dst, i, d, src, g);
    dst->cnt[i][d] += src->cnt[i][g];
}

/* Aggregator::executeOnBlock -> handleOneBatch (Interpreters/Aggregator.cpp:852-1024):
 * emplace key, then IAggregateFunction::addBatch in row order (IAggregateFunction.h:242-266);
 * AggregateFunctionSumData::add (AggregateFunctionSum.h:64-80); count (AggregateFunctionCount.h:46);
 * Nullable arguments skip NULL rows (AggregateFunctionNull.h:373). */
void orc_agg_consume(orc_agg *a, const void *keys, const uint8_t *key_null, const void *const *args,
                     const uint8_t *const *arg_nulls, const uint8_t *mask, size_t n)
{
    for (size_t r = 0; r < n; ++r) {
        if (mask && !mask[r]) continue;
        int kn = key_null && key_null[r];
        uint64_t key = (a->key_type && !kn) ? load_key_bits(a->key_type, keys, r) : 0;
        int64_t g = agg_lookup(a, key, kn);
        for (int i = 0; i < a->n_aggs; ++i) {
            if (a->kinds[i] == TFG_AGG_COUNT_ALL) { a->cnt[i][g]++; continue; }
            if (is_ord_kind(a->kinds[i])) {
                ord_offer(a, i, g, a->arg_types[i], args[i], r, arg_nulls && arg_nulls[i] && arg_nulls[i][r]);
                continue;
            }
            if (arg_nulls && arg_nulls[i] && arg_nulls[i][r]) continue;
            a->cnt[i][g]++;
            if (a->kinds[i] == TFG_AGG_COUNT) continue;
            int t = a->arg_types[i];
            if (is_float(t)) a->acc_f[i][g] += load_f(t, args[i], r);
            else if (a->wide[i]) {
                uint64_t x[4];
                load_i256(t, args[i], r, x);
                add256(a->acc_w[i] + 4 * g, x);
            } else a->acc_i[i][g] = (__int128)((unsigned __int128)a->acc_i[i][g] + (unsigned __int128)load_i128(t, args[i], r));
        }
    }
}

/* mergeDataImpl (Aggregator.cpp:2338-2363): add src states into dst, src groups in src order. */
void orc_agg_merge(orc_agg *dst, const orc_agg *src)
{
    for (size_t g = 0; g < src->n_groups; ++g) {
        int64_t d = agg_lookup(dst, src->gkeys[g], src->gkey_null[g]);
        for (int i = 0; i < dst->n_aggs; ++i) {
            if (is_ord_kind(dst->kinds[i])) {
                ord_merge(dst, i, d, src, g);
                continue;
            }
            dst->cnt[i][d] += src->cnt[i][g];
            dst->acc_f[i][d] += src->acc_f[i][g];
            dst->acc_i[i][d] = (__int128)((unsigned __int128)dst->acc_i[i][d] + (unsigned __int128)src->acc_i[i][g]);
            add256(dst->acc_w[i] + 4 * d, src->acc_w[i] + 4 * g);
        }
    }
}

size_t orc_agg_size(const orc_agg *a) { return a->n_groups; }

/* chars bytes of the String result of aggregate i (orc_agg_result writes them) */
size_t orc_agg_result_chars(const orc_agg *a, int i)
{
    size_t b = 0;
    for (size_t g = 0; g < a->n_groups; ++g) b += a->cnt[i][g] ? a->slen[i][g] : 1;
    return b;
}

static int sum_result_width(const orc_agg *a, int i)
{
    return a->wide[i] ? 32 : is_decimal_t(a->arg_types[i]) ? 16 : 8;
}

/* insertAggregatesIntoColumns (Aggregator.cpp:1651-1780). Order: group creation order. */
void orc_agg_result(const orc_agg *a, uint64_t *out_keys, uint8_t *out_key_null, void *const *out_states,
                    uint8_t *const *out_state_null)
{
    for (size_t g = 0; g < a->n_groups; ++g) {
        if (out_keys) out_keys[g] = a->gkeys[g];
        if (out_key_null) out_key_null[g] = a->gkey_null[g];
        for (int i = 0; i < a->n_aggs; ++i) {
            if (out_state_null && out_state_null[i]) out_state_null[i][g] = a->cnt[i][g] == 0;
            if (!out_states || !out_states[i]) continue;
            if (is_ord_kind(a->kinds[i])) { /* the argument's type and width */
                const int t = a->arg_types[i];
                char *o = (char *)out_states[i];
                if (t == TFG_STRING) { /* an orc_str_out; NULL / no value: the empty String */
                    orc_str_out *so = (orc_str_out *)out_states[i];
                    const uint64_t start = g ? so->offsets[g - 1] : 0;
                    const size_t len = a->cnt[i][g] ? a->slen[i][g] : 1;
                    if (a->cnt[i][g]) memcpy(so->chars + start, a->sval[i][g], len);
                    else so->chars[start] = 0;
                    so->offsets[g] = start + len;
                } else if (t == TFG_DECIMAL256) memcpy(o + 32 * g, a->acc_w[i] + 4 * g, 32);
                else if (t == TFG_DECIMAL128) memcpy(o + 16 * g, &a->acc_i[i][g], 16);
                else if (t == TFG_FLOAT64) ((double *)o)[g] = a->acc_f[i][g];
                else if (t == TFG_FLOAT32) ((float *)o)[g] = (float)a->acc_f[i][g];
                else {
                    const int64_t v = (int64_t)a->acc_i[i][g];
                    switch (t) {
                    case TFG_INT8: case TFG_UINT8: ((uint8_t *)o)[g] = (uint8_t)v; break;
                    case TFG_INT16: case TFG_UINT16: ((uint16_t *)o)[g] = (uint16_t)v; break;
                    case TFG_INT32: case TFG_UINT32: case TFG_DECIMAL32: ((uint32_t *)o)[g] = (uint32_t)v; break;
                    default: ((int64_t *)o)[g] = v; break;
                    }
                }
                continue;
            }
            if (a->kinds[i] != TFG_AGG_SUM) { ((uint64_t *)out_states[i])[g] = a->cnt[i][g]; continue; }
            int t = a->arg_types[i];
            if (is_float(t)) ((double *)out_states[i])[g] = a->acc_f[i][g];
            else if (sum_result_width(a, i) == 32) memcpy((char *)out_states[i] + 32 * g, a->acc_w[i] + 4 * g, 32);
            else if (sum_result_width(a, i) == 16) memcpy((char *)out_states[i] + 16 * g, &a->acc_i[i][g], 16);
            else ((int64_t *)out_states[i])[g] = (int64_t)a->acc_i[i][g];
        }
    }
}

/* ------------------------------------------------------------------ Aggregator, several keys / String key */
/* Methods keys128 / nullable_keys128 / key_string / serialized (Interpreters/Aggregator.cpp:394-537,
 * Common/ColumnsHashing.h:179-629): every method groups rows by the tuple of key values, a NULL
 * key value being its own value, and a String key by its collator sort key
 * (HashMethodString::getKeyHolder, ColumnsHashing.h:224-236; BIN padding = right-trim ' ').  The
 * restatement serialises each row's tuple like the serialized method (serializeValueIntoArena):
 * per key one NULL byte, then the fixed value's bytes or an 8-byte length + the sort-key bytes;
 * the bytes map to a dense group id (first-seen order) through a byte-string hash map, and the
 * states live in an inner orc_agg keyed by that id. */
struct orc_aggk {
    int nkeys;
    int key_types[8];
    int collators[8];
    /* byte-string map: open addressing over (hash, id) cells; keys in one arena */
    uint64_t *cells; /* (crc << 32) | (id + 1), 0 = empty */
    size_t cap, size;
    uint8_t *arena;
    size_t arena_len, arena_cap;
    uint64_t *key_off; /* id -> arena offset, id + 1 -> end */
    size_t key_cap;
    orc_agg *inner;
    uint32_t *ids;
    size_t ids_cap;
};

static uint32_t bytes_hash(const uint8_t *p, size_t n) { return orc_update_weak_hash32_bytes(p, n, 0xFFFFFFFFu); }

orc_aggk *orc_aggk_create(int nkeys, const int *key_types, const int *collators, int n_aggs, const int *kinds,
                          const int *arg_types)
{
    if (nkeys < 1 || nkeys > 8) return NULL;
    orc_aggk *a = (orc_aggk *)calloc(1, sizeof(orc_aggk));
    a->nkeys = nkeys;
    for (int j = 0; j < nkeys; ++j) {
        a->key_types[j] = key_types[j];
        a->collators[j] = collators ? collators[j] : 0;
    }
    a->cap = 1024;
    a->cells = (uint64_t *)calloc(a->cap, 8);
    a->key_cap = 1024;
    a->key_off = (uint64_t *)malloc(a->key_cap * 8);
    a->key_off[0] = 0;
    a->inner = orc_agg_create(TFG_UINT32, n_aggs, kinds, arg_types);
    return a;
}

void orc_aggk_destroy(orc_aggk *a)
{
    if (!a) return;
    free(a->cells);
    free(a->arena);
    free(a->key_off);
    free(a->ids);
    orc_agg_destroy(a->inner);
    free(a);
}

static void aggk_grow(orc_aggk *a)
{
    size_t nc = a->cap * 2;
    uint64_t *c = (uint64_t *)calloc(nc, 8);
    for (size_t i = 0; i < a->cap; ++i) {
        if (!a->cells[i]) continue;
        size_t p = (a->cells[i] >> 32) & (nc - 1);
        while (c[p]) p = (p + 1) & (nc - 1);
        c[p] = a->cells[i];
    }
    free(a->cells);
    a->cells = c;
    a->cap = nc;
}

static uint32_t aggk_id(orc_aggk *a, const uint8_t *k, size_t len)
{
    const uint32_t h = bytes_hash(k, len);
    size_t p = h & (a->cap - 1);
    for (;; p = (p + 1) & (a->cap - 1)) {
        const uint64_t c = a->cells[p];
        if (!c) break;
        if ((uint32_t)(c >> 32) != h) continue;
        const uint32_t id = (uint32_t)c - 1;
        if (a->key_off[id + 1] - a->key_off[id] == len && !memcmp(a->arena + a->key_off[id], k, len)) return id;
    }
    const uint32_t id = (uint32_t)a->size++;
    a->cells[p] = ((uint64_t)h << 32) | (id + 1);
    if (a->arena_len + len > a->arena_cap) {
        a->arena_cap = (a->arena_len + len) * 2 + 4096;
        a->arena = (uint8_t *)realloc(a->arena, a->arena_cap);
    }
    memcpy(a->arena + a->arena_len, k, len);
    a->arena_len += len;
    if (id + 2 > a->key_cap) {
        a->key_cap *= 2;
        a->key_off = (uint64_t *)realloc(a->key_off, a->key_cap * 8);
    }
    a->key_off[id + 1] = a->arena_len;
    if (a->size * 2 > a->cap) aggk_grow(a);
    return id;
}

/* serialise row r's key tuple into buf (<= 4 keys x (1 + 16) bytes, or 9 + string length) */
static size_t aggk_serialize(const orc_aggk *a, const void *const *cols, const uint64_t *const *offs,
                             const uint8_t *const *nulls, size_t r, uint8_t **buf, size_t *bcap)
{
    size_t need = 0;
    for (int j = 0; j < a->nkeys; ++j) {
        if (a->key_types[j] == TFG_STRING) need += 9 + ORC_KEY_MULT * (offs[j][r] - (r ? offs[j][r - 1] : 0));
        else need += 17;
    }
    if (need > *bcap) {
        *bcap = need * 2;
        *buf = (uint8_t *)realloc(*buf, *bcap);
    }
    uint8_t *o = *buf;
    for (int j = 0; j < a->nkeys; ++j) {
        const int isnull = nulls && nulls[j] && nulls[j][r];
        *o++ = (uint8_t)isnull;
        if (isnull) continue;
        if (a->key_types[j] == TFG_STRING) {
            const uint64_t s = r ? offs[j][r - 1] : 0;
            uint64_t len = offs[j][r] - s - 1;
            const uint8_t *c = (const uint8_t *)cols[j] + s;
            if (orc_collator_transforms(a->collators[j])) { /* the sort key, written in place */
                const uint64_t kl = orc_collate(a->collators[j], c, len, len + 1, o + 8);
                memcpy(o, &kl, 8);
                o += 8 + kl;
                continue;
            }
            if (a->collators[j] == TFG_COLLATOR_BIN_PADDING)
                while (len > 0 && c[len - 1] == ' ') --len;
            memcpy(o, &len, 8);
            memcpy(o + 8, c, len);
            o += 8 + len;
        } else {
            const size_t w = type_width(a->key_types[j]);
            memcpy(o, (const uint8_t *)cols[j] + w * r, w);
            o += w;
        }
    }
    return (size_t)(o - *buf);
}

static uint32_t *aggk_ids(orc_aggk *a, const void *const *key_cols, const uint64_t *const *key_offsets,
                          const uint8_t *const *key_nulls, const uint8_t *mask, size_t n)
{
    if (n > a->ids_cap) {
        a->ids_cap = n;
        a->ids = (uint32_t *)realloc(a->ids, n * 4);
    }
    uint8_t *buf = NULL;
    size_t bcap = 0;
    for (size_t r = 0; r < n; ++r) {
        if (mask && !mask[r]) { a->ids[r] = 0; continue; }
        size_t len = aggk_serialize(a, key_cols, key_offsets, key_nulls, r, &buf, &bcap);
        a->ids[r] = aggk_id(a, buf, len);
    }
    free(buf);
    return a->ids;
}

void orc_aggk_consume(orc_aggk *a, const void *const *key_cols, const uint64_t *const *key_offsets,
                      const uint8_t *const *key_nulls, const void *const *args, const uint8_t *const *arg_nulls,
                      const uint8_t *mask, size_t n)
{
    uint32_t *ids = aggk_ids(a, key_cols, key_offsets, key_nulls, mask, n);
    orc_agg_consume(a->inner, ids, NULL, args, arg_nulls, mask, n);
}

size_t orc_aggk_size(const orc_aggk *a) { return orc_agg_size(a->inner); }
size_t orc_aggk_result_chars(const orc_aggk *a, int i) { return orc_agg_result_chars(a->inner, i); }

/* groups in creation order: serialized keys (out_keys: arena bytes, out_key_offsets: end offsets,
 * pass NULL to get the byte count first) and states as orc_agg_result. */
size_t orc_aggk_result(const orc_aggk *a, uint8_t *out_keys, uint64_t *out_key_offsets, void *const *out_states,
                       uint8_t *const *out_state_null)
{
    const size_t g = orc_agg_size(a->inner);
    uint64_t *ids = (uint64_t *)malloc((g ? g : 1) * 8);
    orc_agg_result(a->inner, ids, NULL, out_states, out_state_null);
    size_t total = 0;
    for (size_t i = 0; i < g; ++i) {
        const uint64_t id = ids[i], s = a->key_off[id], e = a->key_off[id + 1];
        if (out_keys) memcpy(out_keys + total, a->arena + s, e - s);
        total += e - s;
        if (out_key_offsets) out_key_offsets[i] = total;
    }
    free(ids);
    return total;
}

/* ------------------------------------------------------------------ Join (hash join v1) */
/* MapsAll = HashMap<UInt64, RowRefList, HashCRC32<UInt64>> (Interpreters/JoinHashMap.h:175-188).
 * Inserter<All>::insert (JoinPartition.cpp:494-524): the first row of a key lives in the cell; every
 * later row is inserted SECOND in the list (insertRowToList, :39-60), so iteration order is
 * first, then newest ... oldest. */
struct orc_join {
    int key_type;
    hmap map; /* key -> list id */
    size_t n_lists, cap_lists;
    int64_t *first, *after; /* per list: head row, most recent non-head row (-1) */
    size_t n_rows, cap_rows;
    int64_t *next; /* per build row: next row in list (-1) */
};

orc_join *orc_join_create(int key_type)
{
    orc_join *j = (orc_join *)calloc(1, sizeof(orc_join));
    j->key_type = key_type;
    hmap_init(&j->map);
    return j;
}

void orc_join_destroy(orc_join *j)
{
    if (!j) return;
    hmap_free(&j->map);
    free(j->first);
    free(j->after);
    free(j->next);
    free(j);
}

/* insertBlockIntoMapsTypeCase (JoinPartition.cpp:584-728); NULL keys are not inserted
 * (extractNestedColumnsAndNullMap, Join.cpp:686). Row ids continue across calls. */
void orc_join_build(orc_join *j, const void *keys, const uint8_t *key_null, size_t n)
{
    if (j->n_rows + n > j->cap_rows) {
        size_t nc = (j->n_rows + n) * 2;
        j->next = (int64_t *)realloc(j->next, nc * sizeof(int64_t));
        j->cap_rows = nc;
    }
    for (size_t r = 0; r < n; ++r) {
        int64_t row = (int64_t)(j->n_rows + r);
        j->next[row] = -1;
        if (key_null && key_null[r]) continue;
        uint64_t key = load_key_bits(j->key_type, keys, r);
        int ins;
        int64_t *slot = hmap_emplace(&j->map, key, &ins);
        if (ins) {
            if (j->n_lists == j->cap_lists) {
                size_t nc = j->cap_lists ? j->cap_lists * 2 : 1024;
                j->first = (int64_t *)realloc(j->first, nc * sizeof(int64_t));
                j->after = (int64_t *)realloc(j->after, nc * sizeof(int64_t));
                j->cap_lists = nc;
            }
            *slot = (int64_t)j->n_lists;
            j->first[j->n_lists] = row;
            j->after[j->n_lists] = -1;
            j->n_lists++;
        } else {
            j->next[row] = j->after[*slot];
            j->after[*slot] = row;
        }
    }
    j->n_rows += n;
}

/* probeBlockImplTypeCase + Adder<KIND, All> (JoinPartition.cpp:1290-1378, 1465-1644): probe rows in
 * order; found -> every row of the list; not found -> inner: nothing, left: one default row
 * (build index 0xFFFFFFFF); semi: probe row once if found; anti: probe row if not found. */
size_t orc_join_probe(const orc_join *j, int kind, const void *keys, const uint8_t *key_null, size_t n,
                      uint32_t *out_probe, uint32_t *out_build, size_t capacity)
{
    size_t k = 0;
#define EMIT(p, b)                                                        \
    do {                                                                  \
        if (k < capacity) {                                               \
            if (out_probe) out_probe[k] = (uint32_t)(p);                  \
            if (out_build) out_build[k] = (uint32_t)(b);                  \
        }                                                                 \
        ++k;                                                              \
    } while (0)
    for (size_t r = 0; r < n; ++r) {
        const int64_t *slot = NULL;
        if (!(key_null && key_null[r])) slot = hmap_find(&j->map, load_key_bits(j->key_type, keys, r));
        if (!slot) {
            if (kind == TFG_JOIN_LEFT) EMIT(r, 0xFFFFFFFFu);
            else if (kind == TFG_JOIN_ANTI) EMIT(r, 0xFFFFFFFFu);
            continue;
        }
        if (kind == TFG_JOIN_ANTI) continue;
        if (kind == TFG_JOIN_SEMI) { EMIT(r, j->first[*slot]); continue; }
        EMIT(r, j->first[*slot]);
        for (int64_t b = j->after[*slot]; b >= 0; b = j->next[b]) EMIT(r, b);
    }
#undef EMIT
    return k;
}

/* ------------------------------------------------------------------ CPU baseline legs */
typedef struct {
    const int64_t *f, *k;
    const double *v;
    int64_t threshold;
    size_t begin, end, block_rows;
    orc_agg *agg;
} fa_task;

/* One source stream of the pipeline: per Block of block_rows (max_block_size, Core/Defines.h:65):
 * FilterTransformAction::transform = compare -> countBytesInFilter -> filter each column
 * (DataStreams/FilterTransformAction.cpp:72-173), then Aggregator::executeOnBlock. */
static void *fa_worker(void *arg)
{
    fa_task *t = (fa_task *)arg;
    size_t B = t->block_rows;
    uint8_t *mask = (uint8_t *)malloc(B);
    int64_t *fk = (int64_t *)malloc(B * 8);
    double *fv = (double *)malloc(B * 8);
    int64_t thr = t->threshold;
    for (size_t s = t->begin; s < t->end; s += B) {
        size_t m = t->end - s < B ? t->end - s : B;
        orc_cmp(TFG_INT64, t->f + s, 0, TFG_LT, TFG_INT64, &thr, 1, NULL, NULL, m, mask);
        size_t cnt = orc_count_bytes_in_filter(mask, NULL, m);
        if (cnt == 0) continue;
        const void *args[1];
        if (cnt == m) {
            args[0] = t->v + s;
            orc_agg_consume(t->agg, t->k + s, NULL, args, NULL, NULL, m);
        } else {
            orc_filter(8, t->k + s, mask, m, fk);
            orc_filter(8, t->v + s, mask, m, fv);
            args[0] = fv;
            orc_agg_consume(t->agg, fk, NULL, args, NULL, NULL, cnt);
        }
    }
    free(mask);
    free(fk);
    free(fv);
    return NULL;
}

size_t orc_bench_filter_agg(const int64_t *f, int64_t threshold, const int64_t *k, const double *v, size_t n,
                            int nthreads, size_t block_rows, double *checksum)
{
    if (nthreads < 1) nthreads = 1;
    int kinds[2] = {TFG_AGG_SUM, TFG_AGG_COUNT_ALL};
    int types[2] = {TFG_FLOAT64, 0};
    fa_task *tasks = (fa_task *)calloc((size_t)nthreads, sizeof(fa_task));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int i = 0; i < nthreads; ++i) {
        tasks[i].f = f;
        tasks[i].k = k;
        tasks[i].v = v;
        tasks[i].threshold = threshold;
        tasks[i].begin = per * (size_t)i < n ? per * (size_t)i : n;
        tasks[i].end = per * (size_t)(i + 1) < n ? per * (size_t)(i + 1) : n;
        tasks[i].block_rows = block_rows;
        tasks[i].agg = orc_agg_create(TFG_INT64, 2, kinds, types);
        pthread_create(&th[i], NULL, fa_worker, &tasks[i]);
    }
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    /* merge per-thread tables after the barrier */
    orc_agg *res = tasks[0].agg;
    for (int i = 1; i < nthreads; ++i) {
        orc_agg_merge(res, tasks[i].agg);
        orc_agg_destroy(tasks[i].agg);
    }
    size_t groups = orc_agg_size(res);
    double cs = 0;
    for (size_t g = 0; g < groups; ++g) cs += res->acc_f[0][g] + (double)res->cnt[1][g];
    if (checksum) *checksum = cs;
    orc_agg_destroy(res);
    free(tasks);
    free(th);
    return groups;
}

typedef struct {
    const orc_join *j;
    const int64_t *keys;
    size_t begin, end;
    size_t matches;
    uint64_t checksum;
} jp_task;

static void *jp_worker(void *arg)
{
    jp_task *t = (jp_task *)arg;
    const size_t B = 65536;
    uint32_t *pi = (uint32_t *)malloc(B * 4 * 4), *bi = (uint32_t *)malloc(B * 4 * 4);
    for (size_t s = t->begin; s < t->end; s += B) {
        size_t m = t->end - s < B ? t->end - s : B;
        size_t c = orc_join_probe(t->j, TFG_JOIN_INNER, t->keys + s, NULL, m, pi, bi, B * 4);
        for (size_t i = 0; i < c && i < B * 4; ++i) t->checksum += (uint64_t)bi[i] + (uint64_t)(pi[i] + s);
        t->matches += c;
    }
    free(pi);
    free(bi);
    return NULL;
}

size_t orc_bench_join(const int64_t *build_keys, size_t nb, const int64_t *probe_keys, size_t np, int nthreads,
                      uint64_t *checksum)
{
    orc_join *j = orc_join_create(TFG_INT64);
    orc_join_build(j, build_keys, NULL, nb);
    if (nthreads < 1) nthreads = 1;
    jp_task *tasks = (jp_task *)calloc((size_t)nthreads, sizeof(jp_task));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    size_t per = (np + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int i = 0; i < nthreads; ++i) {
        tasks[i].j = j;
        tasks[i].keys = probe_keys;
        tasks[i].begin = per * (size_t)i < np ? per * (size_t)i : np;
        tasks[i].end = per * (size_t)(i + 1) < np ? per * (size_t)(i + 1) : np;
        pthread_create(&th[i], NULL, jp_worker, &tasks[i]);
    }
    size_t total = 0;
    uint64_t cs = 0;
    for (int i = 0; i < nthreads; ++i) {
        pthread_join(th[i], NULL);
        total += tasks[i].matches;
        cs += tasks[i].checksum;
    }
    if (checksum) *checksum = cs;
    orc_join_destroy(j);
    free(tasks);
    free(th);
    return total;
}
