/*
 * cpu_baseline.c — the reference's CPU algorithm for the C2 step (filter -> GROUP BY key64 with
 * sum(Float64) + count()), restated with the reference's data structures so bench.py's
 * cpu_baseline leg times what TiFlash would do on the same host cores.
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY (see oracle.h): never linked into the product path.
 *
 * Per thread (one ParallelAggregatingBlockInputStream source, DataStreams/
 * ParallelAggregatingBlockInputStream.cpp:77-159), per Block of block_rows:
 *   FilterTransformAction::transform (DataStreams/FilterTransformAction.cpp:72-173): compare
 *     column -> countBytesInFilter -> filter each column (stable compaction);
 *   Aggregator::executeOnBlock, method key64 (Interpreters/Aggregator.cpp:852-1024):
 *     HashMap<UInt64, AggregateDataPtr, HashCRC32> — 16-byte cells (key, state pointer), linear
 *     probing from intHashCRC32(key) & mask, key 0 in a side cell (ZeroValueStorage), grower
 *     +2 degrees while < 2^23 then +1, resize when size > cap/2 (HashTable.h:254-296, 875-1000);
 *     states (sum Float64, count UInt64; 16 B) bump-allocated in an Arena on insert;
 *     prefetch of the cell 16 rows ahead once the table exceeds 2 MB (Aggregator.cpp:53,573-600);
 *     conversion to a two-level table (256 sub-tables, bucket = (hash >> 24) & 255,
 *     TwoLevelHashTable.h:71) once the table holds > group_by_two_level_threshold = 100000 keys
 *     (Interpreters/Settings.h:89).
 * After the barrier: MergingBuckets — threads take buckets from a shared counter and merge bucket
 * b of every thread's table into thread 0's (Aggregator.cpp:2940-3097), then
 * convertToBlockImplFinal writes key / sum / count columns per bucket (Aggregator.cpp:1651-1780).
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

#include "oracle.h"

static inline uint32_t crc_key(uint64_t x)
{
#if defined(__SSE4_2__)
    return (uint32_t)_mm_crc32_u64(0xFFFFFFFFull, x); /* intHashCRC32 (Hash.h:70-95) */
#else
    return orc_crc32c_u64(0xFFFFFFFFu, x);
#endif
}

typedef struct {
    double sum;
    uint64_t count;
} agg_state; /* AggregateFunctionSumData<Float64> + AggregateFunctionCountData */

typedef struct {
    uint64_t key;
    agg_state *mapped; /* NULL = empty cell */
} cell;

typedef struct {
    cell *cells;
    int degree;
    size_t size;
    agg_state *zero; /* ZeroValueStorage for key 0 */
} hmap64;

typedef struct arena_chunk {
    struct arena_chunk *prev;
    size_t used, cap;
    char data[];
} arena_chunk;

typedef struct {
    arena_chunk *head;
} arena;

static agg_state *arena_alloc_state(arena *a)
{
    if (!a->head || a->head->used + sizeof(agg_state) > a->head->cap) {
        size_t cap = a->head ? a->head->cap * 2 : 4096;
        if (cap > (64u << 20)) cap = 64u << 20;
        arena_chunk *c = (arena_chunk *)malloc(sizeof(arena_chunk) + cap);
        c->prev = a->head;
        c->used = 0;
        c->cap = cap;
        a->head = c;
    }
    agg_state *s = (agg_state *)(a->head->data + a->head->used);
    a->head->used += sizeof(agg_state);
    s->sum = 0;
    s->count = 0;
    return s;
}

static void arena_free(arena *a)
{
    while (a->head) {
        arena_chunk *p = a->head->prev;
        free(a->head);
        a->head = p;
    }
}

static void hm_init(hmap64 *m, int degree)
{
    m->degree = degree;
    m->cells = (cell *)calloc((size_t)1 << degree, sizeof(cell));
    m->size = 0;
    m->zero = NULL;
}

static void hm_free(hmap64 *m) { free(m->cells); }

static void hm_resize(hmap64 *m)
{
    const size_t old_cap = (size_t)1 << m->degree;
    cell *old = m->cells;
    m->degree += m->degree >= 23 ? 1 : 2;
    const size_t mask = ((size_t)1 << m->degree) - 1;
    m->cells = (cell *)calloc(mask + 1, sizeof(cell));
    for (size_t i = 0; i < old_cap; ++i) {
        if (!old[i].mapped) continue;
        size_t p = crc_key(old[i].key) & mask;
        while (m->cells[p].mapped) p = (p + 1) & mask;
        m->cells[p] = old[i];
    }
    free(old);
}

/* emplace with a precomputed hash; returns the state (allocated on insert) */
static inline agg_state *hm_emplace(hmap64 *m, uint64_t key, uint32_t h, arena *ar)
{
    if (key == 0) {
        if (!m->zero) m->zero = arena_alloc_state(ar);
        return m->zero;
    }
    size_t mask = ((size_t)1 << m->degree) - 1;
    size_t p = h & mask;
    while (m->cells[p].mapped && m->cells[p].key != key) p = (p + 1) & mask;
    if (m->cells[p].mapped) return m->cells[p].mapped;
    agg_state *s = arena_alloc_state(ar);
    m->cells[p].key = key;
    m->cells[p].mapped = s;
    if (++m->size > ((size_t)1 << (m->degree - 1))) hm_resize(m);
    return s;
}

#define BUCKETS 256

typedef struct {
    int two_level;
    hmap64 single;
    hmap64 sub[BUCKETS];
    arena ar;
} variants;

static void variants_init(variants *v)
{
    v->two_level = 0;
    hm_init(&v->single, 8);
    v->ar.head = NULL;
}

static void convert_to_two_level(variants *v)
{
    for (int b = 0; b < BUCKETS; ++b) hm_init(&v->sub[b], 8);
    const size_t cap = (size_t)1 << v->single.degree;
    for (size_t i = 0; i < cap; ++i) {
        const cell c = v->single.cells[i];
        if (!c.mapped) continue;
        const uint32_t h = crc_key(c.key);
        hmap64 *s = &v->sub[(h >> 24) & 255];
        size_t mask = ((size_t)1 << s->degree) - 1, p = h & mask;
        while (s->cells[p].mapped) p = (p + 1) & mask;
        s->cells[p] = c;
        if (++s->size > ((size_t)1 << (s->degree - 1))) hm_resize(s);
    }
    v->sub[(crc_key(0) >> 24) & 255].zero = v->single.zero; /* key 0: its bucket's ZeroValueStorage */
    hm_free(&v->single);
    v->two_level = 1;
}

static size_t variants_bytes(const variants *v)
{
    if (!v->two_level) return ((size_t)1 << v->single.degree) * sizeof(cell);
    size_t b = 0;
    for (int i = 0; i < BUCKETS; ++i) b += ((size_t)1 << v->sub[i].degree) * sizeof(cell);
    return b;
}

/* executeImplBatch over one filtered block: emplace + add, prefetching 16 rows ahead */
static void agg_block(variants *v, const int64_t *k, const double *x, size_t n)
{
    const int prefetch = variants_bytes(v) >= (2u << 20);
    for (size_t i = 0; i < n; ++i) {
        if (prefetch && i + 16 < n) {
            const uint32_t hp = crc_key((uint64_t)k[i + 16]);
            const hmap64 *m = v->two_level ? &v->sub[(hp >> 24) & 255] : &v->single;
            __builtin_prefetch(&m->cells[hp & (((size_t)1 << m->degree) - 1)]);
        }
        const uint64_t key = (uint64_t)k[i];
        const uint32_t h = crc_key(key);
        agg_state *s = v->two_level ? hm_emplace(&v->sub[(h >> 24) & 255], key, h, &v->ar)
                                    : hm_emplace(&v->single, key, h, &v->ar);
        s->sum += x[i];
        s->count += 1;
    }
    if (!v->two_level && v->single.size + (v->single.zero ? 1 : 0) > 100000) convert_to_two_level(v);
}

typedef struct {
    const int64_t *f, *k;
    const double *x;
    int64_t threshold;
    size_t begin, end, block_rows;
    variants var;
} src_task;

/* the typed, auto-vectorised forms the reference instantiates for Int64 (NumComparisonImpl<Int64,
 * Int64, LessOp>::vectorConstant, countBytesInFilter, filterImpl<8 B>) */
static void cmp_lt_i64(const int64_t *a, int64_t b, size_t n, uint8_t *out)
{
    for (size_t i = 0; i < n; ++i) out[i] = a[i] < b;
}

static size_t count_bytes(const uint8_t *f, size_t n)
{
    size_t c = 0;
    for (size_t i = 0; i < n; ++i) c += f[i] != 0;
    return c;
}

static size_t filter8(const void *col, const uint8_t *f, size_t n, void *out)
{
    const uint64_t *src = (const uint64_t *)col;
    uint64_t *dst = (uint64_t *)out;
    size_t k = 0, i = 0;
    for (; i + 64 <= n; i += 64) {
        uint64_t mask = 0;
        for (int b = 0; b < 64; ++b) mask |= (uint64_t)(f[i + b] != 0) << b; /* ToBits64 */
        if (mask == ~0ull) { /* prefixToCopy covers the whole group */
            memcpy(dst + k, src + i, 64 * 8);
            k += 64;
            continue;
        }
        while (mask) {
            dst[k++] = src[i + (size_t)__builtin_ctzll(mask)];
            mask &= mask - 1;
        }
    }
    for (; i < n; ++i)
        if (f[i]) dst[k++] = src[i];
    return k;
}

static void *src_worker(void *arg)
{
    src_task *t = (src_task *)arg;
    const size_t B = t->block_rows;
    uint8_t *mask = (uint8_t *)malloc(B);
    int64_t *fk = (int64_t *)malloc(B * 8);
    double *fx = (double *)malloc(B * 8);
    const int64_t thr = t->threshold;
    variants_init(&t->var);
    for (size_t s = t->begin; s < t->end; s += B) {
        const size_t m = t->end - s < B ? t->end - s : B;
        /* FilterTransformAction: NumComparisonImpl::vectorConstant -> countBytesInFilter -> filter */
        cmp_lt_i64(t->f + s, thr, m, mask);
        const size_t cnt = count_bytes(mask, m);
        if (cnt == 0) continue;
        if (cnt == m) {
            agg_block(&t->var, t->k + s, t->x + s, m);
        } else {
            filter8(t->k + s, mask, m, fk);
            filter8(t->x + s, mask, m, fx);
            agg_block(&t->var, fk, fx, cnt);
        }
    }
    free(mask);
    free(fk);
    free(fx);
    return NULL;
}

typedef struct {
    src_task *tasks;
    int nthreads;
    atomic_int next_bucket;
    uint64_t *out_keys;
    double *out_sum;
    uint64_t *out_cnt;
    size_t *bucket_off; /* filled after merge */
    int phase;          /* 0 merge, 1 convert */
} merge_ctx;

typedef struct {
    merge_ctx *mc;
} merge_arg;

static void merge_bucket(merge_ctx *mc, int b)
{
    hmap64 *dst = &mc->tasks[0].var.sub[b]; /* states move by pointer: no allocation while merging */
    for (int t = 1; t < mc->nthreads; ++t) {
        hmap64 *src = &mc->tasks[t].var.sub[b];
        const size_t cap = (size_t)1 << src->degree;
        for (size_t i = 0; i < cap; ++i) {
            const cell c = src->cells[i];
            if (!c.mapped) continue;
            const uint32_t h = crc_key(c.key);
            size_t mask = ((size_t)1 << dst->degree) - 1, p = h & mask;
            while (dst->cells[p].mapped && dst->cells[p].key != c.key) p = (p + 1) & mask;
            if (dst->cells[p].mapped) {
                dst->cells[p].mapped->sum += c.mapped->sum;
                dst->cells[p].mapped->count += c.mapped->count;
            } else { /* the source's state moves over (no new allocation) */
                dst->cells[p] = c;
                if (++dst->size > ((size_t)1 << (dst->degree - 1))) hm_resize(dst);
            }
        }
        if (src->zero) {
            if (dst->zero) {
                dst->zero->sum += src->zero->sum;
                dst->zero->count += src->zero->count;
            } else {
                dst->zero = src->zero;
            }
        }
    }
}

static void convert_bucket(merge_ctx *mc, int b)
{
    const hmap64 *m = &mc->tasks[0].var.sub[b];
    size_t o = mc->bucket_off[b];
    if (m->zero) {
        mc->out_keys[o] = 0;
        mc->out_sum[o] = m->zero->sum;
        mc->out_cnt[o++] = m->zero->count;
    }
    const size_t cap = (size_t)1 << m->degree;
    for (size_t i = 0; i < cap; ++i) {
        if (!m->cells[i].mapped) continue;
        mc->out_keys[o] = m->cells[i].key;
        mc->out_sum[o] = m->cells[i].mapped->sum;
        mc->out_cnt[o++] = m->cells[i].mapped->count;
    }
}

static void *merge_worker(void *arg)
{
    merge_ctx *mc = ((merge_arg *)arg)->mc;
    for (;;) {
        const int b = atomic_fetch_add(&mc->next_bucket, 1);
        if (b >= BUCKETS) break;
        if (mc->phase == 0) merge_bucket(mc, b);
        else convert_bucket(mc, b);
    }
    return NULL;
}

static void run_parallel(merge_ctx *mc, int phase)
{
    mc->phase = phase;
    atomic_store(&mc->next_bucket, 0);
    pthread_t *th = (pthread_t *)calloc((size_t)mc->nthreads, sizeof(pthread_t));
    merge_arg a = {mc};
    for (int i = 0; i < mc->nthreads; ++i) pthread_create(&th[i], NULL, merge_worker, &a);
    for (int i = 0; i < mc->nthreads; ++i) pthread_join(th[i], NULL);
    free(th);
}

size_t orc_bench_filter_agg_ref(const int64_t *f, int64_t threshold, const int64_t *k, const double *x, size_t n,
                                int nthreads, size_t block_rows, double *checksum)
{
    if (nthreads < 1) nthreads = 1;
    src_task *tasks = (src_task *)calloc((size_t)nthreads, sizeof(src_task));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    const size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int i = 0; i < nthreads; ++i) {
        tasks[i].f = f;
        tasks[i].k = k;
        tasks[i].x = x;
        tasks[i].threshold = threshold;
        tasks[i].begin = per * (size_t)i < n ? per * (size_t)i : n;
        tasks[i].end = per * (size_t)(i + 1) < n ? per * (size_t)(i + 1) : n;
        tasks[i].block_rows = block_rows;
        pthread_create(&th[i], NULL, src_worker, &tasks[i]);
    }
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    /* a thread that stayed single-level converts before the bucket-wise merge (the reference
     * converts every variant to two-level when any is two-level, Aggregator.cpp:2940-2960) */
    for (int i = 0; i < nthreads; ++i)
        if (!tasks[i].var.two_level) convert_to_two_level(&tasks[i].var);
    merge_ctx mc;
    memset(&mc, 0, sizeof(mc));
    mc.tasks = tasks;
    mc.nthreads = nthreads;
    run_parallel(&mc, 0);
    size_t groups = 0;
    size_t *off = (size_t *)malloc((BUCKETS + 1) * sizeof(size_t));
    for (int b = 0; b < BUCKETS; ++b) {
        off[b] = groups;
        groups += tasks[0].var.sub[b].size + (tasks[0].var.sub[b].zero ? 1 : 0);
    }
    off[BUCKETS] = groups;
    mc.bucket_off = off;
    mc.out_keys = (uint64_t *)malloc(groups * 8 + 8);
    mc.out_sum = (double *)malloc(groups * 8 + 8);
    mc.out_cnt = (uint64_t *)malloc(groups * 8 + 8);
    run_parallel(&mc, 1);
    double cs = 0;
    for (size_t g = 0; g < groups; ++g) cs += mc.out_sum[g] + (double)mc.out_cnt[g];
    if (checksum) *checksum = cs;
    free(mc.out_keys);
    free(mc.out_sum);
    free(mc.out_cnt);
    free(off);
    for (int i = 0; i < nthreads; ++i) {
        for (int b = 0; b < BUCKETS; ++b) hm_free(&tasks[i].var.sub[b]);
        arena_free(&tasks[i].var.ar);
    }
    free(tasks);
    free(th);
    return groups;
}
