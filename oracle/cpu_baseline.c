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

/* ------------------------------------------------------------------ C3 join leg
 * Join with the reference's structures (Interpreters/Join.cpp:532-735, JoinPartition.cpp:584-728,
 * 1290-1644; JoinHashMap.h:24-60,175-188): build_concurrency = nthreads segment maps
 * HashMap<UInt64, RowRefList, HashCRC32> (32-byte cells: key + RowRefList{block, row,
 * list_length, next}), segment = hash % build_concurrency; a later row of a key goes into the
 * list at position 2 (insertRowToList).  Probe: each thread takes 65536-row probe blocks
 * (max_block_size), finds each key in its segment's map and appends the matched rows to the
 * output block columns (probe key, probe payload replicated; build payload inserted) —
 * Adder<Inner, All> + replicateRange.  Only the probe is timed by the caller's leg. */
typedef struct {
    uint64_t key;
    uint32_t row;
    uint32_t list_length;
    int64_t next; /* extra RowRefList node, -1 = end */
    uint64_t block; /* the RowRef's Block pointer (kept for the cell size) */
} jcell;

typedef struct {
    jcell *cells;
    int degree;
    size_t size;
    int has_zero;
    jcell zero;
    /* extra list nodes (RowRefList allocated in the pool) */
    uint32_t *node_row;
    int64_t *node_next;
    size_t nodes, node_cap;
} jmap;

static void jm_init(jmap *m)
{
    memset(m, 0, sizeof(*m));
    m->degree = 8;
    m->cells = (jcell *)calloc((size_t)1 << m->degree, sizeof(jcell));
}

static void jm_resize(jmap *m)
{
    const size_t old_cap = (size_t)1 << m->degree;
    jcell *old = m->cells;
    m->degree += m->degree >= 23 ? 1 : 2;
    const size_t mask = ((size_t)1 << m->degree) - 1;
    m->cells = (jcell *)calloc(mask + 1, sizeof(jcell));
    for (size_t i = 0; i < old_cap; ++i) {
        if (!old[i].list_length) continue;
        size_t p = crc_key(old[i].key) & mask;
        while (m->cells[p].list_length) p = (p + 1) & mask;
        m->cells[p] = old[i];
    }
    free(old);
}

static void jm_insert(jmap *m, uint64_t key, uint32_t h, uint32_t row)
{
    jcell *c;
    if (key == 0) {
        c = &m->zero;
        m->has_zero = 1;
    } else {
        const size_t mask = ((size_t)1 << m->degree) - 1;
        size_t p = h & mask;
        while (m->cells[p].list_length && m->cells[p].key != key) p = (p + 1) & mask;
        c = &m->cells[p];
        if (!c->list_length) {
            c->key = key;
            c->row = row;
            c->list_length = 1;
            c->next = -1;
            if (++m->size > ((size_t)1 << (m->degree - 1))) jm_resize(m);
            return;
        }
    }
    if (!c->list_length) {
        c->key = key;
        c->row = row;
        c->list_length = 1;
        c->next = -1;
        return;
    }
    if (m->nodes == m->node_cap) {
        m->node_cap = m->node_cap ? m->node_cap * 2 : 1024;
        m->node_row = (uint32_t *)realloc(m->node_row, m->node_cap * 4);
        m->node_next = (int64_t *)realloc(m->node_next, m->node_cap * 8);
    }
    m->node_row[m->nodes] = row; /* insertRowToList: new node right after the head */
    m->node_next[m->nodes] = c->next;
    c->next = (int64_t)m->nodes++;
    c->list_length++;
}

static const jcell *jm_find(const jmap *m, uint64_t key, uint32_t h)
{
    if (key == 0) return m->has_zero ? &m->zero : NULL;
    const size_t mask = ((size_t)1 << m->degree) - 1;
    size_t p = h & mask;
    while (m->cells[p].list_length) {
        if (m->cells[p].key == key) return &m->cells[p];
        p = (p + 1) & mask;
    }
    return NULL;
}

typedef struct orc_join_ref {
    int segs;
    jmap *maps;
    const int64_t *bpay;
} orc_join_ref;

typedef struct {
    orc_join_ref *j;
    const int64_t *bk;
    size_t nb;
    int seg;
    uint32_t **seg_rows; /* [thread][seg] lists (filled by the dispatch step) */
    size_t **seg_cnt;
    int nthreads;
    size_t begin, end;
} jb_task;

static void *jb_dispatch(void *arg)
{
    jb_task *t = (jb_task *)arg;
    const int S = t->j->segs;
    size_t *cnt = t->seg_cnt[t->seg];
    for (size_t r = t->begin; r < t->end; ++r) cnt[crc_key((uint64_t)t->bk[r]) % (uint32_t)S]++;
    size_t *off = (size_t *)calloc((size_t)S + 1, sizeof(size_t));
    for (int s = 0; s < S; ++s) off[s + 1] = off[s] + cnt[s];
    uint32_t *rows = (uint32_t *)malloc((t->end - t->begin + 1) * 4);
    size_t *pos = (size_t *)malloc((size_t)S * sizeof(size_t));
    memcpy(pos, off, (size_t)S * sizeof(size_t));
    for (size_t r = t->begin; r < t->end; ++r) rows[pos[crc_key((uint64_t)t->bk[r]) % (uint32_t)S]++] = (uint32_t)r;
    t->seg_rows[t->seg] = rows;
    memcpy(cnt, off, (size_t)(S + 1) * sizeof(size_t)); /* becomes the offsets */
    free(off);
    free(pos);
    return NULL;
}

static void *jb_build(void *arg)
{
    jb_task *t = (jb_task *)arg;
    jmap *m = &t->j->maps[t->seg];
    for (int th = 0; th < t->nthreads; ++th) {
        const size_t *off = t->seg_cnt[th];
        const uint32_t *rows = t->seg_rows[th];
        for (size_t i = off[t->seg]; i < off[t->seg + 1]; ++i) {
            const uint32_t r = rows[i];
            const uint64_t key = (uint64_t)t->bk[r];
            jm_insert(m, key, crc_key(key), r);
        }
    }
    return NULL;
}

orc_join_ref *orc_join_ref_build(const int64_t *bk, const int64_t *bpay, size_t nb, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    orc_join_ref *j = (orc_join_ref *)calloc(1, sizeof(orc_join_ref));
    j->segs = nthreads;
    j->bpay = bpay;
    j->maps = (jmap *)calloc((size_t)nthreads, sizeof(jmap));
    for (int s = 0; s < nthreads; ++s) jm_init(&j->maps[s]);
    jb_task *tasks = (jb_task *)calloc((size_t)nthreads, sizeof(jb_task));
    uint32_t **seg_rows = (uint32_t **)calloc((size_t)nthreads, sizeof(uint32_t *));
    size_t **seg_cnt = (size_t **)calloc((size_t)nthreads, sizeof(size_t *));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    const size_t per = (nb + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int i = 0; i < nthreads; ++i) {
        seg_cnt[i] = (size_t *)calloc((size_t)nthreads + 1, sizeof(size_t));
        tasks[i] = (jb_task){j, bk, nb, i, seg_rows, seg_cnt, nthreads, per * (size_t)i < nb ? per * (size_t)i : nb,
                             per * (size_t)(i + 1) < nb ? per * (size_t)(i + 1) : nb};
        pthread_create(&th[i], NULL, jb_dispatch, &tasks[i]);
    }
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, jb_build, &tasks[i]);
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    for (int i = 0; i < nthreads; ++i) {
        free(seg_rows[i]);
        free(seg_cnt[i]);
    }
    free(seg_rows);
    free(seg_cnt);
    free(tasks);
    free(th);
    return j;
}

void orc_join_ref_destroy(orc_join_ref *j)
{
    for (int s = 0; s < j->segs; ++s) {
        free(j->maps[s].cells);
        free(j->maps[s].node_row);
        free(j->maps[s].node_next);
    }
    free(j->maps);
    free(j);
}

typedef struct {
    const orc_join_ref *j;
    const int64_t *pk, *ppay;
    size_t begin, end;
    size_t matches;
    uint64_t checksum;
} jp_ref_task;

static void *jp_ref_worker(void *arg)
{
    jp_ref_task *t = (jp_ref_task *)arg;
    const orc_join_ref *j = t->j;
    const size_t B = 65536;
    size_t cap = B * 2;
    int64_t *ok = (int64_t *)malloc(cap * 8), *op = (int64_t *)malloc(cap * 8), *ob = (int64_t *)malloc(cap * 8);
    for (size_t s = t->begin; s < t->end; s += B) {
        const size_t m = t->end - s < B ? t->end - s : B;
        size_t k = 0;
        for (size_t i = 0; i < m; ++i) {
            const uint64_t key = (uint64_t)t->pk[s + i];
            const uint32_t h = crc_key(key);
            const jcell *c = jm_find(&j->maps[h % (uint32_t)j->segs], key, h);
            if (!c) continue;
            if (k + c->list_length > cap) {
                cap = (k + c->list_length) * 2;
                ok = (int64_t *)realloc(ok, cap * 8);
                op = (int64_t *)realloc(op, cap * 8);
                ob = (int64_t *)realloc(ob, cap * 8);
            }
            const jmap *mm = &j->maps[h % (uint32_t)j->segs];
            ok[k] = (int64_t)key;
            op[k] = t->ppay[s + i];
            ob[k++] = j->bpay[c->row];
            for (int64_t nd = c->next; nd >= 0; nd = mm->node_next[nd]) {
                ok[k] = (int64_t)key;
                op[k] = t->ppay[s + i];
                ob[k++] = j->bpay[mm->node_row[nd]];
            }
        }
        for (size_t q = 0; q < k; q += 97) t->checksum += (uint64_t)ob[q] ^ (uint64_t)op[q]; /* consume the block */
        t->matches += k;
    }
    free(ok);
    free(op);
    free(ob);
    return NULL;
}

size_t orc_join_ref_probe(const orc_join_ref *j, const int64_t *pk, const int64_t *ppay, size_t np, int nthreads,
                          uint64_t *checksum)
{
    if (nthreads < 1) nthreads = 1;
    jp_ref_task *tasks = (jp_ref_task *)calloc((size_t)nthreads, sizeof(jp_ref_task));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    const size_t per = (np + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int i = 0; i < nthreads; ++i) {
        tasks[i].j = j;
        tasks[i].pk = pk;
        tasks[i].ppay = ppay;
        tasks[i].begin = per * (size_t)i < np ? per * (size_t)i : np;
        tasks[i].end = per * (size_t)(i + 1) < np ? per * (size_t)(i + 1) : np;
        pthread_create(&th[i], NULL, jp_ref_worker, &tasks[i]);
    }
    size_t total = 0;
    uint64_t cs = 0;
    for (int i = 0; i < nthreads; ++i) {
        pthread_join(th[i], NULL);
        total += tasks[i].matches;
        cs += tasks[i].checksum;
    }
    if (checksum) *checksum = cs;
    free(tasks);
    free(th);
    return total;
}
