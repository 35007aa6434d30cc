/*
 * cpu_baseline_str.c — the reference's CPU algorithm for the C5 partial aggregation (GROUP BY a
 * String key: sum(Decimal(15,2)) -> Decimal(37,2), count()), restated with the reference's data
 * structures so bench.py's C5 cpu_baseline leg times what TiFlash would do on the same cores.
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY (see oracle.h): never linked into the product path.
 *
 * Per thread (one ParallelAggregatingBlockInputStream source), per Block of block_rows:
 *   Aggregator::executeOnBlock with method key_string (Aggregator.cpp:394-537 ->
 *   HashMethodString, Common/ColumnsHashing.h:179-241): the key is the row's bytes without the
 *   trailing '\0' (ColumnString offsets); StringHashMap (Common/HashTable/StringHashTable.h:211-310)
 *   dispatches keys of 9..16 bytes to its StringKey16 sub-map: 24-byte cells (two key words and
 *   the state pointer), hash = CRC32-C over both words (StringHashTableHash), linear probing,
 *   grower +2 degrees below 2^23, resize above half full; states (Decimal128 sum + UInt64 count,
 *   32 B) bump-allocated in an Arena on insert; conversion to the two-level table (256 buckets,
 *   bucket = (hash >> 24) & 255) past 100000 keys (Settings.h:89).
 * After the barrier: MergingBuckets (Aggregator.cpp:2940-3097), threads take buckets from a shared
 * counter; then convertToBlockImplFinal writes the key column (chars + offsets), sums and counts.
 *
 * Keys of the C5 workload are "k%08d" (9 bytes); keys longer than 16 bytes (other sub-maps) are
 * outside this baseline and abort the run (returns SIZE_MAX).
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

typedef struct {
    __int128 sum;
    uint64_t count;
    uint64_t pad;
} sstate;

typedef struct {
    uint64_t a, b;
    sstate *mapped;
} scell;

typedef struct {
    scell *cells;
    int degree;
    size_t size;
} smap;

typedef struct schunk {
    struct schunk *prev;
    size_t used, cap, pad; /* 32-byte header: states (with __int128) stay 16-byte aligned */
    char data[];
} schunk;

static inline uint32_t key16_hash(uint64_t a, uint64_t b)
{
#if defined(__SSE4_2__)
    return (uint32_t)_mm_crc32_u64(_mm_crc32_u64(0xFFFFFFFFull, a), b);
#else
    return orc_crc32c_u64(orc_crc32c_u64(0xFFFFFFFFu, a), b);
#endif
}

static sstate *salloc(schunk **head)
{
    if (!*head || (*head)->used + sizeof(sstate) > (*head)->cap) {
        size_t cap = *head ? (*head)->cap * 2 : 4096;
        if (cap > (64u << 20)) cap = 64u << 20;
        schunk *c = (schunk *)malloc(sizeof(schunk) + cap);
        c->prev = *head;
        c->used = 0;
        c->cap = cap;
        *head = c;
    }
    sstate *s = (sstate *)((*head)->data + (*head)->used);
    (*head)->used += sizeof(sstate);
    s->sum = 0;
    s->count = 0;
    return s;
}

static void sm_init(smap *m, int degree)
{
    m->degree = degree;
    m->cells = (scell *)calloc((size_t)1 << degree, sizeof(scell));
    m->size = 0;
}

static void sm_insert_cell(smap *m, scell c);

static void sm_resize(smap *m)
{
    const size_t old_cap = (size_t)1 << m->degree;
    scell *old = m->cells;
    m->degree += m->degree >= 23 ? 1 : 2;
    m->cells = (scell *)calloc((size_t)1 << m->degree, sizeof(scell));
    m->size = 0;
    for (size_t i = 0; i < old_cap; ++i)
        if (old[i].mapped) sm_insert_cell(m, old[i]);
    free(old);
}

static void sm_insert_cell(smap *m, scell c)
{
    const size_t mask = ((size_t)1 << m->degree) - 1;
    size_t p = key16_hash(c.a, c.b) & mask;
    while (m->cells[p].mapped) p = (p + 1) & mask;
    m->cells[p] = c;
    if (++m->size > ((size_t)1 << (m->degree - 1))) sm_resize(m);
}

static inline sstate *sm_emplace(smap *m, uint64_t a, uint64_t b, uint32_t h, schunk **ar)
{
    const size_t mask = ((size_t)1 << m->degree) - 1;
    size_t p = h & mask;
    while (m->cells[p].mapped && (m->cells[p].a != a || m->cells[p].b != b)) p = (p + 1) & mask;
    if (m->cells[p].mapped) return m->cells[p].mapped;
    sstate *s = salloc(ar);
    m->cells[p].a = a;
    m->cells[p].b = b;
    m->cells[p].mapped = s;
    if (++m->size > ((size_t)1 << (m->degree - 1))) sm_resize(m);
    return s;
}

#define SB 256
typedef struct {
    const uint8_t *chars;
    const uint64_t *offsets;
    const int64_t *v;
    size_t begin, end, block_rows;
    int two_level, bad;
    smap single, sub[SB];
    schunk *ar;
} stask;

static void to_two_level(stask *t)
{
    for (int b = 0; b < SB; ++b) sm_init(&t->sub[b], 8);
    const size_t cap = (size_t)1 << t->single.degree;
    for (size_t i = 0; i < cap; ++i) {
        const scell c = t->single.cells[i];
        if (c.mapped) sm_insert_cell(&t->sub[(key16_hash(c.a, c.b) >> 24) & 255], c);
    }
    free(t->single.cells);
    t->two_level = 1;
}

static size_t task_bytes(const stask *t)
{
    if (!t->two_level) return ((size_t)1 << t->single.degree) * sizeof(scell);
    size_t s = 0;
    for (int b = 0; b < SB; ++b) s += ((size_t)1 << t->sub[b].degree) * sizeof(scell);
    return s;
}

static inline void key_words(const stask *t, size_t r, uint64_t *a, uint64_t *b, size_t *len)
{
    const uint64_t s = r ? t->offsets[r - 1] : 0;
    *len = (size_t)(t->offsets[r] - s - 1);
    uint64_t w[2] = {0, 0};
    memcpy(w, t->chars + s, *len <= 16 ? *len : 16);
    *a = w[0];
    *b = w[1];
}

static void *str_worker(void *arg)
{
    stask *t = (stask *)arg;
    t->two_level = 0;
    t->ar = NULL;
    sm_init(&t->single, 8);
    for (size_t s = t->begin; s < t->end; s += t->block_rows) {
        const size_t e = s + t->block_rows < t->end ? s + t->block_rows : t->end;
        const int prefetch = task_bytes(t) >= (2u << 20);
        for (size_t r = s; r < e; ++r) {
            uint64_t a, b;
            size_t len;
            if (prefetch && r + 16 < e) {
                key_words(t, r + 16, &a, &b, &len);
                const uint32_t hp = key16_hash(a, b);
                const smap *m = t->two_level ? &t->sub[(hp >> 24) & 255] : &t->single;
                __builtin_prefetch(&m->cells[hp & (((size_t)1 << m->degree) - 1)]);
            }
            key_words(t, r, &a, &b, &len);
            if (len > 16) {
                t->bad = 1;
                return NULL;
            }
            const uint32_t h = key16_hash(a, b);
            sstate *st = t->two_level ? sm_emplace(&t->sub[(h >> 24) & 255], a, b, h, &t->ar)
                                      : sm_emplace(&t->single, a, b, h, &t->ar);
            st->sum += (__int128)t->v[r]; /* Decimal64 -> Decimal128 accumulator */
            st->count += 1;
        }
        if (!t->two_level && t->single.size > 100000) to_two_level(t);
    }
    return NULL;
}

typedef struct {
    stask *tasks;
    int nthreads;
    atomic_int next;
    int phase;
    size_t *bucket_off;
    uint8_t *out_chars;
    uint64_t *out_offsets;
    __int128 *out_sum;
    uint64_t *out_cnt;
} smerge;

static void *smerge_worker(void *arg)
{
    smerge *mc = (smerge *)arg;
    for (;;) {
        const int b = atomic_fetch_add(&mc->next, 1);
        if (b >= SB) break;
        smap *dst = &mc->tasks[0].sub[b];
        if (mc->phase == 0) {
            for (int t = 1; t < mc->nthreads; ++t) {
                const smap *src = &mc->tasks[t].sub[b];
                const size_t cap = (size_t)1 << src->degree;
                for (size_t i = 0; i < cap; ++i) {
                    const scell c = src->cells[i];
                    if (!c.mapped) continue;
                    const size_t mask = ((size_t)1 << dst->degree) - 1;
                    size_t p = key16_hash(c.a, c.b) & mask;
                    while (dst->cells[p].mapped && (dst->cells[p].a != c.a || dst->cells[p].b != c.b))
                        p = (p + 1) & mask;
                    if (dst->cells[p].mapped) {
                        dst->cells[p].mapped->sum += c.mapped->sum;
                        dst->cells[p].mapped->count += c.mapped->count;
                    } else {
                        sm_insert_cell(dst, c);
                    }
                }
            }
        } else { /* convertToBlockImplFinal: key column (chars + '\0' + offsets), sum, count */
            size_t g = mc->bucket_off[b];
            size_t co = g * 17; /* per-bucket regions (keys <= 16 bytes + NUL) */
            const size_t cap = (size_t)1 << dst->degree;
            for (size_t i = 0; i < cap; ++i) {
                const scell c = dst->cells[i];
                if (!c.mapped) continue;
                uint64_t w[2] = {c.a, c.b};
                const size_t len = strnlen((const char *)w, 16);
                memcpy(mc->out_chars + co, w, len);
                mc->out_chars[co + len] = 0;
                co += len + 1;
                mc->out_offsets[g] = co;
                mc->out_sum[g] = c.mapped->sum;
                mc->out_cnt[g] = c.mapped->count;
                ++g;
            }
        }
    }
    return NULL;
}

/* C5 partial aggregation over n String rows with nthreads sources; returns the number of groups
 * (SIZE_MAX if a key does not fit the StringKey16 sub-map), *checksum = sum of counts. */
size_t orc_bench_string_agg(const uint8_t *chars, const uint64_t *offsets, const int64_t *v, size_t n, int nthreads,
                            size_t block_rows, uint64_t *checksum)
{
    stask *tasks = (stask *)calloc((size_t)nthreads, sizeof(stask));
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int i = 0; i < nthreads; ++i) {
        tasks[i].chars = chars;
        tasks[i].offsets = offsets;
        tasks[i].v = v;
        tasks[i].begin = n * (size_t)i / (size_t)nthreads;
        tasks[i].end = n * (size_t)(i + 1) / (size_t)nthreads;
        tasks[i].block_rows = block_rows;
        pthread_create(&th[i], NULL, str_worker, &tasks[i]);
    }
    int bad = 0;
    for (int i = 0; i < nthreads; ++i) {
        pthread_join(th[i], NULL);
        bad |= tasks[i].bad;
        if (!tasks[i].two_level) to_two_level(&tasks[i]); /* merge is bucket-wise */
    }
    size_t groups = SIZE_MAX;
    if (!bad) {
        smerge mc;
        memset(&mc, 0, sizeof(mc));
        mc.tasks = tasks;
        mc.nthreads = nthreads;
        for (int phase = 0; phase < 2; ++phase) {
            if (phase == 1) {
                mc.bucket_off = (size_t *)malloc(sizeof(size_t) * (SB + 1));
                mc.bucket_off[0] = 0;
                for (int b = 0; b < SB; ++b) mc.bucket_off[b + 1] = mc.bucket_off[b] + tasks[0].sub[b].size;
                groups = mc.bucket_off[SB];
                mc.out_chars = (uint8_t *)malloc(groups * 17 + 1);
                mc.out_offsets = (uint64_t *)malloc(groups * 8 + 8);
                mc.out_sum = (__int128 *)malloc(groups * 16 + 16);
                mc.out_cnt = (uint64_t *)malloc(groups * 8 + 8);
            }
            mc.phase = phase;
            atomic_store(&mc.next, 0);
            for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, smerge_worker, &mc);
            for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
        }
        uint64_t cs = 0;
        for (size_t g = 0; g < groups; ++g) cs += mc.out_cnt[g];
        if (checksum) *checksum = cs;
        free(mc.bucket_off);
        free(mc.out_chars);
        free(mc.out_offsets);
        free(mc.out_sum);
        free(mc.out_cnt);
    }
    for (int i = 0; i < nthreads; ++i) {
        for (int b = 0; b < SB; ++b) free(tasks[i].sub[b].cells);
        while (tasks[i].ar) {
            schunk *p = tasks[i].ar->prev;
            free(tasks[i].ar);
            tasks[i].ar = p;
        }
    }
    free(tasks);
    free(th);
    return groups;
}
