// serial.hip — the `serialized` GROUP BY method (see serial.h).
//
// Reference: AggregationMethodSerialized / HashMethodSerialized (Common/ColumnsHashing.h:578-629)
// serialise each row's key tuple (IColumn::serializeValueIntoArena: ColumnNullable writes a null
// flag byte and then the nested value, ColumnString its length and the collator's sort key,
// ColumnVector the raw value bytes) and key a HashMap on the bytes.  Two rows are the same group
// iff their serialised bytes are equal; that equality is what this dictionary decides on the device.
//
// Layout in HBM (all owned by the dictionary, grown by doubling):
//   fp[cap]  u64 fingerprint per slot (0 = empty), gid[cap] u32 group id, owner[cap] u32 the
//            smallest row of the current block that claimed a new slot;
//   arena    the serialised key tuples of the groups, goff[g] / glen[g] locate group g's bytes;
//   slot / list rows: per-row slot index and the retry lists.
// Per block: insert (fingerprint -> slot, CAS-claimed) -> assign (the owner row of each new slot
// appends its tuple to the arena, takes the next group id) -> verify (each row compares its tuple
// with its slot's bytes; a mismatch is a fingerprint collision and the row retries with the next
// seed).  The number of retries is read back once per round; collisions of 64-bit fingerprints
// are rare, so a block almost always takes one round.
#include "serial.h"

namespace tfg {

constexpr int SKMAX = 8;
constexpr uint32_t SER_NONE = 0xFFFFFFFFu;

struct SerCols {
    int nkeys;
    int width[SKMAX]; // bytes; 0 = String
    int collator[SKMAX];
    const uint8_t *col[SKMAX];
    const uint64_t *offsets[SKMAX];
    const uint8_t *nullmap[SKMAX];
};

struct SerialDict {
    Ctx *ctx = nullptr;
    int nkeys = 0;
    int types[SKMAX] = {};
    int width[SKMAX] = {};
    int collator[SKMAX] = {};
    // slot table
    uint64_t *fp = nullptr;
    uint32_t *gid = nullptr;
    uint32_t *owner = nullptr;
    uint64_t cap = 0;
    // key arena
    uint8_t *arena = nullptr;
    uint64_t arena_cap = 0, arena_used = 0;
    uint64_t *goff = nullptr;
    uint32_t *glen = nullptr;
    uint64_t gcap = 0, G = 0;
    // per-row buffers
    uint32_t *rows = nullptr; // slot[n] | listA[n] | listB[n]
    uint64_t rows_cap = 0;
    uint64_t *dcnt = nullptr; // [0] groups, [1] arena bytes, [2] retries, [3] table-full flag
};

__device__ __forceinline__ uint64_t ser_mix(uint64_t h, uint64_t w) {
    h = (h ^ w) * 0xbf58476d1ce4e5b9ull;
    return h ^ (h >> 31);
}

// the collator's sort key of String row r (BinCollatorSortKey<true> right-trims spaces)
__device__ __forceinline__ const uint8_t *ser_sort_key(const SerCols &k, int j, int64_t r, uint32_t &len) {
    const uint64_t s = r ? k.offsets[j][r - 1] : 0, e = k.offsets[j][r];
    const uint8_t *c = k.col[j] + s;
    int64_t l = (int64_t)(e - s) - 1; // rows end with '\0'
    if (k.collator[j] == TFG_COLLATOR_BIN_PADDING)
        while (l > 0 && c[l - 1] == ' ') --l;
    len = (uint32_t)(l < 0 ? 0 : l);
    return c;
}

__device__ __forceinline__ bool ser_null(const SerCols &k, int j, int64_t r) {
    return k.nullmap[j] && k.nullmap[j][r];
}

__device__ uint64_t ser_hash(const SerCols &k, int64_t r, uint64_t seed) {
    uint64_t h = 0x2545F4914F6CDD1Dull ^ (seed * 0x9E3779B97F4A7C15ull);
    for (int j = 0; j < k.nkeys; ++j) {
        if (ser_null(k, j, r)) {
            h = ser_mix(h, 0xA5A5A5A5A5A50000ull | (uint64_t)j);
            continue;
        }
        const int wd = k.width[j];
        if (wd == 0) {
            uint32_t len;
            const uint8_t *c = ser_sort_key(k, j, r, len);
            uint64_t w = 0;
            for (uint32_t i = 0; i < len; ++i) {
                w |= (uint64_t)c[i] << ((i & 7) * 8);
                if ((i & 7) == 7) {
                    h = ser_mix(h, w);
                    w = 0;
                }
            }
            h = ser_mix(h, w ^ ((uint64_t)len << 40));
        } else {
            const uint8_t *p = k.col[j] + (int64_t)wd * r;
            uint64_t w = 0;
            for (int i = 0; i < wd; ++i) {
                w |= (uint64_t)p[i] << ((i & 7) * 8);
                if ((i & 7) == 7 || i == wd - 1) {
                    h = ser_mix(h, w);
                    w = 0;
                }
            }
        }
    }
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9aa6b8f5d35ull;
    h ^= h >> 33;
    return h ? h : 1; // 0 marks an empty slot
}

// serialised size: per key a null-flag byte, then width bytes (fixed) or u32 length + sort key
__device__ uint32_t ser_len(const SerCols &k, int64_t r) {
    uint32_t n = 0;
    for (int j = 0; j < k.nkeys; ++j) {
        n += 1;
        if (ser_null(k, j, r)) continue;
        if (k.width[j]) {
            n += k.width[j];
        } else {
            uint32_t len;
            ser_sort_key(k, j, r, len);
            n += 4 + len;
        }
    }
    return n;
}

__device__ void ser_write(const SerCols &k, int64_t r, uint8_t *d) {
    for (int j = 0; j < k.nkeys; ++j) {
        if (ser_null(k, j, r)) {
            *d++ = 1;
            continue;
        }
        *d++ = 0;
        if (k.width[j]) {
            const uint8_t *p = k.col[j] + (int64_t)k.width[j] * r;
            for (int i = 0; i < k.width[j]; ++i) *d++ = p[i];
        } else {
            uint32_t len;
            const uint8_t *c = ser_sort_key(k, j, r, len);
            for (int i = 0; i < 4; ++i) *d++ = (uint8_t)(len >> (8 * i));
            for (uint32_t i = 0; i < len; ++i) *d++ = c[i];
        }
    }
}

__device__ bool ser_equal(const SerCols &k, int64_t r, const uint8_t *b, uint32_t blen) {
    const uint8_t *e = b + blen;
    for (int j = 0; j < k.nkeys; ++j) {
        if (b >= e) return false;
        const uint8_t isnull = *b++;
        if (ser_null(k, j, r)) {
            if (!isnull) return false;
            continue;
        }
        if (isnull) return false;
        if (k.width[j]) {
            if (b + k.width[j] > e) return false;
            const uint8_t *p = k.col[j] + (int64_t)k.width[j] * r;
            for (int i = 0; i < k.width[j]; ++i)
                if (b[i] != p[i]) return false;
            b += k.width[j];
        } else {
            if (b + 4 > e) return false;
            const uint32_t bl = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
            b += 4;
            uint32_t len;
            const uint8_t *c = ser_sort_key(k, j, r, len);
            if (bl != len || b + len > e) return false;
            for (uint32_t i = 0; i < len; ++i)
                if (b[i] != c[i]) return false;
            b += len;
        }
    }
    return b == e;
}

__global__ void ser_insert_kernel(SerCols k, int64_t m, const uint32_t *list, const uint8_t *mask, uint64_t seed,
                                  uint64_t *fp, const uint32_t *gid, uint32_t *owner, uint64_t cmask, uint32_t *slot,
                                  uint64_t *cnt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = list ? list[i] : i;
        if (mask && !mask[r]) {
            slot[r] = SER_NONE;
            continue;
        }
        const uint64_t h = ser_hash(k, r, seed);
        uint64_t s = h & cmask;
        // bounded probe: the host sizes the table for every claim of this round at fill <= 1/2,
        // so a full sweep never happens; if it did, the row lands on a claimed slot (the verify
        // then fails it) and cnt[3] makes the host report the table as full
        for (uint64_t step = 0;; ++step) {
            uint64_t cur = fp[s];
            if (cur == 0) {
                cur = atomicCAS((unsigned long long *)&fp[s], 0ull, (unsigned long long)h);
                if (cur == 0) cur = h;
            }
            if (cur == h) break;
            if (step == cmask) {
                atomicOr((unsigned long long *)&cnt[3], 1ull);
                break;
            }
            s = (s + 1) & cmask;
        }
        slot[r] = (uint32_t)s;
        if (gid[s] == SER_NONE) atomicMin(&owner[s], (uint32_t)r);
    }
}

__global__ void ser_assign_kernel(SerCols k, int64_t m, const uint32_t *list, const uint8_t *mask,
                                  const uint32_t *slot, uint32_t *gid, uint32_t *owner, uint64_t *cnt, uint8_t *arena,
                                  uint64_t *goff, uint32_t *glen) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = list ? list[i] : i;
        if (mask && !mask[r]) continue;
        const uint32_t s = slot[r];
        if (owner[s] != (uint32_t)r) continue;
        const uint32_t len = ser_len(k, r);
        const uint64_t g = atomicAdd((unsigned long long *)&cnt[0], 1ull);
        const uint64_t off = atomicAdd((unsigned long long *)&cnt[1], (unsigned long long)len);
        ser_write(k, r, arena + off);
        goff[g] = off;
        glen[g] = len;
        gid[s] = (uint32_t)g;
        owner[s] = SER_NONE;
    }
}

__global__ void ser_verify_kernel(SerCols k, int64_t m, const uint32_t *list, const uint8_t *mask,
                                  const uint32_t *slot, const uint32_t *gid, const uint8_t *arena, const uint64_t *goff,
                                  const uint32_t *glen, uint32_t *out, uint64_t *cnt, uint32_t *retry) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = list ? list[i] : i;
        if (mask && !mask[r]) {
            out[r] = 0;
            continue;
        }
        const uint32_t g = gid[slot[r]];
        if (ser_equal(k, r, arena + goff[g], glen[g])) {
            out[r] = g;
        } else { // a fingerprint collision: the row retries with the next seed
            const uint64_t p = atomicAdd((unsigned long long *)&cnt[2], 1ull);
            retry[p] = (uint32_t)r;
        }
    }
}

__global__ void ser_rehash_kernel(const uint64_t *ofp, const uint32_t *ogid, uint64_t ocap, uint64_t *fp,
                                  uint32_t *gid, uint64_t cmask) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < (int64_t)ocap;
         s += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = ofp[s];
        if (!h) continue;
        uint64_t p = h & cmask;
        while (atomicCAS((unsigned long long *)&fp[p], 0ull, (unsigned long long)h) != 0ull) p = (p + 1) & cmask;
        gid[p] = ogid[s];
    }
}

// ---------------------------------------------------------------- unpack (convertToBlock)
struct SerOut {
    int nkeys;
    int width[SKMAX];
    uint8_t *col[SKMAX];
    uint64_t *offsets[SKMAX];
    uint8_t *nullmap[SKMAX];
    const uint64_t *start[SKMAX];
};

// locate key j of a serialised tuple: returns the value bytes (nullptr = NULL), len for Strings
__device__ const uint8_t *ser_field(const uint8_t *b, const int *width, int j, uint32_t &len) {
    for (int t = 0;; ++t) {
        const uint8_t isnull = *b++;
        const uint8_t *v = isnull ? nullptr : b;
        len = 0;
        if (!isnull) {
            if (width[t]) {
                len = (uint32_t)width[t];
                b += width[t];
            } else {
                len = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
                v = b + 4;
                b += 4 + len;
            }
        }
        if (t == j) return v;
    }
}

__global__ void ser_str_len_kernel(SerOut o, int j, const uint32_t *gid, uint64_t G, const uint8_t *arena,
                                   const uint64_t *goff, uint64_t *len1) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)G; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t len;
        const uint8_t *v = ser_field(arena + goff[gid[i]], o.width, j, len);
        len1[i] = (v ? len : 0) + 1;
    }
}

__global__ void ser_unpack_kernel(SerOut o, const uint32_t *gid, uint64_t G, const uint8_t *arena, const uint64_t *goff) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)G; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t *b = arena + goff[gid[i]];
        for (int j = 0; j < o.nkeys; ++j) {
            uint32_t len;
            const uint8_t *v = ser_field(b, o.width, j, len);
            if (o.nullmap[j]) o.nullmap[j][i] = v ? 0 : 1;
            if (o.width[j]) {
                if (!o.col[j]) continue;
                uint8_t *d = o.col[j] + (int64_t)o.width[j] * i;
                for (int t = 0; t < o.width[j]; ++t) d[t] = v ? v[t] : 0;
            } else {
                const uint64_t s = o.start[j][i];
                if (o.col[j]) {
                    uint8_t *d = o.col[j] + s;
                    for (uint32_t t = 0; v && t < len; ++t) d[t] = v[t];
                    d[v ? len : 0] = 0;
                }
                if (o.offsets[j]) o.offsets[j][i] = o.start[j][i + 1];
            }
        }
    }
}

// ---------------------------------------------------------------- host
static int ser_grow_u8(Ctx *ctx, uint8_t *&p, uint64_t &cap, uint64_t used, uint64_t need) {
    if (cap >= need && p) return TFG_OK;
    const uint64_t nc = std::max<uint64_t>(need + need / 2, 1 << 16);
    uint8_t *q = nullptr;
    TFG_HIP(hipMalloc(&q, nc));
    if (p) {
        if (used) TFG_HIP(hipMemcpyAsync(q, p, used, hipMemcpyDeviceToDevice, ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
        TFG_HIP(hipFree(p));
    }
    p = q;
    cap = nc;
    return TFG_OK;
}

static int ser_grow_groups(SerialDict *d, uint64_t need) {
    if (d->gcap >= need && d->goff) return TFG_OK;
    const uint64_t nc = std::max<uint64_t>(need + need / 2, 4096);
    uint64_t *o = nullptr;
    uint32_t *l = nullptr;
    TFG_HIP(hipMalloc(&o, nc * 8));
    TFG_HIP(hipMalloc(&l, nc * 4));
    if (d->goff) {
        if (d->G) {
            TFG_HIP(hipMemcpyAsync(o, d->goff, d->G * 8, hipMemcpyDeviceToDevice, d->ctx->stream));
            TFG_HIP(hipMemcpyAsync(l, d->glen, d->G * 4, hipMemcpyDeviceToDevice, d->ctx->stream));
        }
        TFG_HIP(hipStreamSynchronize(d->ctx->stream));
        TFG_HIP(hipFree(d->goff));
        TFG_HIP(hipFree(d->glen));
    }
    d->goff = o;
    d->glen = l;
    d->gcap = nc;
    return TFG_OK;
}

// slot table with room for `entries` at fill <= 1/2 (rehashes the committed slots)
static int ser_grow_table(SerialDict *d, uint64_t entries) {
    uint64_t nc = 4096;
    while (nc < 2 * entries) nc *= 2;
    if (d->cap >= nc && d->fp) return TFG_OK;
    Ctx *ctx = d->ctx;
    uint64_t *fp = nullptr;
    uint32_t *gid = nullptr, *owner = nullptr;
    TFG_HIP(hipMalloc(&fp, nc * 8));
    TFG_HIP(hipMalloc(&gid, nc * 4));
    TFG_HIP(hipMalloc(&owner, nc * 4));
    TFG_HIP(hipMemsetAsync(fp, 0, nc * 8, ctx->stream));
    TFG_HIP(hipMemsetAsync(gid, 0xFF, nc * 4, ctx->stream));
    TFG_HIP(hipMemsetAsync(owner, 0xFF, nc * 4, ctx->stream));
    if (d->fp) {
        hipLaunchKernelGGL(ser_rehash_kernel, dim3(stream_grid((int64_t)d->cap, 256)), dim3(256), 0, ctx->stream, d->fp,
                           d->gid, d->cap, fp, gid, nc - 1);
        TFG_LAUNCH_CHECK();
        TFG_HIP(hipStreamSynchronize(ctx->stream));
        TFG_HIP(hipFree(d->fp));
        TFG_HIP(hipFree(d->gid));
        TFG_HIP(hipFree(d->owner));
    }
    d->fp = fp;
    d->gid = gid;
    d->owner = owner;
    d->cap = nc;
    return TFG_OK;
}

int serial_dict_create(Ctx *ctx, int nkeys, const int *key_types, const int *key_collators, SerialDict **out) {
    TFG_CHECK(nkeys >= 1 && nkeys <= SKMAX, TFG_ERR_NOT_IMPLEMENTED, "%d GROUP BY keys: 1-%d supported", nkeys, SKMAX);
    SerialDict *d = new SerialDict();
    d->ctx = ctx;
    d->nkeys = nkeys;
    for (int j = 0; j < nkeys; ++j) {
        const int t = key_types[j];
        const int c = key_collators ? key_collators[j] : TFG_COLLATOR_NONE;
        d->types[j] = t;
        d->collator[j] = c;
        if (t == TFG_STRING) {
            d->width[j] = 0;
            if (c < TFG_COLLATOR_NONE || c > TFG_COLLATOR_BIN_PADDING) {
                delete d;
                return fail(TFG_ERR_NOT_IMPLEMENTED, "collator %d not supported", c);
            }
        } else {
            const size_t w = type_width(t);
            if (w == 0 || w > 32) {
                delete d;
                return fail(TFG_ERR_ILLEGAL_TYPE, "GROUP BY key %d of type %d cannot be serialised", j, t);
            }
            d->width[j] = (int)w;
        }
    }
    if (hipMalloc(&d->dcnt, 4 * sizeof(uint64_t)) != hipSuccess) {
        delete d;
        return fail(TFG_ERR_OOM, "dictionary counters");
    }
    if (hipMemsetAsync(d->dcnt, 0, 4 * sizeof(uint64_t), ctx->stream) != hipSuccess) {
        serial_dict_destroy(d);
        return fail(TFG_ERR_HIP, "dictionary counters");
    }
    *out = d;
    return TFG_OK;
}

void serial_dict_destroy(SerialDict *d) {
    if (!d) return;
    (void)hipStreamSynchronize(d->ctx->stream);
    for (void *p : {(void *)d->fp, (void *)d->gid, (void *)d->owner, (void *)d->arena, (void *)d->goff,
                    (void *)d->glen, (void *)d->rows, (void *)d->dcnt})
        if (p) (void)hipFree(p);
    delete d;
}

void serial_dict_reset(SerialDict *d) {
    Ctx *ctx = d->ctx;
    if (d->fp) {
        (void)hipMemsetAsync(d->fp, 0, d->cap * 8, ctx->stream);
        (void)hipMemsetAsync(d->gid, 0xFF, d->cap * 4, ctx->stream);
        (void)hipMemsetAsync(d->owner, 0xFF, d->cap * 4, ctx->stream);
    }
    (void)hipMemsetAsync(d->dcnt, 0, 4 * sizeof(uint64_t), ctx->stream);
    d->G = 0;
    d->arena_used = 0;
}

uint64_t serial_dict_groups(const SerialDict *d) { return d->G; }

int serial_dict_assign(SerialDict *d, const void *const *key_cols, const uint64_t *const *key_offsets,
                       const uint8_t *const *key_nullmaps, const uint8_t *mask, int64_t n, uint32_t *out_gid) {
    if (n <= 0) return TFG_OK;
    TFG_CHECK(key_cols && out_gid, TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(n < (int64_t)SER_NONE, TFG_ERR_INVALID_ARG, "block of %lld rows: at most 2^32-2", (long long)n);
    Ctx *ctx = d->ctx;
    SerCols k{};
    k.nkeys = d->nkeys;
    // arena bound for this block: every row a new group
    uint64_t bound = 0;
    for (int j = 0; j < d->nkeys; ++j) {
        TFG_CHECK(key_cols[j], TFG_ERR_INVALID_ARG, "key column %d is null", j);
        k.width[j] = d->width[j];
        k.collator[j] = d->collator[j];
        k.col[j] = (const uint8_t *)key_cols[j];
        k.nullmap[j] = key_nullmaps ? key_nullmaps[j] : nullptr;
        if (d->width[j] == 0) {
            TFG_CHECK(key_offsets && key_offsets[j], TFG_ERR_INVALID_ARG, "String key %d needs its offsets", j);
            k.offsets[j] = key_offsets[j];
            uint64_t chars = 0;
            TFG_HIP(hipMemcpyAsync(&chars, key_offsets[j] + (n - 1), 8, hipMemcpyDeviceToHost, ctx->stream));
            TFG_HIP(hipStreamSynchronize(ctx->stream));
            bound += (uint64_t)n * 5 + chars;
        } else {
            bound += (uint64_t)n * (1 + d->width[j]);
        }
    }
    if (int rc = ser_grow_table(d, d->G + (uint64_t)n)) return rc;
    if (int rc = ser_grow_groups(d, d->G + (uint64_t)n)) return rc;
    if (int rc = ser_grow_u8(ctx, d->arena, d->arena_cap, d->arena_used, d->arena_used + bound + 16)) return rc;
    if (d->rows_cap < (uint64_t)n) {
        if (d->rows) {
            TFG_HIP(hipStreamSynchronize(ctx->stream));
            TFG_HIP(hipFree(d->rows));
            d->rows = nullptr;
        }
        const uint64_t nc = std::max<uint64_t>((uint64_t)n + (uint64_t)n / 4, 4096);
        TFG_HIP(hipMalloc(&d->rows, nc * 3 * sizeof(uint32_t)));
        d->rows_cap = nc;
    }
    uint32_t *slot = d->rows, *lists[2] = {d->rows + d->rows_cap, d->rows + 2 * d->rows_cap};
    const uint32_t *list = nullptr;
    int64_t m = n;
    uint64_t claimed = d->G + (uint64_t)n; // fingerprint slots this consume may claim
    ProfScope _ps(ctx, "agg.serial_dict");
    for (int round = 0;; ++round) {
        TFG_CHECK(round < 16, TFG_ERR_LOGICAL, "serialized keys: fingerprint collisions persist after 16 seeds");
        const uint8_t *mk = round == 0 ? mask : nullptr; // retries hold unmasked rows only
        uint32_t *retry = lists[round & 1];
        // a retry round claims up to m slots for fingerprints at the new seed: keep the table at
        // fill <= 1/2 for them (round 0 was sized above for G + n)
        if (round > 0) {
            claimed += (uint64_t)m;
            if (int rc = ser_grow_table(d, claimed)) return rc;
        }
        const unsigned grid = stream_grid(m, 256);
        TFG_HIP(hipMemsetAsync(d->dcnt + 2, 0, 8, ctx->stream));
        hipLaunchKernelGGL(ser_insert_kernel, dim3(grid), dim3(256), 0, ctx->stream, k, m, list, mk, (uint64_t)round,
                           d->fp, d->gid, d->owner, d->cap - 1, slot, d->dcnt);
        hipLaunchKernelGGL(ser_assign_kernel, dim3(grid), dim3(256), 0, ctx->stream, k, m, list, mk, slot, d->gid,
                           d->owner, d->dcnt, d->arena, d->goff, d->glen);
        hipLaunchKernelGGL(ser_verify_kernel, dim3(grid), dim3(256), 0, ctx->stream, k, m, list, mk, slot, d->gid,
                           d->arena, d->goff, d->glen, out_gid, d->dcnt, retry);
        TFG_LAUNCH_CHECK();
        uint64_t c[4];
        TFG_HIP(hipMemcpyAsync(c, d->dcnt, sizeof(c), hipMemcpyDeviceToHost, ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
        TFG_CHECK(c[3] == 0, TFG_ERR_LOGICAL, "serialized keys: fingerprint table full");
        d->G = c[0];
        d->arena_used = c[1];
        if (c[2] == 0) break;
        list = retry;
        m = (int64_t)c[2];
    }
    return TFG_OK;
}

int serial_dict_unpack(SerialDict *d, const uint32_t *gid, uint64_t G, void *const *out_cols,
                       uint64_t *const *out_offsets, uint8_t *const *out_nullmaps, uint64_t chars_capacity,
                       uint64_t *out_chars_max) {
    Ctx *ctx = d->ctx;
    if (out_chars_max) *out_chars_max = 0;
    if (G == 0) return TFG_OK;
    SerOut o{};
    o.nkeys = d->nkeys;
    int nstr = 0;
    for (int j = 0; j < d->nkeys; ++j) {
        o.width[j] = d->width[j];
        o.col[j] = out_cols ? (uint8_t *)out_cols[j] : nullptr;
        o.offsets[j] = out_offsets ? out_offsets[j] : nullptr;
        o.nullmap[j] = out_nullmaps ? out_nullmaps[j] : nullptr;
        nstr += d->width[j] == 0;
    }
    const unsigned grid = stream_grid((int64_t)G, 256);
    if (nstr) {
        Carver cv;
        const size_t o_len = cv.take<uint64_t>(G), o_tmp = cv.take<uint8_t>(scan_tmp_bytes((int64_t)G));
        size_t o_start[SKMAX] = {};
        for (int j = 0; j < d->nkeys; ++j)
            if (!d->width[j]) o_start[j] = cv.take<uint64_t>(G + 1);
        void *sp;
        if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
        char *sb = (char *)sp;
        uint64_t chars_max = 0;
        for (int j = 0; j < d->nkeys; ++j) {
            if (d->width[j]) continue;
            uint64_t *len1 = (uint64_t *)(sb + o_len), *start = (uint64_t *)(sb + o_start[j]);
            hipLaunchKernelGGL(ser_str_len_kernel, dim3(grid), dim3(256), 0, ctx->stream, o, j, gid, G, d->arena,
                               d->goff, len1);
            TFG_LAUNCH_CHECK();
            if (int rc = exclusive_scan_u64(ctx, len1, start, (int64_t)G, sb + o_tmp)) return rc;
            uint64_t chars = 0;
            if (int rc = read_back_u64(ctx, start + G, &chars, 1)) return rc;
            chars_max = std::max(chars_max, chars);
            o.start[j] = start;
            TFG_CHECK(!o.col[j] || o.offsets[j], TFG_ERR_INVALID_ARG, "String key %d needs its offsets", j);
        }
        if (out_chars_max) *out_chars_max = chars_max;
        if (chars_max > chars_capacity)
            return fail(TFG_ERR_CAPACITY, "String keys need %llu bytes, capacity %llu", (unsigned long long)chars_max,
                        (unsigned long long)chars_capacity);
    }
    {
        ProfScope _ps(ctx, "agg.serial_unpack");
        hipLaunchKernelGGL(ser_unpack_kernel, dim3(grid), dim3(256), 0, ctx->stream, o, gid, G, d->arena, d->goff);
    }
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

} // namespace tfg
