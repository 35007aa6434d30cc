/*
 * codec.c — CPU restatement of the MPP packet codec (§8 f1).
 *
 * TEST INFRASTRUCTURE ONLY (checker + timed CPU baseline).  Never linked by the product.
 * Restates, from the reference's text (paths relative to /root/reference/dbms/src):
 *   CHBlockChunkCodecStream::encode         Flash/Coprocessor/CHBlockChunkCodec.cpp:134-166
 *   EncodeHeader + encodeColumnImpl + V1     Flash/Coprocessor/CHBlockChunkCodecV1.cpp:45-58, 293-312, 370-432
 *   writeVarUInt / writeStringBinary         IO/VarInt.h:224-240
 *   DataTypeNumberBase::serializeBinaryBulk  DataTypes/DataTypeNumberBase.cpp:220-232
 *   DataTypeDecimal::serializeBinaryBulk     DataTypes/DataTypeDecimal.cpp:93-105
 *   DataTypeNullable (null map, then nested) DataTypes/DataTypeNullable.cpp:66-89
 *   DataTypeString legacy (varuint size + bytes per row)  DataTypes/DataTypeString.cpp:93-117
 *   DataTypeString V2 (UInt64 sizes incl. terminator, then chars)  DataTypes/DataTypeString.cpp:339-430
 *   readVarUInt + deserializeBinarySSE2      DataTypes/DataTypeString.cpp:120-176 (decode)
 * Pinned by the format spec only (the reference's codec gtests are round trips of random data,
 * gtest_block_chunk_codec.cpp:125-453); tests/test_codec.py adds hand-derived packets.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/tiflash_amd.h"

typedef struct {
    int width;    /* fixed-width payload bytes, 0 for strings */
    int nullable;
    int string;
    int v2;
} orc_ctype;

static int parse_type(const char *s, orc_ctype *t)
{
    char x[128];
    memset(t, 0, sizeof(*t));
    size_t L = strlen(s);
    if (L >= sizeof(x)) return -1;
    strcpy(x, s);
    if (strncmp(x, "Nullable(", 9) == 0 && x[L - 1] == ')') {
        t->nullable = 1;
        memmove(x, x + 9, L - 9);
        x[L - 10] = 0;
    }
    static const struct { const char *n; int w; } fixed[] = {
        {"Int8", 1}, {"Int16", 2}, {"Int32", 4}, {"Int64", 8}, {"UInt8", 1}, {"UInt16", 2},
        {"UInt32", 4}, {"UInt64", 8}, {"Float32", 4}, {"Float64", 8}, {"MyDate", 8}};
    for (size_t i = 0; i < sizeof(fixed) / sizeof(fixed[0]); ++i)
        if (strcmp(x, fixed[i].n) == 0) {
            t->width = fixed[i].w;
            return 0;
        }
    if (strncmp(x, "MyDateTime(", 11) == 0 || strncmp(x, "MyDuration(", 11) == 0) {
        t->width = 8;
        return 0;
    }
    if (strcmp(x, "String") == 0 || strcmp(x, "StringV2") == 0) {
        t->string = 1;
        t->v2 = strcmp(x, "StringV2") == 0;
        return 0;
    }
    int p, sc;
    if (sscanf(x, "Decimal(%d,%d)", &p, &sc) == 2 || sscanf(x, "Decimal(%d, %d)", &p, &sc) == 2) {
        if (p <= 0 || p > 38) return -1;
        t->width = p <= 9 ? 4 : p <= 18 ? 8 : 16;
        return 0;
    }
    return -1;
}

typedef struct {
    uint8_t *out; /* NULL: size only */
    size_t cap, at;
    int overflow;
} wbuf;

static void put(wbuf *w, const void *p, size_t n)
{
    if (w->out && !w->overflow) {
        if (w->at + n > w->cap) w->overflow = 1;
        else if (n) memcpy(w->out + w->at, p, n);
    }
    w->at += n;
}

static void put_varuint(wbuf *w, uint64_t x) /* writeVarUInt: at most 9 bytes */
{
    for (int i = 0; i < 9; ++i) {
        uint8_t b = x & 0x7F;
        if (x > 0x7F) b |= 0x80;
        put(w, &b, 1);
        x >>= 7;
        if (!x) return;
    }
}

static void put_str(wbuf *w, const char *s)
{
    size_t n = strlen(s);
    put_varuint(w, n);
    put(w, s, n);
}

/* rows [r0, r1) of one column */
static void put_column(wbuf *w, const orc_ctype *t, const void *data, const uint64_t *offs, const uint8_t *nm,
                       int64_t r0, int64_t r1)
{
    if (t->nullable) put(w, nm + r0, (size_t)(r1 - r0));
    if (!t->string) {
        put(w, (const uint8_t *)data + (size_t)r0 * t->width, (size_t)(r1 - r0) * t->width);
        return;
    }
    const uint8_t *chars = (const uint8_t *)data;
    if (t->v2) {
        for (int64_t i = r0; i < r1; ++i) {
            uint64_t sz = offs[i] - (i ? offs[i - 1] : 0);
            put(w, &sz, 8);
        }
        uint64_t b = r0 ? offs[r0 - 1] : 0;
        put(w, chars + b, offs[r1 - 1] - b);
        return;
    }
    for (int64_t i = r0; i < r1; ++i) {
        uint64_t b = i ? offs[i - 1] : 0;
        uint64_t sz = offs[i] - b - 1;
        put_varuint(w, sz);
        put(w, chars + b, sz);
    }
}

/* Encodes n rows as one packet.  version TFG_CODEC_V1 may split the rows into nparts parts of
 * part_rows[] rows (CHBlockChunkCodecV1::encode of a vector of blocks); nparts == 0 means one
 * part.  Returns the packet bytes, or (size_t)-1 on a bad type / overflow of `cap`. */
size_t orc_codec_encode(int version, int ncols, const char *const *names, const char *const *types,
                        const void *const *data, const uint64_t *const *offsets, const uint8_t *const *nullmaps,
                        int64_t n, int nparts, const int64_t *part_rows, uint8_t *out, size_t cap)
{
    orc_ctype t[256];
    if (ncols > 256) return (size_t)-1;
    for (int c = 0; c < ncols; ++c)
        if (parse_type(types[c], &t[c])) return (size_t)-1;
    wbuf w = {out, cap, 0, 0};
    if (version == TFG_CODEC_V1) {
        if (n == 0) return 0;
        uint8_t m = 0x02; /* CompressionMethodByte::NONE */
        put(&w, &m, 1);
        put_varuint(&w, (uint64_t)ncols);
        put_varuint(&w, (uint64_t)n);
        for (int c = 0; c < ncols; ++c) {
            put_str(&w, names[c]);
            put_str(&w, types[c]);
        }
        int64_t r0 = 0;
        int np = nparts > 0 ? nparts : 1;
        for (int p = 0; p < np; ++p) {
            int64_t rows = nparts > 0 ? part_rows[p] : n;
            if (rows == 0) continue; /* encodeColumnImpl skips empty blocks */
            put_varuint(&w, (uint64_t)rows);
            for (int c = 0; c < ncols; ++c) put_column(&w, &t[c], data[c], offsets[c], nullmaps[c], r0, r0 + rows);
            r0 += rows;
        }
    } else {
        put_varuint(&w, (uint64_t)ncols);
        put_varuint(&w, (uint64_t)n);
        for (int c = 0; c < ncols; ++c) {
            put_str(&w, names[c]);
            put_str(&w, types[c]);
            if (n) put_column(&w, &t[c], data[c], offsets[c], nullmaps[c], 0, n);
        }
    }
    return w.overflow ? (size_t)-1 : w.at;
}

/* Legacy String bulk decode (deserializeBinarySSE2): rows records at p -> chars (with '\0'
 * terminators) + end offsets; returns bytes consumed, or (size_t)-1 if truncated.  The CPU
 * baseline of the decode side. */
size_t orc_codec_decode_strings(const uint8_t *p, size_t avail, int64_t rows, uint8_t *chars, uint64_t *offs)
{
    size_t pos = 0;
    uint64_t o = 0;
    for (int64_t i = 0; i < rows; ++i) {
        uint64_t sz = 0;
        int k = 0;
        for (;; ++k) {
            if (pos >= avail || k >= 10) return (size_t)-1;
            uint8_t b = p[pos++];
            sz |= (uint64_t)(b & 0x7F) << (7 * k);
            if (!(b & 0x80)) break;
        }
        if (sz > avail - pos) return (size_t)-1;
        memcpy(chars + o, p + pos, sz);
        pos += sz;
        o += sz;
        chars[o++] = 0;
        offs[i] = o;
    }
    return pos;
}
