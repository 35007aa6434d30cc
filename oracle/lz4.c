/* lz4.c — TEST INFRASTRUCTURE ONLY (the checker, never the product path).
 *
 * CPU restatement of the LZ4 block format and of the frame wrapping of LZ4 MPP packets:
 *  - frames: CompressedWriteBuffer<false> / CompressedReadBuffer<false> as CHBlockChunkCodecV1
 *    uses them (reference dbms/src/Flash/Coprocessor/CHBlockChunkCodecV1.cpp:391-429, 555-581;
 *    IO/Compression/CompressionInfo.h:24,53-58): 0x82 | UInt32 frame bytes incl. the 9-byte header
 *    | UInt32 raw bytes | LZ4 block; no checksum in the <false> instantiation;
 *  - the block: the published LZ4 block format (lz4 1.9.x, doc/lz4_Block_format.md) of the lz4
 *    library the reference links (third-party, not vendored under /root/reference).  The decoder
 *    follows LZ4_decompress_safe's acceptance rules; the compressor is a plain greedy hash-chain-
 *    free matcher (any valid block decodes to the same bytes: block bytes are not unique, parity
 *    is on round trips and on decoding independently-built blocks).
 * Parity: pinned by hand-derived blocks from the format description (tests/test_oracle_cpu.py);
 * the reference's own LZ4 tests are round trips (gtest_block_chunk_codec.cpp:260-360). */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

#define LZ4_MINMATCH 4
#define LZ4_LASTLITERALS 5
#define LZ4_MFLIMIT 12

/* LZ4_decompress_safe: returns the decoded size, or -1 on malformed input / overflow of dstcap.
 * A block is sequences; the last one holds literals only and ends the input exactly. */
int64_t orc_lz4_decompress_block(const uint8_t *src, size_t srclen, uint8_t *dst, size_t dstcap)
{
    size_t ip = 0, op = 0;
    if (srclen == 0) return -1;
    for (;;) {
        if (ip >= srclen) return -1;
        unsigned token = src[ip++];
        size_t lit = token >> 4;
        if (lit == 15) {
            unsigned b;
            do {
                if (ip >= srclen) return -1;
                b = src[ip++];
                lit += b;
            } while (b == 255);
        }
        if (lit > srclen - ip || lit > dstcap - op) return -1;
        memcpy(dst + op, src + ip, lit);
        ip += lit;
        op += lit;
        if (ip == srclen) return (int64_t)op;
        if (srclen - ip < 2) return -1;
        size_t off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
        ip += 2;
        size_t ml = (token & 15) + LZ4_MINMATCH;
        if ((token & 15) == 15) {
            unsigned b;
            do {
                if (ip >= srclen) return -1;
                b = src[ip++];
                ml += b;
            } while (b == 255);
        }
        if (off == 0 || off > op || ml > dstcap - op) return -1;
        for (size_t i = 0; i < ml; ++i) dst[op + i] = dst[op - off + i]; /* overlapping copy */
        op += ml;
    }
}

static size_t put_len(uint8_t *o, size_t v)
{
    size_t k = 0;
    v -= 15;
    while (v >= 255) {
        o[k++] = 255;
        v -= 255;
    }
    o[k++] = (uint8_t)v;
    return k;
}

static size_t emit(uint8_t *o, const uint8_t *lits, size_t lit, size_t off, size_t ml)
{
    size_t k = 0;
    size_t mcode = ml ? ml - LZ4_MINMATCH : 0;
    o[k++] = (uint8_t)(((lit < 15 ? lit : 15) << 4) | (mcode < 15 ? mcode : 15));
    if (lit >= 15) k += put_len(o + k, lit);
    memcpy(o + k, lits, lit);
    k += lit;
    if (!ml) return k;
    o[k++] = (uint8_t)off;
    o[k++] = (uint8_t)(off >> 8);
    if (mcode >= 15) k += put_len(o + k, mcode);
    return k;
}

/* Greedy LZ4 block of src[0, n) (window 64 KB, one-probe hash table); dst holds at least
 * orc_lz4_bound(n).  Returns the block size. */
size_t orc_lz4_bound(size_t n) { return n + n / 255 + 16; }

size_t orc_lz4_compress_block(const uint8_t *src, size_t n, uint8_t *dst)
{
    enum { HLOG = 14 };
    static __thread int64_t table[1 << HLOG];
    for (int i = 0; i < (1 << HLOG); ++i) table[i] = -1;
    size_t o = 0, anchor = 0, ip = 0;
    if (n >= LZ4_MFLIMIT + 1) {
        const size_t mflimit = n - LZ4_MFLIMIT, matchlimit = n - LZ4_LASTLITERALS;
        while (ip < mflimit) {
            uint32_t seq;
            memcpy(&seq, src + ip, 4);
            uint32_t h = (seq * 2654435761u) >> (32 - HLOG);
            int64_t ref = table[h];
            table[h] = (int64_t)ip;
            uint32_t rseq = 0;
            if (ref >= 0) memcpy(&rseq, src + ref, 4);
            if (ref >= 0 && ip - (size_t)ref <= 65535 && rseq == seq) {
                size_t ml = LZ4_MINMATCH;
                while (ip + ml < matchlimit && src[ref + ml] == src[ip + ml]) ++ml;
                o += emit(dst + o, src + anchor, ip - anchor, ip - (size_t)ref, ml);
                ip += ml;
                anchor = ip;
            } else {
                ++ip;
            }
        }
    }
    o += emit(dst + o, src + anchor, n - anchor, 0, 0);
    return o;
}

/* The LZ4 packet of an uncompressed V1 packet (0x02 + body): frames of frame_raw body bytes
 * (frame_raw = 0: one frame, as the reference's write buffer sized to the packet gives).
 * out == NULL: returns an upper bound; else the packet size. */
size_t orc_lz4_packet_compress(const uint8_t *pkt, size_t bytes, size_t frame_raw, uint8_t *out)
{
    if (bytes <= 1) return 0;
    const uint8_t *body = pkt + 1;
    size_t n = bytes - 1;
    if (frame_raw == 0) frame_raw = n;
    size_t nframes = (n + frame_raw - 1) / frame_raw;
    if (!out) return nframes * (9 + 16) + n + n / 255 + 16;
    size_t o = 0;
    for (size_t f = 0; f < nframes; ++f) {
        size_t len = n - f * frame_raw < frame_raw ? n - f * frame_raw : frame_raw;
        size_t blk = orc_lz4_compress_block(body + f * frame_raw, len, out + o + 9);
        uint32_t fb = (uint32_t)(blk + 9), rb = (uint32_t)len;
        out[o] = 0x82;
        memcpy(out + o + 1, &fb, 4);
        memcpy(out + o + 5, &rb, 4);
        o += fb;
    }
    return o;
}

/* CompressedReadBuffer over a whole LZ4 packet -> 0x02 + body.  out == NULL: the decoded size.
 * Returns -1 on malformed frames (wrong method byte, truncated, size mismatch). */
int64_t orc_lz4_packet_decompress(const uint8_t *pkt, size_t bytes, uint8_t *out, size_t cap)
{
    size_t pos = 0, raw = 0;
    while (pos < bytes) {
        if (bytes - pos < 9 || pkt[pos] != 0x82) return -1;
        uint32_t fb, rb;
        memcpy(&fb, pkt + pos + 1, 4);
        memcpy(&rb, pkt + pos + 5, 4);
        if (fb <= 9 || fb > bytes - pos) return -1;
        if (out) {
            if (1 + raw + rb > cap) return -1;
            int64_t got = orc_lz4_decompress_block(pkt + pos + 9, fb - 9, out + 1 + raw, rb);
            if (got != (int64_t)rb) return -1;
        }
        raw += rb;
        pos += fb;
    }
    if (out) {
        if (cap < 1) return -1;
        out[0] = 0x02;
    }
    return (int64_t)(raw + 1);
}
