// zstd_dec.h — ZSTD frame decoder (RFC 8878) for the HC-mode MPP packets (§8 f1).
//
// The reference compresses each CompressedWriteBuffer frame of a V1 packet with ZSTD in
// HIGH_COMPRESSION mode (Flash/Coprocessor/CHBlockChunkCodecV1.cpp:150-160; IO/Compression/
// CompressionCodecZSTD.cpp:38-65: ZSTD_compress2 / ZSTD_decompress of contrib zstd, a third-party
// dependency the reference does not vendor).  This is a from-scratch restatement of the published
// format: frame header, raw / RLE / compressed blocks, Huffman-coded literals (1 or 4 streams,
// FSE-compressed or direct weights, treeless reuse), FSE-coded sequences (predefined, RLE,
// compressed and repeat modes) with the three repeat offsets, and the XXH64 content checksum.
// No dictionaries.  Every read is bounds-checked: a malformed frame is an error, never a write
// outside the caller's buffers.
//
// The decode is split so that the serial parts are short and the byte work is parallel:
//   1. scan (zstd_scan, one thread per packet frame): frame and block headers, the literal-section
//      and sequence-section headers and the table descriptions' extents — no entropy decoding.
//      Emits one ZBlockDesc per block (where its literals / sequences start, which Huffman and
//      FSE table descriptions are in force — treeless / repeat modes point at an earlier block's)
//      and one ZFrameDesc per ZSTD frame; a first pass only counts, so the outputs are sized
//      exactly.  Every block's literals and records then have fixed slots.
//   2. entropy (per block, independently): tables from the descriptions, Huffman literals,
//      FSE sequences -> records {literal length, match length, offset code} (repeat codes
//      unresolved: they depend on earlier blocks).  Every block ends with a literal-run record.
//   3. resolve (one wave per packet frame): repeat offsets in order, each record's output and
//      literal positions (wave scans), and the checks (offsets inside their frame, sizes).
//   4. execution: every output byte at once — literal bytes copied, a match byte points at its
//      source byte; pointer jumping (src = src[src]) until every byte points at a literal; one
//      gather.  Matches that copy matches (chains) resolve in log2(chain) rounds.
// The device runs 2-4 as kernels (zstd.hip); zstd_frame below runs 1-3 on the host plus a serial
// replay: the CPU check of the decoder's source against the system libzstd (tests/test_zstd.py).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define ZHD __host__ __device__ __forceinline__
#else
#define ZHD inline
#endif

namespace tfz {

constexpr int ZMAX_BLOCK = 128 * 1024;
constexpr int ZHUF_MAXBITS = 11;
constexpr uint32_t ZNONE = 0xFFFFFFFFu;
constexpr uint32_t ZDIRECT = 0x80000000u; // ZRec::of flag: a literal run / RLE copy, not a sequence

struct FseEntry {
    uint16_t base; // newState base
    uint8_t sym;
    uint8_t bits;
};

// A sequence decoding-table entry: the FSE state transition (base, bits) and the symbol's
// baseline + additional bits (literal / match length codes, or offset code c: 1 << c, c bits),
// so each of the three codes of a sequence costs one table read (zstd's ZSTD_seqSymbol).
struct alignas(8) ZSeqEntry { // 8 bytes: one LDS read per code
    uint32_t value; // baseline of the decoded value
    uint16_t base;  // next-state base
    uint8_t bits;   // next-state bits
    uint8_t sym;    // the code while the table is built, then the value's additional bits
};

// The sequence tables of one block (LDS on the device, 10 KB)
struct ZSeqTables {
    ZSeqEntry ll[512], of[256], ml[512]; // accuracy logs <= 9 / 8 / 9
    int ll_log, of_log, ml_log;
};
// ... and the one-symbol Huffman table (the host form; the device builds a two-symbol table
// straight from the weights, zstd.hip)
struct ZTables : ZSeqTables {
    uint16_t huf[1 << ZHUF_MAXBITS]; // symbol | nbBits << 8
    int huf_bits;
};

// One block (scan output).  Offsets are into the packet frame's ZSTD body.
struct ZBlockDesc {
    uint32_t src, size; // block content
    uint8_t type;       // 0 raw, 1 RLE, 2 compressed
    uint8_t ltype;      // literals: 0 raw, 1 RLE, 2 compressed, 3 treeless
    uint8_t streams;    // Huffman streams (1 / 4)
    uint8_t pad;
    uint32_t lit_at;    // literal section payload: raw / RLE bytes, or the Huffman streams
    uint32_t lsize;     // regenerated literal bytes (raw block: size, RLE block: 1)
    uint32_t lbytes;    // compressed literal bytes (streams incl. the jump table)
    uint32_t huf;       // Huffman tree description in force (ltype 2 / 3), its extent huf_n
    uint32_t huf_n;
    uint32_t tab[3];    // LL / OF / ML: mode << 30 | offset of the description (mode 2) / byte (mode 1)
    uint32_t tab_n[3];  // description extents (mode 2)
    uint32_t seq_at, seq_n; // sequence bitstream
    uint32_t nseq;
    uint32_t pframe;    // packet frame (launch-relative)
    uint32_t rec, lit;  // launch-relative index of the block's first record / literal byte
};

// One ZSTD frame (scan output; resolve fills out0 / out1, frame-relative output positions)
struct ZFrameDesc {
    uint32_t rec0, rec1;   // its records, launch-relative
    uint64_t fcs;          // content size, ~0 = absent
    uint32_t checksum, has_checksum;
    uint32_t out0, out1;
    uint32_t pframe, pad;
};

// A record.  Stage 2 writes {ll, ml, of, 0}: of = the sequence's offset value (RFC "Offset_Value":
// 1-3 repeat codes, offset + 3 otherwise), or ZDIRECT | offset for a literal run / RLE copy.
// Resolve rewrites it in place as {pos, ll, lpos, off}: output position (packet-frame-relative),
// literal run length, literal position (launch-relative) and the resolved offset; the record's
// end is the next record's pos.
struct ZRec {
    uint32_t a, b, c, d;
};

// counts of one packet frame (scan pass 1)
struct ZCounts {
    uint32_t blocks, frames, recs, max_comp;
};

// ---------------------------------------------------------------- constants (RFC 8878 §3.1.1.3.2.2)
ZHD uint32_t ll_base(int c) {
    static constexpr uint32_t t[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10,  11,  12,  13,   14,   15,   16,   18,
                            20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
    return t[c];
}
ZHD int ll_bits(int c) {
    static constexpr uint8_t t[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                           1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
    return t[c];
}
ZHD uint32_t ml_base(int c) {
    if (c < 32) return (uint32_t)c + 3;
    static constexpr uint32_t t[21] = {35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
    return t[c - 32];
}
ZHD int ml_bits(int c) {
    if (c < 32) return 0;
    static constexpr uint8_t t[21] = {1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
    return t[c - 32];
}
// predefined distributions (RFC 8878 §3.1.1.3.2.2.1-3)
ZHD int16_t ll_default(int s) {
    static constexpr int16_t t[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                           2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
    return t[s];
}
ZHD int16_t ml_default(int s) {
    if (s == 0) return 1;
    if (s <= 8) {
        static constexpr int16_t t[8] = {4, 3, 2, 2, 2, 2, 2, 2};
        return t[s - 1];
    }
    return s <= 45 ? 1 : -1;
}
ZHD int16_t of_default(int s) {
    static constexpr int16_t t[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
    return t[s];
}

ZHD int highbit(uint32_t v) { // index of the highest set bit (v > 0)
    int r = 0;
    while (v >>= 1) ++r;
    return r;
}

// ---------------------------------------------------------------- bit readers
// forward, LSB first (FSE table descriptions)
struct FwdBits {
    const uint8_t *p;
    int64_t nbytes;
    int64_t pos; // bits consumed
    ZHD uint32_t peek(int n) const { // n <= 25
        uint32_t v = 0;
        const int64_t b0 = pos >> 3;
        for (int k = 0; k < 4; ++k)
            if (b0 + k < nbytes) v |= (uint32_t)p[b0 + k] << (8 * k);
        return (v >> (pos & 7)) & ((n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1));
    }
    ZHD void skip(int n) { pos += n; }
};

// backward bitstream (Huffman streams, FSE bitstreams): the stream's last byte holds a 1 marker
// above the padding; bits are read from the top down.  `pos` = bits still unread; a 64-bit window
// of stream bits [wlo, wlo + 64) (wlo a multiple of 8) is refilled when a read would leave it:
// after a refill at least 57 bits can be read.  Bytes outside the stream read as zeros (a read
// past the start makes pos negative: the overflow the decoders check).  ALIGNED: the stream lives
// in a buffer that may be read in aligned 8-byte words up to 15 bytes past its end (the LDS stage).
ZHD uint64_t zload64(const uint8_t *p, int64_t off, int64_t n) {
    uint64_t v = 0;
    for (int k = 0; k < 8; ++k)
        if (off + k >= 0 && off + k < n) v |= (uint64_t)p[off + k] << (8 * k);
    return v;
}
template <bool ALIGNED = false> struct BitR {
    const uint8_t *p;
    int64_t n;
    int64_t pos;
    int64_t wlo;
    uint64_t win;
    ZHD bool init(const uint8_t *buf, int64_t len) {
        p = buf;
        n = len;
        if (len <= 0) return false;
        const uint8_t last = buf[len - 1];
        if (!last) return false;
        int hb = 0;
        for (uint32_t v = last; v >>= 1;) ++hb;
        pos = (len - 1) * 8 + hb;
        refill();
        return true;
    }
    ZHD void refill() { // the window ends at the byte holding bit pos - 1
        const int64_t b0 = ((pos + 7) >> 3) - 8;
        wlo = b0 * 8;
#if defined(__HIP_DEVICE_COMPILE__)
        if (ALIGNED && b0 >= 0 && b0 + 8 <= n) { // two aligned LDS words (local address space)
            typedef __attribute__((address_space(3))) const uint64_t lds_u64;
            const uint8_t *q = p + b0;
            const uint32_t sh = (uint32_t)((uintptr_t)q & 7) * 8;
            lds_u64 *w = (lds_u64 *)(q - ((uintptr_t)q & 7));
            const uint64_t lo = w[0], hi = w[1];
            win = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
            return;
        }
#endif
        win = zload64(p, b0, n);
    }
    ZHD void need(int k) { // the next k bits (k <= 57) are in the window
        if (pos - k < wlo) refill();
    }
    ZHD uint64_t peek(int k) const { // k <= 57, after need(k)
        if (k == 0) return 0;
        return (win >> (pos - k - wlo)) & ((1ull << k) - 1);
    }
    ZHD uint64_t read(int k) {
        need(k);
        const uint64_t v = peek(k);
        pos -= k;
        return v;
    }
};

// ---------------------------------------------------------------- FSE
// FSE table description -> normalized counts (RFC 8878 §4.1.1); returns bytes used, -1 on error
ZHD int64_t fse_read_ncount(const uint8_t *src, int64_t n, int max_log, int max_sym, int16_t *norm, int &log,
                            int &nsym) {
    if (n < 1) return -1;
    FwdBits fb{src, n, 0};
    log = (int)fb.peek(4) + 5;
    fb.skip(4);
    if (log > max_log) return -1;
    int remaining = (1 << log) + 1, threshold = 1 << log, nbits = log + 1, s = 0;
    bool prev0 = false;
    while (remaining > 1 && s <= max_sym) {
        if (prev0) { // repeat flags: 2-bit fields, 3 = three more zeros and another field
            int z = 0;
            for (;;) {
                if ((fb.pos >> 3) > n) return -1;
                const int f = (int)fb.peek(2);
                fb.skip(2);
                z += f;
                if (f != 3) break;
            }
            if (s + z > max_sym + 1) return -1;
            for (int k = 0; k < z; ++k) norm[s++] = 0;
            if (s > max_sym) break;
        }
        const int max = (2 * threshold - 1) - remaining;
        int count;
        const uint32_t v = fb.peek(nbits);
        if ((int)(v & (threshold - 1)) < max) {
            count = (int)(v & (threshold - 1));
            fb.skip(nbits - 1);
        } else {
            count = (int)(v & (2 * threshold - 1));
            if (count >= threshold) count -= max;
            fb.skip(nbits);
        }
        --count; // -1: "less than 1" probability
        remaining -= count < 0 ? -count : count;
        norm[s++] = (int16_t)count;
        prev0 = count == 0;
        while (remaining < threshold) {
            --nbits;
            threshold >>= 1;
        }
        if ((fb.pos >> 3) > n) return -1;
    }
    if (remaining != 1) return -1;
    nsym = s;
    return (fb.pos + 7) >> 3;
}

// decoding table from normalized counts (FSE_buildDTable)
// next: 256 words of work space (device: LDS — a private array would live in scratch memory)
template <typename E> ZHD bool fse_build(E *t, const int16_t *norm, int nsym, int log, uint16_t *next) {
    const int size = 1 << log;
    int high = size - 1;
    for (int s = 0; s < nsym; ++s) {
        if (norm[s] == -1) {
            t[high--].sym = (uint8_t)s;
            next[s] = 1;
        } else {
            next[s] = (uint16_t)norm[s];
        }
    }
    const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    int pos = 0;
    for (int s = 0; s < nsym; ++s)
        for (int i = 0; i < norm[s]; ++i) {
            t[pos].sym = (uint8_t)s;
            do
                pos = (pos + step) & mask;
            while (pos > high);
        }
    if (pos != 0) return false;
    for (int u = 0; u < size; ++u) {
        const int s = t[u].sym;
        const uint32_t ns = next[s]++;
        const int nb = log - highbit(ns);
        t[u].bits = (uint8_t)nb;
        t[u].base = (uint16_t)((ns << nb) - size);
    }
    return true;
}

template <typename E> ZHD void fse_rle(E *t, int sym) {
    t[0].sym = (uint8_t)sym;
    t[0].bits = 0;
    t[0].base = 0;
}

// ---------------------------------------------------------------- Huffman
// Huffman tree description (RFC 8878 §4.2.1) -> the weights of symbols 0 .. nw - 1 (the last
// one completed to a power of two) and the table's index bits; returns bytes used or -1.
// Work space: ft (64 entries), norm (16), next (256) — LDS on the device.
ZHD int64_t huf_weights(const uint8_t *src, int64_t n, uint8_t *weight, int &nw_out, int &maxbits_out, FseEntry *ft,
                        int16_t *norm, uint16_t *next) {
    if (n < 1) return -1;
    int nw = 0;
    int64_t used;
    const int hb = src[0];
    if (hb >= 128) { // direct 4-bit weights
        nw = hb - 127;
        used = 1 + (nw + 1) / 2;
        if (used > n) return -1;
        for (int i = 0; i < nw; ++i) {
            const uint8_t b = src[1 + i / 2];
            weight[i] = (i & 1) ? (b & 15) : (b >> 4);
        }
    } else { // FSE-compressed weights, two interleaved states
        used = 1 + hb;
        if (used > n || hb == 0) return -1;
        int log, nsym;
        const int64_t hd = fse_read_ncount(src + 1, hb, 6, 15, norm, log, nsym);
        if (hd < 0 || hd >= hb) return -1;
        if (!fse_build(ft, norm, nsym, log, next)) return -1;
        BitR<> bb;
        if (!bb.init(src + 1 + hd, hb - hd)) return -1;
        uint32_t s1 = (uint32_t)bb.read(log), s2 = (uint32_t)bb.read(log);
        for (;;) {
            if (nw > 253) return -1;
            weight[nw++] = ft[s1].sym;
            s1 = ft[s1].base + (uint32_t)bb.read(ft[s1].bits);
            if (bb.pos < 0) {
                weight[nw++] = ft[s2].sym;
                break;
            }
            weight[nw++] = ft[s2].sym;
            s2 = ft[s2].base + (uint32_t)bb.read(ft[s2].bits);
            if (bb.pos < 0) {
                weight[nw++] = ft[s1].sym;
                break;
            }
        }
    }
    // the last symbol's weight: completes the sum to the next power of two
    uint32_t sum = 0;
    for (int i = 0; i < nw; ++i) {
        if (weight[i] > ZHUF_MAXBITS) return -1;
        if (weight[i]) sum += 1u << (weight[i] - 1);
    }
    if (sum == 0 || nw > 255) return -1;
    const int maxbits = highbit(sum) + 1;
    if (maxbits > ZHUF_MAXBITS) return -1;
    const uint32_t rest = (1u << maxbits) - sum;
    if (rest & (rest - 1)) return -1; // not a power of two
    weight[nw++] = (uint8_t)(highbit(rest) + 1);
    nw_out = nw;
    maxbits_out = maxbits;
    return used;
}

// weight class k of a table of `maxbits` index bits: symbols of weight k take 2^(k-1) entries
// each, in symbol order, from start[k] (HUF_readDTableX1); false when the weights do not fill it
ZHD bool huf_class_starts(const uint8_t *weight, int nw, int maxbits, uint32_t (&start)[ZHUF_MAXBITS + 2]) {
    uint32_t cnt[ZHUF_MAXBITS + 2] = {};
    for (int i = 0; i < nw; ++i) cnt[weight[i]]++;
    uint32_t acc = 0;
    for (int k = 0; k <= ZHUF_MAXBITS + 1; ++k) start[k] = 0;
    for (int k = 1; k <= maxbits; ++k) {
        start[k] = acc;
        acc += cnt[k] << (k - 1);
    }
    start[maxbits + 1] = acc;
    return acc == (1u << maxbits);
}

// the one-symbol table: entry = symbol | nbBits << 8, nbBits = maxbits + 1 - weight
ZHD int64_t huf_read(const uint8_t *src, int64_t n, ZTables &t) {
    uint8_t weight[256];
    FseEntry ft[64];
    int16_t norm[16];
    uint16_t next[256];
    int nw = 0, maxbits = 0;
    const int64_t used = huf_weights(src, n, weight, nw, maxbits, ft, norm, next);
    if (used < 0) return -1;
    uint32_t start[ZHUF_MAXBITS + 2];
    if (!huf_class_starts(weight, nw, maxbits, start)) return -1;
    for (int i = 0; i < nw; ++i) {
        const int wt = weight[i];
        if (!wt) continue;
        const uint32_t len = 1u << (wt - 1);
        const uint16_t e = (uint16_t)(i | ((maxbits + 1 - wt) << 8));
        for (uint32_t k = 0; k < len; ++k) t.huf[start[wt] + k] = e;
        start[wt] += len;
    }
    t.huf_bits = maxbits;
    return used;
}

// one Huffman stream of `count` literals into out
template <bool AL = false> ZHD bool huf_stream(const ZTables &t, const uint8_t *src, int64_t n, uint8_t *out, int64_t count) {
    BitR<AL> bb;
    if (!bb.init(src, n)) return false;
    const int mb = t.huf_bits;
    for (int64_t i = 0; i < count; ++i) {
        bb.need(mb);
        const uint16_t e = t.huf[bb.peek(mb)];
        out[i] = (uint8_t)e;
        bb.pos -= e >> 8;
        if (bb.pos < 0) return false;
    }
    return bb.pos == 0;
}

// the four streams of a block's literals: extents from the 6-byte jump table; stream k decodes
// literals [k * seg, ...) of the block (seg = ceil(lsize / 4)); false when the table is invalid
struct Huf4 {
    int64_t at[4], len[4], cnt[4], seg;
};
ZHD bool huf4_split(const uint8_t *cs, int64_t cn, uint32_t lsize, Huf4 &h) {
    if (cn < 6) return false;
    const int64_t s1 = cs[0] | (cs[1] << 8), s2 = cs[2] | (cs[3] << 8), s3 = cs[4] | (cs[5] << 8);
    const int64_t s4 = cn - 6 - s1 - s2 - s3;
    if (s4 < 1) return false;
    h.seg = (lsize + 3) / 4;
    if (3 * h.seg > (int64_t)lsize) return false;
    h.at[0] = 6;
    h.at[1] = 6 + s1;
    h.at[2] = 6 + s1 + s2;
    h.at[3] = 6 + s1 + s2 + s3;
    h.len[0] = s1;
    h.len[1] = s2;
    h.len[2] = s3;
    h.len[3] = s4;
    for (int k = 0; k < 4; ++k) h.cnt[k] = k < 3 ? h.seg : (int64_t)lsize - 3 * h.seg;
    return true;
}

// ---------------------------------------------------------------- XXH64 (content checksum)
ZHD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
ZHD uint64_t rd64(const uint8_t *p) {
    uint64_t v = 0;
    for (int k = 0; k < 8; ++k) v |= (uint64_t)p[k] << (8 * k);
    return v;
}
ZHD uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
ZHD uint64_t xxh64(const uint8_t *p, uint64_t len) {
    const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                   P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
    const uint8_t *e = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
        const uint8_t *lim = e - 32;
        do {
            v1 = rotl64(v1 + rd64(p) * P2, 31) * P1;
            v2 = rotl64(v2 + rd64(p + 8) * P2, 31) * P1;
            v3 = rotl64(v3 + rd64(p + 16) * P2, 31) * P1;
            v4 = rotl64(v4 + rd64(p + 24) * P2, 31) * P1;
            p += 32;
        } while (p <= lim);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        const uint64_t vs[4] = {v1, v2, v3, v4};
        for (int k = 0; k < 4; ++k) {
            const uint64_t v = rotl64(vs[k] * P2, 31) * P1;
            h = (h ^ v) * P1 + P4;
        }
    } else {
        h = P5;
    }
    h += len;
    while (p + 8 <= e) {
        h ^= rotl64(rd64(p) * P2, 31) * P1;
        h = rotl64(h, 27) * P1 + P4;
        p += 8;
    }
    if (p + 4 <= e) {
        h ^= (uint64_t)rd32(p) * P1;
        h = rotl64(h, 23) * P2 + P3;
        p += 4;
    }
    while (p < e) {
        h ^= (*p) * P5;
        h = rotl64(h, 11) * P1;
        ++p;
    }
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

// ---------------------------------------------------------------- sequence tables
// symbol -> baseline and additional bits for every entry of a sequence table of `size` entries
// (kind 0 literal lengths, 1 offsets, 2 match lengths); false on a symbol past the kind's range.
// Offset codes stop at 30: a larger offset cannot fall inside a packet frame (<= 1 GB), and the
// record's offset field keeps its top bit for ZDIRECT.
ZHD bool seq_finish(ZSeqEntry *t, int size, int kind) {
    const int max_sym = kind == 0 ? 35 : kind == 1 ? 30 : 52;
    for (int u = 0; u < size; ++u) {
        const int c = t[u].sym;
        if (c > max_sym) return false;
        t[u].value = kind == 0 ? ll_base(c) : kind == 1 ? (1u << c) : ml_base(c);
        t[u].sym = (uint8_t)(kind == 0 ? ll_bits(c) : kind == 1 ? c : ml_bits(c)); // now: additional bits
    }
    return true;
}

// the table of one kind from its description (ZBlockDesc::tab: mode << 30 | offset into `body`)
// norm (53 entries) and next (256): work space, LDS on the device
ZHD bool seq_table_build(ZSeqTables &t, int kind, uint32_t tab, uint32_t tab_n, const uint8_t *body, int16_t *norm,
                         uint16_t *next) {
    ZSeqEntry *e = kind == 0 ? t.ll : kind == 1 ? t.of : t.ml;
    int &log = kind == 0 ? t.ll_log : kind == 1 ? t.of_log : t.ml_log;
    const int mode = (int)(tab >> 30);
    const uint32_t at = tab & 0x3FFFFFFFu;
    const int max_sym = kind == 0 ? 35 : kind == 1 ? 31 : 52, max_log = kind == 1 ? 8 : 9;
    if (mode == 0) { // predefined
        const int nsym = kind == 0 ? 36 : kind == 1 ? 29 : 53;
        for (int s = 0; s < nsym; ++s) norm[s] = kind == 0 ? ll_default(s) : kind == 1 ? of_default(s) : ml_default(s);
        log = kind == 1 ? 5 : 6;
        return fse_build(e, norm, nsym, log, next) && seq_finish(e, 1 << log, kind);
    }
    if (mode == 1) { // RLE
        fse_rle(e, body[at]);
        log = 0;
        return seq_finish(e, 1, kind);
    }
    int nsym;
    if (fse_read_ncount(body + at, tab_n, max_log, max_sym, norm, log, nsym) < 0) return false;
    return fse_build(e, norm, nsym, log, next) && seq_finish(e, 1 << log, kind);
}

// The sequences of one block: put(q, record) for q = 0 .. nseq (the last: the block's trailing
// literal run).  false when the bitstream is malformed or a literal length runs past lsize.
template <bool AL, typename Put>
ZHD bool seq_decode(const ZSeqTables &t, const uint8_t *bits, int64_t n, uint32_t nseq, uint32_t lsize, Put &&put) {
    uint32_t lit_pos = 0;
    if (nseq) {
        BitR<AL> bb;
        if (!bb.init(bits, n)) return false;
        uint32_t sll = (uint32_t)bb.read(t.ll_log), sof = (uint32_t)bb.read(t.of_log), sml = (uint32_t)bb.read(t.ml_log);
        for (uint32_t q = 0; q < nseq; ++q) {
            const ZSeqEntry el = t.ll[sll], eo = t.of[sof], em = t.ml[sml];
            const uint32_t ofv = eo.value + (uint32_t)bb.read(eo.sym);
            bb.need(32);
            const uint32_t ml = em.value + (uint32_t)bb.peek(em.sym);
            bb.pos -= em.sym;
            const uint32_t ll = el.value + (uint32_t)bb.peek(el.sym);
            bb.pos -= el.sym;
            if (q + 1 < nseq) { // state updates: LL, ML, OF
                bb.need(26);
                sll = el.base + (uint32_t)bb.peek(el.bits);
                bb.pos -= el.bits;
                sml = em.base + (uint32_t)bb.peek(em.bits);
                bb.pos -= em.bits;
                sof = eo.base + (uint32_t)bb.peek(eo.bits);
                bb.pos -= eo.bits;
            }
            if (bb.pos < 0 || lit_pos + ll > lsize) return false;
            put(q, ZRec{ll, ml, ofv, 0});
            lit_pos += ll;
        }
        if (bb.pos != 0) return false;
    }
    put(nseq, ZRec{lsize - lit_pos, 0, ZDIRECT, 0});
    return true;
}

// ---------------------------------------------------------------- stage 1: scan
// One packet frame's ZSTD body (n bytes), which decodes to `raw` bytes.  Pass 1 (blocks null)
// only counts; pass 2 writes the descriptors at the launch-relative bases (by `writer` lanes).
struct ZScan {
    ZBlockDesc *blocks = nullptr;
    ZFrameDesc *frames = nullptr;
    uint32_t block0 = 0, frame0 = 0, rec0 = 0, lit0 = 0, pframe = 0;
    bool writer = true;
    ZCounts c{};
};

// byte source of the scan: at(off, k) -> k readable bytes at off (k <= ZSCAN_WIN, off + k <= n)
constexpr int ZSCAN_WIN = 512; // covers a sequence section's header and its three table descriptions
struct ZSrcMem {
    const uint8_t *p;
    ZHD const uint8_t *at(int64_t off, int64_t) const { return p + off; }
};

template <typename Src> ZHD bool zstd_scan(Src &S, int64_t n, uint64_t raw, ZScan &o) {
    if (n >= (1ll << 30)) return false; // description offsets keep 30 bits
    o.c = ZCounts{0, 0, 0, 0};
    int64_t ip = 0;
    uint64_t lits = 0;
    while (ip < n) {
        if (ip + 4 > n) return false;
        const uint32_t magic = rd32(S.at(ip, 4));
        ip += 4;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) { // skippable
            if (ip + 4 > n) return false;
            const uint32_t sz = rd32(S.at(ip, 4));
            ip += 4 + (int64_t)sz;
            if (ip > n) return false;
            continue;
        }
        if (magic != 0xFD2FB528u || ip >= n) return false;
        const uint8_t *h = S.at(ip, n - ip < 14 ? n - ip : 14); // descriptor .. content size: <= 14 bytes
        const int64_t h0 = ip;
        const int fhd = h[0];
        ++ip;
        const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did = fhd & 3;
        if (fhd & 8) return false; // reserved bit
        if (!single) ++ip;         // window descriptor (the output buffer is the whole frame)
        const int did_len = did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4;
        if (ip + did_len > n) return false;
        uint32_t dict = 0;
        for (int k = 0; k < did_len; ++k) dict |= (uint32_t)h[ip - h0 + k] << (8 * k);
        if (dict) return false;
        ip += did_len;
        const int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        if (ip + fcs_len > n) return false;
        uint64_t fcs = 0;
        for (int k = 0; k < fcs_len; ++k) fcs |= (uint64_t)h[ip - h0 + k] << (8 * k);
        if (fcs_len == 2) fcs += 256;
        ip += fcs_len;
        ZFrameDesc fd{};
        fd.rec0 = o.rec0 + o.c.recs;
        fd.fcs = fcs_len ? fcs : ~0ull;
        fd.pframe = o.pframe;
        uint32_t huf = ZNONE, huf_n = 0, tab[3] = {ZNONE, ZNONE, ZNONE}, tab_n[3] = {0, 0, 0};
        for (;;) {
            if (ip + 3 > n) return false;
            const int64_t hk = n - ip < 8 ? n - ip : 8; // block header + the literals header
            const uint8_t *bh8 = S.at(ip, hk);
            const uint32_t bh = (uint32_t)bh8[0] | (uint32_t)bh8[1] << 8 | (uint32_t)bh8[2] << 16;
            ip += 3;
            const int last = bh & 1, btype = (bh >> 1) & 3;
            const uint32_t bsize = bh >> 3;
            if (btype == 3 || bsize > (uint32_t)ZMAX_BLOCK) return false;
            ZBlockDesc d{};
            d.src = (uint32_t)ip;
            d.size = bsize;
            d.type = (uint8_t)(btype == 0 ? 0 : btype == 1 ? 1 : 2);
            d.pframe = o.pframe;
            d.rec = o.rec0 + o.c.recs;
            d.lit = o.lit0 + (uint32_t)lits;
            uint32_t nrec = 1;
            if (btype == 0) {
                if (ip + bsize > n) return false;
                d.lsize = bsize;
                ip += bsize;
            } else if (btype == 1) {
                if (ip + 1 > n) return false;
                d.lsize = bsize ? 1 : 0;
                ip += 1;
            } else {
                if (ip + bsize > n || bsize < 1) return false;
                const int64_t bn = bsize;
                const uint8_t *b = bh8 + 3; // the literals header (bytes past the block read as 0)
                uint8_t lh[5];
                for (int k = 0; k < 5; ++k) lh[k] = 3 + k < hk && k < bn ? b[k] : 0;
                // literals section header
                const int ltype = lh[0] & 3, sf = (lh[0] >> 2) & 3;
                int64_t lp = 0;
                uint32_t lsize = 0, csize = 0;
                int streams = 1;
                if (ltype <= 1) {
                    if ((sf & 1) == 0) {
                        lsize = lh[0] >> 3;
                        lp = 1;
                    } else if (sf == 1) {
                        if (bn < 2) return false;
                        lsize = (lh[0] >> 4) | ((uint32_t)lh[1] << 4);
                        lp = 2;
                    } else {
                        if (bn < 3) return false;
                        lsize = (lh[0] >> 4) | ((uint32_t)lh[1] << 4) | ((uint32_t)lh[2] << 12);
                        lp = 3;
                    }
                    csize = ltype == 0 ? lsize : 1;
                } else {
                    const int hl = sf <= 1 ? 3 : sf == 2 ? 4 : 5;
                    if (bn < hl) return false;
                    uint64_t v = 0;
                    for (int k = 0; k < hl; ++k) v |= (uint64_t)lh[k] << (8 * k);
                    const int bits = sf <= 1 ? 10 : sf == 2 ? 14 : 18;
                    lsize = (uint32_t)((v >> 4) & ((1u << bits) - 1));
                    csize = (uint32_t)((v >> (4 + bits)) & ((1u << bits) - 1));
                    streams = sf == 0 ? 1 : 4;
                    lp = hl;
                }
                if (lsize > (uint32_t)ZMAX_BLOCK || lp + csize > bn) return false;
                d.ltype = (uint8_t)ltype;
                d.streams = (uint8_t)streams;
                d.lsize = lsize;
                d.lit_at = (uint32_t)(ip + lp);
                d.lbytes = csize;
                if (ltype == 2) { // the tree description, then the streams
                    if (csize < 1) return false;
                    const int hb = S.at(ip + lp, 1)[0];
                    const int64_t tl = hb >= 128 ? 1 + (hb - 127 + 1) / 2 : 1 + hb;
                    if (tl >= (int64_t)csize) return false;
                    huf = d.lit_at;
                    huf_n = (uint32_t)tl;
                    d.lit_at += (uint32_t)tl;
                    d.lbytes -= (uint32_t)tl;
                } else if (ltype == 3 && huf == ZNONE) {
                    return false; // treeless without a previous table
                }
                d.huf = ltype >= 2 ? huf : ZNONE;
                d.huf_n = ltype >= 2 ? huf_n : 0;
                // sequences section header and table descriptions (within ZSCAN_WIN bytes)
                int64_t sp = lp + csize;
                if (sp >= bn) return false;
                const int64_t sw = bn - sp < ZSCAN_WIN ? bn - sp : ZSCAN_WIN;
                const uint8_t *q = S.at(ip + sp, sw); // q[x] = block byte sp + x, x < sw
                int64_t x = 0;
                uint32_t nseq;
                const int b0 = q[0];
                if (b0 < 128) {
                    nseq = (uint32_t)b0;
                    x = 1;
                } else if (b0 < 255) {
                    if (2 > sw) return false;
                    nseq = ((uint32_t)(b0 - 128) << 8) + q[1];
                    x = 2;
                } else {
                    if (3 > sw) return false;
                    nseq = q[1] + ((uint32_t)q[2] << 8) + 0x7F00;
                    x = 3;
                }
                if (nseq > (uint32_t)ZMAX_BLOCK / 3 + 1) return false; // every match is >= 3 bytes
                d.nseq = nseq;
                if (nseq) {
                    if (x >= sw) return false;
                    const int modes = q[x++];
                    if (modes & 3) return false; // reserved bits
                    const int mk[3] = {modes >> 6, (modes >> 4) & 3, (modes >> 2) & 3};
                    for (int k = 0; k < 3; ++k) {
                        const int m = mk[k];
                        if (m == 0) {
                            tab[k] = 0;
                            tab_n[k] = 0;
                        } else if (m == 1) {
                            if (x + 1 > sw) return false;
                            tab[k] = 1u << 30 | (uint32_t)(ip + sp + x);
                            tab_n[k] = 1;
                            x += 1;
                        } else if (m == 2) {
                            int16_t norm[53];
                            int log, nsym;
                            const int64_t u = fse_read_ncount(q + x, sw - x, k == 1 ? 8 : 9, k == 0 ? 35 : k == 1 ? 31 : 52,
                                                              norm, log, nsym);
                            if (u < 0) return false;
                            tab[k] = 2u << 30 | (uint32_t)(ip + sp + x);
                            tab_n[k] = (uint32_t)u;
                            x += u;
                        } else if (tab[k] == ZNONE) {
                            return false; // repeat mode without a previous table
                        }
                        d.tab[k] = tab[k];
                        d.tab_n[k] = tab_n[k];
                    }
                    if (sp + x >= bn) return false; // the bitstream holds at least its marker byte
                    d.seq_at = (uint32_t)(ip + sp + x);
                    d.seq_n = (uint32_t)(bn - sp - x);
                } else if (sp + x != bn) {
                    return false;
                }
                nrec = nseq + 1;
                if (bsize > o.c.max_comp) o.c.max_comp = bsize;
                ip += bsize;
            }
            lits += d.lsize;
            if (lits > raw) return false;
            if (o.blocks && o.writer) o.blocks[o.block0 + o.c.blocks] = d;
            ++o.c.blocks;
            o.c.recs += nrec;
            if (last) break;
        }
        if (checksum) {
            if (ip + 4 > n) return false;
            fd.checksum = rd32(S.at(ip, 4));
            fd.has_checksum = 1;
            ip += 4;
        }
        fd.rec1 = o.rec0 + o.c.recs;
        if (o.frames && o.writer) o.frames[o.frame0 + o.c.frames] = fd;
        ++o.c.frames;
    }
    return true;
}
ZHD bool zstd_scan(const uint8_t *src, int64_t n, uint64_t raw, ZScan &o) {
    ZSrcMem m{src};
    return zstd_scan(m, n, raw, o);
}

// ---------------------------------------------------------------- stage 3: resolve (one ZSTD frame)
// Repeat offsets in record order (RFC 8878 §3.1.2.5), positions, checks.  `pos` / `lpos`: the
// frame's first output position (packet-frame-relative) and literal index; advanced past it.
// One record: returns the resolved offset (0 = malformed) and updates the repeat offsets.
ZHD uint32_t rep_resolve(uint32_t of, uint32_t ll, uint32_t &r0, uint32_t &r1, uint32_t &r2) {
    if (of & ZDIRECT) return of & ~ZDIRECT;
    if (of > 3) {
        const uint32_t off = of - 3;
        r2 = r1;
        r1 = r0;
        r0 = off;
        return off;
    }
    const int idx = (int)of - 1 + (ll == 0 ? 1 : 0);
    if (idx == 0) return r0;
    const uint32_t t = idx == 3 ? r0 - 1 : idx == 1 ? r1 : r2;
    if (idx != 1) r2 = r1;
    r1 = r0;
    r0 = t;
    return t;
}

ZHD bool zstd_resolve_serial(ZRec *recs, ZFrameDesc &fr, uint64_t raw, uint64_t &pos, uint64_t &lpos) {
    const uint64_t zstart = pos;
    uint32_t r0 = 1, r1 = 4, r2 = 8;
    fr.out0 = (uint32_t)pos;
    for (uint32_t q = fr.rec0; q < fr.rec1; ++q) {
        const ZRec r = recs[q];
        const uint32_t ll = r.a, ml = r.b;
        const uint32_t off = rep_resolve(r.c, ll, r0, r1, r2);
        if (ml && (off == 0 || off > pos + ll - zstart)) return false;
        if (pos + ll + ml > raw) return false;
        recs[q] = ZRec{(uint32_t)pos, ll, (uint32_t)lpos, off};
        pos += (uint64_t)ll + ml;
        lpos += ll;
    }
    fr.out1 = (uint32_t)pos;
    return fr.fcs == ~0ull || pos - zstart == fr.fcs;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// ---------------------------------------------------------------- host form (tests)
// Stage 2 of one block on the host: literals to lits[d.lit ...], records to recs[d.rec ...].
inline bool zblock_decode_host(const uint8_t *body, const ZBlockDesc &d, ZTables &t, uint8_t *lits, ZRec *recs) {
    if (d.type == 0) {
        for (uint32_t i = 0; i < d.size; ++i) lits[d.lit + i] = body[d.src + i];
        recs[d.rec] = ZRec{d.size, 0, ZDIRECT, 0};
        return true;
    }
    if (d.type == 1) {
        if (d.size) lits[d.lit] = body[d.src];
        recs[d.rec] = ZRec{d.size ? 1u : 0u, d.size ? d.size - 1 : 0u, ZDIRECT | (d.size > 1 ? 1u : 0u), 0};
        return true;
    }
    uint8_t *lit = lits + d.lit;
    const uint8_t *ls = body + d.lit_at;
    if (d.ltype == 0) {
        for (uint32_t i = 0; i < d.lsize; ++i) lit[i] = ls[i];
    } else if (d.ltype == 1) {
        for (uint32_t i = 0; i < d.lsize; ++i) lit[i] = ls[0];
    } else {
        if (huf_read(body + d.huf, d.huf_n, t) < 0) return false;
        if (d.streams == 1) {
            if (!huf_stream(t, ls, d.lbytes, lit, d.lsize)) return false;
        } else {
            Huf4 h;
            if (!huf4_split(ls, d.lbytes, d.lsize, h)) return false;
            for (int k = 0; k < 4; ++k)
                if (!huf_stream(t, ls + h.at[k], h.len[k], lit + k * h.seg, h.cnt[k])) return false;
        }
    }
    if (d.nseq) {
        int16_t norm[53];
        uint16_t next[256];
        for (int k = 0; k < 3; ++k)
            if (!seq_table_build(t, k, d.tab[k], d.tab_n[k], body, norm, next)) return false;
    }
    return seq_decode<false>(t, body + d.seq_at, d.seq_n, d.nseq, d.lsize, [&](uint32_t q, const ZRec &r) { recs[d.rec + q] = r; });
}

// Host decode of one frame body that decodes to exactly `raw` bytes: the decoded size, or -1
// (tests/cpp/zstd_cpu.cpp).  Stages 1-3 as the device runs them, then a serial replay.
inline int64_t zstd_frame(const uint8_t *src, int64_t n, uint8_t *dst, uint64_t raw, uint64_t *nrec_out = nullptr) {
    ZScan s;
    if (!zstd_scan(src, n, raw, s)) return -1;
    ZScan f;
    f.blocks = new ZBlockDesc[s.c.blocks + 1];
    f.frames = new ZFrameDesc[s.c.frames + 1];
    ZRec *recs = new ZRec[s.c.recs + 1];
    uint8_t *lits = new uint8_t[raw + 1];
    ZTables *t = new ZTables;
    bool ok = zstd_scan(src, n, raw, f);
    for (uint32_t b = 0; ok && b < f.c.blocks; ++b) ok = zblock_decode_host(src, f.blocks[b], *t, lits, recs);
    uint64_t pos = 0, lpos = 0;
    for (uint32_t z = 0; ok && z < f.c.frames; ++z) ok = zstd_resolve_serial(recs, f.frames[z], raw, pos, lpos);
    ok = ok && pos == raw;
    for (uint32_t z = 0; ok && z < f.c.frames; ++z) {
        const ZFrameDesc &fr = f.frames[z];
        for (uint32_t q = fr.rec0; q < fr.rec1; ++q) {
            const ZRec r = recs[q];
            const uint64_t end = q + 1 < fr.rec1 ? recs[q + 1].a : fr.out1;
            for (uint32_t i = 0; i < r.b; ++i) dst[r.a + i] = lits[r.c + i];
            for (uint64_t p = r.a + r.b; p < end; ++p) dst[p] = dst[p - r.d];
        }
        if (fr.has_checksum && (uint32_t)xxh64(dst + fr.out0, fr.out1 - fr.out0) != fr.checksum) ok = false;
    }
    if (nrec_out) *nrec_out = s.c.recs;
    delete[] f.blocks;
    delete[] f.frames;
    delete[] recs;
    delete[] lits;
    delete t;
    return ok ? (int64_t)raw : -1;
}
#endif

} // namespace tfz
