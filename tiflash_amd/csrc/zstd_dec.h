// zstd_dec.h — ZSTD frame decoder (RFC 8878) for the HC-mode MPP packets (§8 f1).
//
// The reference compresses each CompressedWriteBuffer frame of a V1 packet with ZSTD in
// HIGH_COMPRESSION mode (Flash/Coprocessor/CHBlockChunkCodecV1.cpp:150-160; IO/Compression/
// CompressionCodecZSTD.cpp:38-65: ZSTD_compress2 / ZSTD_decompress of contrib zstd, a third-party
// dependency the reference does not vendor).  This is a from-scratch restatement of the published
// format: frame header, raw / RLE / compressed blocks, Huffman-coded literals (1 or 4 streams,
// FSE-compressed or direct weights, treeless reuse), FSE-coded sequences (predefined, RLE,
// compressed and repeat modes) with the three repeat offsets, and the XXH64 content checksum.
// No dictionaries.  Every read is bounds-checked: a malformed frame returns an error, never
// writes outside its buffers.
//
// Decoding is split in two stages, so that neither waits on the other's memory:
//   1. entropy (zstd_frame_entropy): block headers, Huffman literals and FSE sequences are decoded
//      into a flat list of ZSeq records {literal length, match length, resolved offset} and the
//      literal bytes, in output order.  Raw blocks become literal runs, RLE blocks one literal and
//      an offset-1 match; frame starts and content checksums become marker records.
//   2. execution: the records are replayed into the output (literal runs, then LZ77 matches).
// On the device (lz4.hip) stage 1 is one wave per packet frame with the compressed block staged in
// LDS (the wave decodes the sequences in lockstep; the four Huffman streams of a block go to four
// lanes) and stage 2 a second kernel, one wave per frame, whose output passes through a 64 KB LDS
// window: literal runs are copied by all lanes at once, matches are replayed one after another
// with all lanes copying, and the window is flushed to HBM once per batch of records.  The same
// stage-1 source runs on the host with zstd_exec_serial as stage 2 (zstd_frame): the CPU check of
// the decoder against the system libzstd (tests/test_zstd.py).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define ZHD __host__ __device__ __forceinline__
#else
#define ZHD inline
#endif
// Stage 1 on the device: all 64 lanes of a wave run the entropy decoding in lockstep (identical
// loads and branches in every lane) and split the stores: record q is stored by lane q % 64,
// literal bytes by lanes in turn, the four Huffman streams by lanes 0-3.  ZANY combines a per-lane
// condition over the wave (the Huffman stream checks).
#if defined(__HIP_DEVICE_COMPILE__)
#define ZSYNC_LDS() __syncthreads()
#define ZANY(x) (__ballot((int)(x)) != 0)
#else
#define ZSYNC_LDS() do { } while (0)
#define ZANY(x) (x)
#endif

namespace tfz {

constexpr int ZMAX_BLOCK = 128 * 1024;
constexpr int ZHUF_MAXBITS = 11;

struct FseEntry {
    uint16_t base; // newState base
    uint8_t sym;
    uint8_t bits;
};

// A sequence decoding-table entry: the FSE state transition (base, bits) and the symbol's
// baseline + additional bits (literal / match length codes, or offset code c: 1 << c, c bits),
// so each of the three codes of a sequence costs one table read (zstd's ZSTD_seqSymbol).
struct ZSeqEntry {
    uint32_t value; // baseline of the decoded value
    uint16_t base;  // next-state base
    uint8_t bits;   // next-state bits
    uint8_t sym;    // the code (while the table is built)
    uint8_t add;    // additional bits of the value
};

struct ZWork {
    ZSeqEntry ll[512], of[256], ml[512]; // accuracy logs <= 9 / 8 / 9
    int ll_log, of_log, ml_log;
    bool ll_ok, of_ok, ml_ok;             // a table exists for Repeat mode
    uint16_t huf[1 << ZHUF_MAXBITS];      // symbol | nbBits << 8
    int huf_bits;                         // 0: no table yet (Treeless needs one)
    uint8_t *stage;                       // device: an LDS copy of the current compressed block (null: none)
};
// (the tables, ~10 KB, live in LDS on the device)

// One replay record of stage 1.  tag ZS_SEQ: ll literal bytes (the next ones of the literal
// stream), then ml bytes copied from `off` bytes back; ZS_START: a ZSTD frame begins (offsets may
// not reach before it); ZS_CHECK: the frame ends with content checksum `off` (XXH64 low 32 bits).
struct ZSeq {
    uint32_t ll, ml, off, tag;
};
constexpr uint32_t ZS_SEQ = 0, ZS_START = 1, ZS_CHECK = 2;

// Stage-1 outputs of one packet frame (caller-sized: at most raw/3 + blocks + 2 * zstd frames
// records, at most raw literal bytes)
struct ZOut {
    ZSeq *seq;
    uint64_t seq_cap, nseq;
    uint8_t *lit;
    uint64_t lit_cap, nlit;
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

// backward (Huffman streams, FSE bitstreams): the stream's last byte holds a 1 marker above the
// padding; bits are read from the top down.  Reading past the start yields zeros and makes
// `pos` negative (the overflow the decoders check).  A 64-bit window of the stream (bytes
// [wb, wb + 8)) is kept in registers and refilled only when a read leaves it.
struct BackBits {
    const uint8_t *p;
    int64_t nbytes;
    int64_t pos; // bits still unread (from bit 0 of p[0] up)
    uint64_t win;
    int64_t wb;  // first byte of the window (-1: none)
    ZHD bool init(const uint8_t *buf, int64_t n) {
        p = buf;
        nbytes = n;
        wb = -1;
        win = 0;
        if (n <= 0) return false;
        const uint8_t last = buf[n - 1];
        if (!last) return false;
        pos = (n - 1) * 8 + highbit(last);
        return true;
    }
    // bits [lo, lo + n) of the stream (n <= 56, lo >= 0)
    ZHD uint64_t bits_at(int64_t lo, int n) {
        const int64_t b0 = lo >> 3, b1 = (lo + n - 1) >> 3;
        if (wb < 0 || b0 < wb || b1 >= wb + 8) { // refill: the window ends at the read's last byte
            int64_t nb = b1 - 7;
            if (nb < 0) nb = 0;
            win = 0;
            for (int k = 0; k < 8; ++k)
                if (nb + k < nbytes) win |= (uint64_t)p[nb + k] << (8 * k);
            wb = nb;
        }
        return (win >> (lo - wb * 8)) & ((1ull << n) - 1);
    }
    ZHD uint64_t peek(int n) { // n <= 56; bits below the stream's start read as zeros
        if (n == 0) return 0;
        const int64_t lo = pos - n;
        if (lo >= 0) return bits_at(lo, n);
        if (pos <= 0) return 0;
        return bits_at(0, (int)pos) << (-lo);
    }
    ZHD uint64_t read(int n) {
        const uint64_t v = peek(n);
        pos -= n;
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
template <typename E> ZHD bool fse_build(E *t, const int16_t *norm, int nsym, int log) {
    const int size = 1 << log;
    int high = size - 1;
    uint16_t next[256];
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
// Huffman tree description -> w->huf; returns bytes used or -1
ZHD int64_t huf_read(const uint8_t *src, int64_t n, ZWork *w) {
    if (n < 1) return -1;
    uint8_t weight[256];
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
        int16_t norm[16];
        int log, nsym;
        const int64_t hd = fse_read_ncount(src + 1, hb, 6, 15, norm, log, nsym);
        if (hd < 0 || hd >= hb) return -1;
        FseEntry t[64];
        if (!fse_build(t, norm, nsym, log)) return -1;
        BackBits bb;
        if (!bb.init(src + 1 + hd, hb - hd)) return -1;
        uint32_t s1 = (uint32_t)bb.read(log), s2 = (uint32_t)bb.read(log);
        for (;;) {
            if (nw > 253) return -1;
            weight[nw++] = t[s1].sym;
            s1 = t[s1].base + (uint32_t)bb.read(t[s1].bits);
            if (bb.pos < 0) {
                weight[nw++] = t[s2].sym;
                break;
            }
            weight[nw++] = t[s2].sym;
            s2 = t[s2].base + (uint32_t)bb.read(t[s2].bits);
            if (bb.pos < 0) {
                weight[nw++] = t[s1].sym;
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
    // table: weight w -> nbBits = maxbits + 1 - w, 2^(w-1) entries, symbols in order (HUF_readDTableX1)
    uint32_t start[ZHUF_MAXBITS + 2] = {};
    uint32_t cnt[ZHUF_MAXBITS + 2] = {};
    for (int i = 0; i < nw; ++i) cnt[weight[i]]++;
    uint32_t acc = 0;
    for (int k = 1; k <= maxbits; ++k) {
        start[k] = acc;
        acc += cnt[k] << (k - 1);
    }
    if (acc != (1u << maxbits)) return -1;
    for (int i = 0; i < nw; ++i) {
        const int wt = weight[i];
        if (!wt) continue;
        const uint32_t len = 1u << (wt - 1);
        const uint16_t e = (uint16_t)(i | ((maxbits + 1 - wt) << 8));
        for (uint32_t k = 0; k < len; ++k) w->huf[start[wt] + k] = e;
        start[wt] += len;
    }
    w->huf_bits = maxbits;
    return used;
}

// one Huffman stream of `count` literals into out
ZHD bool huf_stream(const ZWork *w, const uint8_t *src, int64_t n, uint8_t *out, int64_t count) {
    BackBits bb;
    if (!bb.init(src, n)) return false;
    const int mb = w->huf_bits;
    for (int64_t i = 0; i < count; ++i) {
        const uint16_t e = w->huf[bb.peek(mb)];
        out[i] = (uint8_t)e;
        bb.pos -= e >> 8;
        if (bb.pos < 0) return false;
    }
    return bb.pos == 0;
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

// symbol -> baseline and additional bits for every entry of a sequence table of `size` entries
// (kind 0 literal lengths, 1 offsets, 2 match lengths); false on a symbol past the kind's range
ZHD bool seq_finish(ZSeqEntry *t, int size, int kind) {
    const int max_sym = kind == 0 ? 35 : kind == 1 ? 31 : 52;
    for (int u = 0; u < size; ++u) {
        const int c = t[u].sym;
        if (c > max_sym) return false;
        t[u].value = kind == 0 ? ll_base(c) : kind == 1 ? (1u << c) : ml_base(c);
        t[u].add = (uint8_t)(kind == 0 ? ll_bits(c) : kind == 1 ? c : ml_bits(c));
    }
    return true;
}

// ---------------------------------------------------------------- stage 1: blocks -> records
// a sequence-table description of one kind (mode from the compression-modes byte)
ZHD int64_t seq_table(const uint8_t *src, int64_t n, int mode, int kind, ZWork *w) {
    ZSeqEntry *t = kind == 0 ? w->ll : kind == 1 ? w->of : w->ml;
    int &log = kind == 0 ? w->ll_log : kind == 1 ? w->of_log : w->ml_log;
    bool &ok = kind == 0 ? w->ll_ok : kind == 1 ? w->of_ok : w->ml_ok;
    const int max_sym = kind == 0 ? 35 : kind == 1 ? 31 : 52, max_log = kind == 1 ? 8 : 9;
    if (mode == 0) { // predefined
        int16_t norm[53];
        const int nsym = kind == 0 ? 36 : kind == 1 ? 29 : 53;
        for (int s = 0; s < nsym; ++s) norm[s] = kind == 0 ? ll_default(s) : kind == 1 ? of_default(s) : ml_default(s);
        log = kind == 1 ? 5 : 6;
        ok = fse_build(t, norm, nsym, log) && seq_finish(t, 1 << log, kind);
        return ok ? 0 : -1;
    }
    if (mode == 1) { // RLE
        if (n < 1 || src[0] > max_sym) return -1;
        fse_rle(t, src[0]);
        log = 0;
        ok = seq_finish(t, 1, kind);
        return ok ? 1 : -1;
    }
    if (mode == 2) {
        int16_t norm[53];
        int nsym;
        const int64_t used = fse_read_ncount(src, n, max_log, max_sym, norm, log, nsym);
        if (used < 0) return -1;
        ok = fse_build(t, norm, nsym, log) && seq_finish(t, 1 << log, kind);
        return ok ? used : -1;
    }
    return ok ? 0 : -1; // repeat: the previous block's table
}

// appends record r (stored by lane nseq % nl; every lane counts)
ZHD bool put_seq(ZOut &o, const ZSeq &r, uint32_t lane, uint32_t nl) {
    if (o.nseq >= o.seq_cap) return false;
    if (o.nseq % nl == lane) o.seq[o.nseq] = r;
    ++o.nseq;
    return true;
}

// One compressed block: its literals appended to o.lit, its sequences (repeat offsets resolved)
// appended as records.  op = the packet frame's output so far, fstart = where the current ZSTD
// frame's output began (offsets reach back into this frame only), cap = the output capacity.
ZHD bool zblock_entropy(const uint8_t *src, int64_t n, uint64_t &op, uint64_t fstart, uint64_t cap, uint32_t (&rep)[3],
                        ZWork *w, ZOut &o, uint32_t lane, uint32_t nl) {
    // ---- literals section
    if (n < 1) return false;
    const int ltype = src[0] & 3, sf = (src[0] >> 2) & 3;
    int64_t ip = 0;
    uint32_t lsize = 0, csize = 0;
    int streams = 1;
    if (ltype <= 1) {
        if ((sf & 1) == 0) {
            lsize = src[0] >> 3;
            ip = 1;
        } else if (sf == 1) {
            if (n < 2) return false;
            lsize = (src[0] >> 4) | ((uint32_t)src[1] << 4);
            ip = 2;
        } else {
            if (n < 3) return false;
            lsize = (src[0] >> 4) | ((uint32_t)src[1] << 4) | ((uint32_t)src[2] << 12);
            ip = 3;
        }
        if (lsize > (uint32_t)ZMAX_BLOCK || o.nlit + lsize > o.lit_cap) return false;
        uint8_t *lit = o.lit + o.nlit;
        if (ltype == 0) {
            if (ip + lsize > n) return false;
            for (uint32_t i = lane; i < lsize; i += nl) lit[i] = src[ip + i];
            ip += lsize;
        } else {
            if (ip + 1 > n) return false;
            for (uint32_t i = lane; i < lsize; i += nl) lit[i] = src[ip];
            ip += 1;
        }
    } else {
        const int hl = sf <= 1 ? 3 : sf == 2 ? 4 : 5;
        if (n < hl) return false;
        uint64_t v = 0;
        for (int k = 0; k < hl; ++k) v |= (uint64_t)src[k] << (8 * k);
        const int bits = sf <= 1 ? 10 : sf == 2 ? 14 : 18;
        lsize = (uint32_t)((v >> 4) & ((1u << bits) - 1));
        csize = (uint32_t)((v >> (4 + bits)) & ((1u << bits) - 1));
        streams = sf == 0 ? 1 : 4;
        ip = hl;
        if (lsize > (uint32_t)ZMAX_BLOCK || ip + csize > n || o.nlit + lsize > o.lit_cap) return false;
        const uint8_t *cs = src + ip;
        int64_t cn = csize;
        if (ltype == 2) {
            const int64_t hu = huf_read(cs, cn, w);
            if (hu < 0) return false;
            cs += hu;
            cn -= hu;
        } else if (!w->huf_bits) {
            return false; // treeless without a previous table
        }
        uint8_t *lit = o.lit + o.nlit;
        bool bad = false;
        if (streams == 1) {
            if (lane == 0) bad = !huf_stream(w, cs, cn, lit, lsize);
        } else {
            if (cn < 6) return false;
            const int64_t s1 = cs[0] | (cs[1] << 8), s2 = cs[2] | (cs[3] << 8), s3 = cs[4] | (cs[5] << 8);
            const int64_t s4 = cn - 6 - s1 - s2 - s3;
            if (s4 < 1) return false;
            const int64_t seg = (lsize + 3) / 4;
            if (3 * seg > lsize) return false;
            const uint8_t *b = cs + 6;
            // stream k by lane k (every stream by lane 0 when the caller runs one lane)
            for (uint32_t k = lane; k < 4; k += nl) {
                const int64_t cnt = k < 3 ? seg : (int64_t)lsize - 3 * seg;
                const int64_t at = k == 0 ? 0 : k == 1 ? s1 : k == 2 ? s1 + s2 : s1 + s2 + s3;
                const int64_t len = k == 0 ? s1 : k == 1 ? s2 : k == 2 ? s3 : s4;
                bad = bad || !huf_stream(w, b + at, len, lit + k * seg, cnt);
            }
        }
        if (ZANY(bad)) return false;
        ip += csize;
    }
    // ---- sequences section
    if (ip >= n) return false;
    uint32_t nseq;
    const int b0 = src[ip];
    if (b0 == 0) {
        nseq = 0;
        ip += 1;
    } else if (b0 < 128) {
        nseq = b0;
        ip += 1;
    } else if (b0 < 255) {
        if (ip + 2 > n) return false;
        nseq = ((uint32_t)(b0 - 128) << 8) + src[ip + 1];
        ip += 2;
    } else {
        if (ip + 3 > n) return false;
        nseq = src[ip + 1] + ((uint32_t)src[ip + 2] << 8) + 0x7F00;
        ip += 3;
    }
    uint32_t lit_pos = 0;
    if (nseq > 0) {
        if (ip >= n) return false;
        const int modes = src[ip++];
        if (modes & 3) return false; // reserved bits
        const int mll = modes >> 6, mof = (modes >> 4) & 3, mml = (modes >> 2) & 3;
        int64_t u;
        if ((u = seq_table(src + ip, n - ip, mll, 0, w)) < 0) return false;
        ip += u;
        if ((u = seq_table(src + ip, n - ip, mof, 1, w)) < 0) return false;
        ip += u;
        if ((u = seq_table(src + ip, n - ip, mml, 2, w)) < 0) return false;
        ip += u;
        BackBits bb;
        if (!bb.init(src + ip, n - ip)) return false;
        uint32_t sll = (uint32_t)bb.read(w->ll_log), sof = (uint32_t)bb.read(w->of_log), sml = (uint32_t)bb.read(w->ml_log);
        uint32_t r0 = rep[0], r1 = rep[1], r2 = rep[2]; // the repeat offsets, in registers
        for (uint32_t q = 0; q < nseq; ++q) {
            // one table read per code (the symbols were checked when the tables were built)
            const ZSeqEntry el = w->ll[sll], eo = w->of[sof], em = w->ml[sml];
            const uint64_t ofv = (uint64_t)eo.value + bb.read(eo.add);
            const uint32_t ml = em.value + (uint32_t)bb.read(em.add);
            const uint32_t ll = el.value + (uint32_t)bb.read(el.add);
            if (q + 1 < nseq) { // state updates: LL, ML, OF
                sll = el.base + (uint32_t)bb.read(el.bits);
                sml = em.base + (uint32_t)bb.read(em.bits);
                sof = eo.base + (uint32_t)bb.read(eo.bits);
            }
            if (bb.pos < 0) return false;
            uint64_t off;
            if (ofv > 3) {
                off = ofv - 3;
                r2 = r1;
                r1 = r0;
                r0 = (uint32_t)off;
            } else {
                const int idx = (int)ofv - 1 + (ll == 0 ? 1 : 0);
                if (idx == 0) {
                    off = r0;
                } else {
                    const uint32_t t = idx == 3 ? r0 - 1 : idx == 1 ? r1 : r2;
                    if (idx != 1) r2 = r1;
                    r1 = r0;
                    r0 = t;
                    off = t;
                }
            }
            if (lit_pos + ll > lsize || op + ll + ml > cap || off == 0 || off > op - fstart + ll) return false;
            if (!put_seq(o, ZSeq{ll, ml, (uint32_t)off, ZS_SEQ}, lane, nl)) return false;
            op += ll + ml;
            lit_pos += ll;
        }
        if (bb.pos != 0) return false;
        rep[0] = r0;
        rep[1] = r1;
        rep[2] = r2;
    } else if (ip != n) {
        return false;
    }
    const uint32_t rest = lsize - lit_pos; // the block's last literals
    if (rest) {
        if (op + rest > cap || !put_seq(o, ZSeq{rest, 0, 0, ZS_SEQ}, lane, nl)) return false;
        op += rest;
    }
    o.nlit += lsize;
    return true;
}

// Stage 1 of one packet frame: every ZSTD frame of src[0, n) (skippable frames decode to
// nothing) into records and literals.  Returns the decoded size, or -1 when the frame is
// malformed, uses a dictionary, or does not fit `cap` / the ZOut capacities.
ZHD int64_t zstd_frame_entropy(const uint8_t *src, int64_t n, uint64_t cap, ZWork *w, ZOut &o, uint32_t lane = 0,
                               uint32_t nl = 1) {
    int64_t ip = 0;
    uint64_t op = 0;
    while (ip < n) {
        if (ip + 4 > n) return -1;
        const uint32_t magic = rd32(src + ip);
        ip += 4;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) { // skippable
            if (ip + 4 > n) return -1;
            const uint32_t sz = rd32(src + ip);
            ip += 4 + (int64_t)sz;
            if (ip > n) return -1;
            continue;
        }
        if (magic != 0xFD2FB528u) return -1;
        if (ip >= n) return -1;
        const int fhd = src[ip++];
        const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did = fhd & 3;
        if (fhd & 8) return -1; // reserved bit
        if (!single) ++ip;      // window descriptor (the output buffer is the whole frame)
        const int did_len = did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4;
        if (ip + did_len > n) return -1;
        uint32_t dict = 0;
        for (int k = 0; k < did_len; ++k) dict |= (uint32_t)src[ip + k] << (8 * k);
        if (dict) return -1;
        ip += did_len;
        const int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        if (ip + fcs_len > n) return -1;
        uint64_t fcs = 0;
        bool has_fcs = fcs_len > 0;
        for (int k = 0; k < fcs_len; ++k) fcs |= (uint64_t)src[ip + k] << (8 * k);
        if (fcs_len == 2) fcs += 256;
        ip += fcs_len;
        const uint64_t fstart = op;
        if (!put_seq(o, ZSeq{0, 0, 0, ZS_START}, lane, nl)) return -1;
        uint32_t rep[3] = {1, 4, 8};
        w->ll_ok = w->of_ok = w->ml_ok = false;
        w->huf_bits = 0;
        for (;;) {
            if (ip + 3 > n) return -1;
            const uint32_t bh = (uint32_t)src[ip] | (uint32_t)src[ip + 1] << 8 | (uint32_t)src[ip + 2] << 16;
            ip += 3;
            const int last = bh & 1, btype = (bh >> 1) & 3;
            const uint32_t bsize = bh >> 3;
            if (btype == 3) return -1;
            if (btype == 1) { // RLE: one literal byte, then an offset-1 match of bsize - 1
                if (ip + 1 > n || op + bsize > cap) return -1;
                if (bsize) {
                    if (o.nlit + 1 > o.lit_cap) return -1;
                    if (lane == 0) o.lit[o.nlit] = src[ip];
                    o.nlit += 1;
                    if (!put_seq(o, ZSeq{1, bsize - 1, bsize > 1 ? 1u : 0u, ZS_SEQ}, lane, nl)) return -1;
                    op += bsize;
                }
                ip += 1;
            } else {
                if (ip + bsize > n) return -1;
                if (btype == 0) { // raw: a literal run
                    if (op + bsize > cap || o.nlit + bsize > o.lit_cap) return -1;
                    for (uint32_t i = lane; i < bsize; i += nl) o.lit[o.nlit + i] = src[ip + i];
                    o.nlit += bsize;
                    if (bsize && !put_seq(o, ZSeq{bsize, 0, 0, ZS_SEQ}, lane, nl)) return -1;
                    op += bsize;
                } else {
                    if (bsize > (uint32_t)ZMAX_BLOCK) return -1;
                    const uint8_t *bsrc = src + ip;
                    if (w->stage) { // the block's bytes into LDS: every bit read then costs an LDS load
                        ZSYNC_LDS();
                        for (uint32_t i0 = lane * 16; i0 < bsize; i0 += nl * 16) { // 16 loads in flight a lane
                            uint8_t v[16];
#pragma unroll
                            for (int k = 0; k < 16; ++k) v[k] = i0 + k < bsize ? bsrc[i0 + k] : 0;
#pragma unroll
                            for (int k = 0; k < 16; ++k)
                                if (i0 + k < bsize) w->stage[i0 + k] = v[k];
                        }
                        ZSYNC_LDS();
                        bsrc = w->stage;
                    }
                    if (!zblock_entropy(bsrc, bsize, op, fstart, cap, rep, w, o, lane, nl)) return -1;
                }
                ip += bsize;
            }
            if (last) break;
        }
        if (has_fcs && op - fstart != fcs) return -1;
        if (checksum) {
            if (ip + 4 > n) return -1;
            if (!put_seq(o, ZSeq{0, 0, rd32(src + ip), ZS_CHECK}, lane, nl)) return -1;
            ip += 4;
        }
    }
    return (int64_t)op;
}

// record capacity of a packet frame of `raw` output bytes and `comp` compressed bytes: sequences
// have a match of >= 3 bytes; every block adds at most one literal-run record and every ZSTD frame
// (>= 8 bytes: magic, descriptor, one block header) two markers
ZHD uint64_t zstd_seq_cap(uint64_t raw, uint64_t comp) { return raw / 3 + comp * 2 / 3 + 16; }

// ---------------------------------------------------------------- stage 2 (host form)
// Replays the records of one packet frame into dst[0, cap); -1 on any inconsistency (a record
// past the literals or the output, an offset before its frame, a checksum mismatch).
ZHD int64_t zstd_exec_serial(const ZSeq *seq, uint64_t nseq, const uint8_t *lit, uint64_t nlit, uint8_t *dst,
                             uint64_t cap) {
    uint64_t op = 0, lp = 0, fstart = 0;
    for (uint64_t q = 0; q < nseq; ++q) {
        const ZSeq r = seq[q];
        if (r.tag == ZS_START) {
            fstart = op;
            continue;
        }
        if (r.tag == ZS_CHECK) {
            if ((uint32_t)xxh64(dst + fstart, op - fstart) != r.off) return -1;
            continue;
        }
        if (r.tag != ZS_SEQ || lp + r.ll > nlit || op + r.ll + r.ml > cap) return -1;
        for (uint32_t i = 0; i < r.ll; ++i) dst[op + i] = lit[lp + i];
        op += r.ll;
        lp += r.ll;
        if (r.ml) {
            if (r.off == 0 || r.off > op - fstart) return -1;
            for (uint32_t i = 0; i < r.ml; ++i) dst[op + i] = dst[op - r.off + i];
            op += r.ml;
        }
    }
    return lp == nlit ? (int64_t)op : -1;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Host decode of one frame body (both stages): the decoded size, or -1 (tests/cpp/zstd_cpu.cpp).
inline int64_t zstd_frame(const uint8_t *src, int64_t n, uint8_t *dst, uint64_t cap, ZWork *w) {
    ZOut o{};
    o.seq_cap = zstd_seq_cap(cap, (uint64_t)n);
    o.lit_cap = cap;
    o.seq = new ZSeq[o.seq_cap];
    o.lit = new uint8_t[o.lit_cap + 1];
    int64_t r = zstd_frame_entropy(src, n, cap, w, o);
    if (r >= 0 && zstd_exec_serial(o.seq, o.nseq, o.lit, o.nlit, dst, cap) != r) r = -1;
    delete[] o.seq;
    delete[] o.lit;
    return r;
}
#endif

} // namespace tfz
