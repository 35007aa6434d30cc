// zstd_enc.hip — the ZSTD sender of an MPP packet (§8 f1, HIGH_COMPRESSION mode: the packet
// codec CHBlockChunkCodecV1::encode(..., CompressionMethod::ZSTD) -> CompressionCodecZSTD,
// reference dbms/src/IO/Compression/CompressionCodecZSTD.cpp:39 ZSTD_compress), one 64 KB frame
// per wave, independent frames (the packet format frames the body in CompressedWriteBuffer units,
// each its own ZSTD frame, so any frame size decodes).
//
// A frame (RFC 8878): magic, a single-segment header with a 4-byte content size, one block.  The
// block is compressed when that is smaller, raw otherwise:
//   matcher   LZ77 over the frame, 64 positions per step (one a lane: 4-byte hash, LDS table
//             slot read, candidates taken in order), matches extended 64 bytes per step by a
//             ballot; literal
//             bytes and sequences {ll, ml, offset value} to a per-frame work area; offsets are
//             coded against the three repeat offsets as RFC 8878 §3.1.1.5 keeps them (repeat
//             codes 1-3, after literals or without them)
//   literals  Huffman (histogram by LDS atomics, leaves ranked by the wave, minimum-redundancy
//             lengths limited to 11 bits on one lane, canonical codes as HUF_buildCTable assigns
//             them, weights FSE-compressed or in the direct 4-bit form; 4 streams, each written
//             64 symbols per step at prefix-sum bit offsets), RLE for one byte value, raw when
//             that is smaller
//   sequences per code kind (LL / OF / ML): counted by LDS atomics, then RLE when one code is
//             used, a table description of the counts (normalized, FSE_optimalTableLog's
//             accuracy) when that costs fewer bits than the predefined distribution, predefined
//             otherwise; FSE-encoded last sequence first, as ZSTD_encodeSequences does: the three
//             states are uniform across the wave (one sequence at a time, 64 sequences per list
//             load), the bitstream written forward 4 bytes at a time
// zstd_dec.h's tables (bases, extra bits, predefined distributions) are shared with the decoder;
// the output is checked by the system libzstd and by the device decoder (tests/test_zstd.py).
#include "common.h"
#include "codec_zstd.h"
#include "zstd_dec.h"

namespace tfg {
namespace {

using namespace tfz;

// match finder: 2^10 table entries and matches of >= 5 bytes; measured on 4 MB payloads and
// 256 MB of k%08d rows (tools/zenc_probe.py): 11/5 ratio 2.405 at 7.45 GB/s, 11/4 2.227 at 7.35,
// 12/4 2.145 at 5.14, 12/5 2.394 at 5.29, 13/5 2.384 at 2.89, 12/6 2.323 at 4.96 (libzstd -1:
// 2.501); shorter matches cost more sequence bits than the literals they replace.  10 bits
// (8.7 KB of LDS a wave: every frame of a 256 MB packet resident at once) 2.391 at 9.54 GB/s.
#ifndef TFG_ZE_HASH
#define TFG_ZE_HASH 10
#endif
#ifndef TFG_ZE_MINMATCH
#define TFG_ZE_MINMATCH 5
#endif
constexpr int ZE_HASH = TFG_ZE_HASH;         // match-finder table bits
constexpr uint32_t ZE_MINMATCH = TFG_ZE_MINMATCH; // shorter matches stay literals

// FSE compression table (FSE_buildCTable's stateTable / symbolTT), accuracy log <= 8
struct ZEncFse {
    uint16_t state[256];
    int32_t dnb[53]; // deltaNbBits
    int32_t dfs[53]; // deltaFindState
};
struct ZEncTables { // the predefined LL / OF / ML distributions (kind 0 / 1 / 2)
    ZEncFse t[3];
};
constexpr int ZE_DEF_LOG[3] = {6, 5, 6};  // predefined accuracy logs
constexpr int ZE_MAX_LOG[3] = {8, 8, 8};  // largest accuracy logs written (the format allows 9 / 8 / 9)
constexpr int ZE_NSYM[3] = {36, 32, 53};  // code alphabet sizes
constexpr uint32_t ZE_CUSTOM_MIN = 32;    // fewer sequences: no table descriptions

ZHD int16_t zdef_norm(int kind, int s) {
    return kind == 0 ? (s < 36 ? ll_default(s) : 0) : kind == 1 ? (s < 29 ? of_default(s) : 0) : ml_default(s);
}

// The table of a distribution norm[0, nsym) (> 0 or -1 entries; sum 2^log).  The spread is the
// decoder's (fse_build): -1 symbols at the top, the rest stepped through the table.  sym_at: 256
// bytes, cumul: 54 words of work space.
ZHD void zenc_build(ZEncFse &t, const int16_t *norm, int nsym, int log, uint8_t *sym_at, uint32_t *cumul) {
    const int size = 1 << log, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    int high = size - 1;
    cumul[0] = 0;
    for (int s = 0; s < nsym; ++s) {
        if (norm[s] == -1) {
            cumul[s + 1] = cumul[s] + 1;
            sym_at[high--] = (uint8_t)s;
        } else {
            cumul[s + 1] = cumul[s] + norm[s];
        }
    }
    int pos = 0;
    for (int s = 0; s < nsym; ++s)
        for (int i = 0; i < norm[s]; ++i) {
            sym_at[pos] = (uint8_t)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    for (int u = 0; u < size; ++u) t.state[cumul[sym_at[u]]++] = (uint16_t)(size + u);
    int total = 0;
    for (int s = 0; s < 53; ++s) {
        const int n = s < nsym ? norm[s] : 0;
        if (n == 0) {
            t.dnb[s] = ((log + 1) << 16) - size;
            t.dfs[s] = 0;
        } else if (n == -1 || n == 1) {
            t.dnb[s] = (log << 16) - size;
            t.dfs[s] = total - 1;
            ++total;
        } else {
            const int out = log - highbit((uint32_t)(n - 1));
            t.dnb[s] = (out << 16) - (n << out);
            t.dfs[s] = total - n;
            total += n;
        }
    }
}

__global__ void zenc_tables_kernel(ZEncTables *t) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        int16_t norm[53];
        uint8_t sym_at[256];
        uint32_t cumul[54];
        for (int k = 0; k < 3; ++k) {
            for (int s = 0; s < 53; ++s) norm[s] = zdef_norm(k, s);
            zenc_build(t->t[k], norm, k == 0 ? 36 : k == 1 ? 29 : 53, ZE_DEF_LOG[k], sym_at, cumul);
        }
    }
}

__device__ __forceinline__ int zhb(uint32_t v) { return 31 - __builtin_clz(v); }
__device__ __forceinline__ uint32_t ufl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// literal length -> code (RFC 8878 §3.1.1.3.2.1.1, LL_Code)
__device__ __forceinline__ uint32_t zll_code(uint32_t ll) {
    if (ll < 16) return ll;
    if (ll >= 64) return (uint32_t)zhb(ll) + 19;
    if (ll < 24) return 16 + ((ll - 16) >> 1);
    if (ll < 32) return 20 + ((ll - 24) >> 2);
    if (ll < 48) return 22 + ((ll - 32) >> 3);
    return 24;
}
// match length (>= 3) -> code (ML_Code)
__device__ __forceinline__ uint32_t zml_code(uint32_t ml) {
    const uint32_t m = ml - 3;
    if (m < 32) return m;
    if (m >= 128) return (uint32_t)zhb(m) + 36;
    if (m < 40) return 32 + ((m - 32) >> 1);
    if (m < 48) return 36 + ((m - 40) >> 2);
    if (m < 64) return 38 + ((m - 48) >> 3);
    if (m < 96) return 40 + ((m - 64) >> 4);
    return 42;
}

__device__ __forceinline__ uint32_t wave_incl(uint32_t x) { // inclusive prefix sum over the wave
    const uint32_t lane = __lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    return x;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x = max(x, (uint32_t)__shfl_xor(x, d, 64));
    return x;
}

// LDS of the literal coder
struct ZHufLds {
    uint32_t hist[256];
    uint32_t code[256]; // val | nbBits << 16
    int32_t len[256];   // leaves in ascending (count, symbol) order: counts, then code lengths
    uint32_t ring[128]; // bitstream staging words
    uint8_t sym[256];
    uint32_t maxbits;
};

__device__ __forceinline__ uint32_t raw_literals(const uint8_t *lt, uint32_t nlit, uint8_t *dst) {
    const uint32_t lane = __lane_id();
    if (lane == 0) { // raw, 3-byte header (20-bit size)
        dst[0] = (uint8_t)(0x0C | ((nlit & 0xF) << 4));
        dst[1] = (uint8_t)(nlit >> 4);
        dst[2] = (uint8_t)(nlit >> 12);
    }
    for (uint32_t i = lane; i < nlit; i += 64) dst[3 + i] = lt[i];
    return 3 + nlit;
}

// Code lengths of the n >= 2 leaves H.len[0, n) (counts, ascending) in place, limited to ZHUF_MAXBITS
// (lane 0).  Minimum-redundancy lengths by the in-place method of Moffat & Katajainen, then the
// lengths over the limit clamped and the Kraft sum brought back to exactly 1: least frequent codes
// lengthened while it is over, the most frequent of the longest codes shortened while it is under
// (the ZSTD Huffman tree must be complete: the last weight is implied).
__device__ void huf_lengths(int32_t *A, int n) {
    int s = 0, r = 0;
    for (int t = 0; t < n - 1; ++t) {
        if (s >= n || (r < t && A[r] < A[s])) {
            A[t] = A[r];
            A[r++] = t;
        } else {
            A[t] = A[s++];
        }
        if (s >= n || (r < t && A[r] < A[s])) {
            A[t] += A[r];
            A[r++] = t;
        } else {
            A[t] += A[s++];
        }
    }
    A[n - 2] = 0;
    for (int t = n - 3; t >= 0; --t) A[t] = A[A[t]] + 1;
    int a = 1, u = 0, d = 0, t = n - 2, x = n - 1;
    while (a > 0) {
        while (t >= 0 && A[t] == d) {
            ++u;
            --t;
        }
        while (a > u) {
            A[x--] = d;
            --a;
        }
        a = 2 * u;
        ++d;
        u = 0;
    }
    constexpr int L = ZHUF_MAXBITS;
    int e = -(1 << L);
    for (int i = 0; i < n; ++i) {
        if (A[i] > L) A[i] = L;
        e += 1 << (L - A[i]);
    }
    while (e > 0)
        for (int l = L - 1; l >= 1 && e > 0; --l)
            for (int i = 0; i < n && e > 0; ++i)
                if (A[i] == l) {
                    ++A[i];
                    e -= 1 << (L - l - 1);
                }
    while (e < 0)
        for (int l = L; l >= 2 && e < 0; --l)
            for (int i = n - 1; i >= 0 && e < 0; --i)
                if (A[i] == l && (1 << (L - l)) <= -e) {
                    --A[i];
                    e += 1 << (L - l);
                }
}

// One Huffman stream of lt[a, b) (encoded last byte first, as HUF_compress1X) at dst, all lanes:
// 64 symbols per step, each lane's code placed at its prefix-sum bit offset in an LDS ring of
// words, whole words flushed 64 bytes at a time.  Returns the stream's bytes (end mark included).
__device__ __forceinline__ uint32_t huf_stream(const uint8_t *lt, uint32_t a, uint32_t b, uint8_t *dst, ZHufLds &H) {
    const uint32_t lane = __lane_id();
    for (uint32_t i = lane; i < 128; i += 64) H.ring[i] = 0;
    __syncthreads();
    uint32_t p = 0, flushed = 0; // bits placed; bytes written
    auto flush = [&](uint32_t upto) __attribute__((always_inline)) { // bytes [flushed, upto), upto % 4 == 0 or the end
        for (uint32_t q = flushed + lane; q < upto; q += 64) {
            const uint32_t w = (q >> 2) & 127;
            dst[q] = (uint8_t)(H.ring[w] >> (8 * (q & 3)));
        }
        __syncthreads();
        for (uint32_t q = flushed + lane * 4; q < (upto & ~3u); q += 256) H.ring[(q >> 2) & 127] = 0;
        __syncthreads();
        flushed = upto & ~3u;
    };
    for (uint32_t c = 0; c < b - a; c += 64) {
        const uint32_t idx = c + lane;
        const bool ok = idx < b - a;
        const uint32_t code = ok ? H.code[lt[b - 1 - idx]] : 0u;
        const uint32_t nb = code >> 16, val = code & 0xFFFF;
        const uint32_t incl = wave_incl(nb);
        const uint32_t bit = p + incl - nb;
        if (nb) {
            const uint32_t w = bit >> 5, sh = bit & 31;
            atomicOr(&H.ring[w & 127], val << sh);
            if (sh + nb > 32) atomicOr(&H.ring[(w + 1) & 127], val >> (32 - sh));
        }
        p += (uint32_t)__shfl(incl, 63, 64);
        __syncthreads();
        if ((p >> 3) - flushed >= 64) flush((p >> 5) << 2);
    }
    if (lane == 0) atomicOr(&H.ring[(p >> 5) & 127], 1u << (p & 31)); // end mark
    ++p;
    __syncthreads();
    const uint32_t bytes = (p + 7) >> 3;
    flush(bytes);
    return bytes;
}

// LDS of the sequence coder
struct ZSeqLds {
    ZEncFse t[3];           // LL / OF / ML tables in force
    uint32_t hist[3][64];   // code counts
    int16_t norm[3][64];    // a custom distribution
    uint8_t desc[3][128];   // its description (mode 2) or the RLE code (mode 1)
    uint32_t desc_n[3], log[3], mode[3];
    uint8_t sym_at[256];
    uint32_t cumul[64];
};

__device__ __forceinline__ uint32_t lg256(uint32_t x) { // log2(x) * 256, linear between powers of two
    const int hb = zhb(x);
    return ((uint32_t)hb << 8) + ((uint32_t)(((uint64_t)x << 8) >> hb) - 256);
}

// counts (sum total, >= 2 symbols present, largest present symbol maxs) -> a distribution of sum
// 2^L: every present symbol at least 1, the rounding error taken from / given to the largest
__device__ void zenc_normalize(const uint32_t *cnt, int maxs, uint32_t total, int L, int16_t *norm) {
    int sum = 0, largest = 0;
    uint32_t lc = 0;
    for (int c = 0; c <= maxs; ++c) {
        if (!cnt[c]) {
            norm[c] = 0;
            continue;
        }
        int v = (int)((((uint64_t)cnt[c] << L) + total / 2) / total);
        if (v < 1) v = 1;
        norm[c] = (int16_t)v;
        sum += v;
        if (cnt[c] > lc) {
            lc = cnt[c];
            largest = c;
        }
    }
    int diff = (1 << L) - sum;
    if (diff >= 0) {
        norm[largest] = (int16_t)(norm[largest] + diff);
        return;
    }
    while (diff < 0) { // over: take from the most probable symbols
        int m = 0;
        for (int c = 1; c <= maxs; ++c)
            if (norm[c] > norm[m]) m = c;
        norm[m] = (int16_t)(norm[m] - 1);
        ++diff;
    }
}

// FSE table description (RFC 8878 §4.1.1, FSE_writeNCount) of norm[0, maxs] at accuracy log L
// -> out; returns its bytes
__device__ uint32_t zenc_write_ncount(uint8_t *out, const int16_t *norm, int maxs, int L) {
    uint32_t bs = (uint32_t)(L - 5), o = 0;
    int bc = 4, remaining = (1 << L) + 1, threshold = 1 << L, nb = L + 1, sym = 0;
    bool prev0 = false;
    auto flush16 = [&]() {
        out[o++] = (uint8_t)bs;
        out[o++] = (uint8_t)(bs >> 8);
        bs >>= 16;
    };
    while (sym <= maxs && remaining > 1) {
        if (prev0) {
            int start = sym;
            while (!norm[sym]) ++sym; // norm[maxs] > 0
            while (sym >= start + 24) {
                start += 24;
                bs |= 0xFFFFu << bc;
                flush16();
            }
            while (sym >= start + 3) {
                start += 3;
                bs |= 3u << bc;
                bc += 2;
            }
            bs |= (uint32_t)(sym - start) << bc;
            bc += 2;
            if (bc > 16) {
                flush16();
                bc -= 16;
            }
        }
        int count = norm[sym++];
        const int max = (2 * threshold - 1) - remaining;
        remaining -= count < 0 ? -count : count;
        ++count;
        if (count >= threshold) count += max;
        bs |= (uint32_t)count << bc;
        bc += nb;
        bc -= count < max;
        prev0 = count == 1;
        while (remaining < threshold) {
            --nb;
            threshold >>= 1;
        }
        if (bc > 16) {
            flush16();
            bc -= 16;
        }
    }
    out[o] = (uint8_t)bs;
    out[o + 1] = (uint8_t)(bs >> 8);
    return o + (uint32_t)(bc + 7) / 8;
}

// The Huffman weights of symbols [0, nw) (codes in H.code, longest mb) FSE-compressed as
// HUF_compressWeights does (lane 0): a description of the weight counts (accuracy log <= 6) and
// a two-state FSE bitstream (even weights through state 1, odd through state 2, the last two
// seeding the states).  Writes header byte + description + bitstream at dst and returns their
// bytes, or 0 when the direct form is as small (or the weights do not compress).  Work space:
// H.len / H.hist (free by now), S's first table.
__device__ uint32_t huf_weights_fse(uint8_t *dst, ZHufLds &H, ZSeqLds &S, uint32_t nw, uint32_t mb) {
    int32_t *w = H.len;
    uint32_t *wh = H.hist;
    for (int c = 0; c < 16; ++c) wh[c] = 0;
    for (uint32_t i = 0; i < nw; ++i) {
        const uint32_t nb = H.code[i] >> 16;
        w[i] = nb ? (int32_t)(mb + 1 - nb) : 0;
        ++wh[w[i]];
    }
    int maxw = 0, distinct = 0;
    for (int c = 0; c <= ZHUF_MAXBITS + 1; ++c)
        if (wh[c]) {
            maxw = c;
            ++distinct;
        }
    if (distinct < 2 || nw < 3) return 0;
    int L = 6;
    const int max_src = zhb(nw - 1) - 2, min_bits = min(zhb(nw) + 1, zhb((uint32_t)maxw) + 2);
    if (max_src < L) L = max_src;
    if (min_bits > L) L = min_bits;
    L = max(5, min(L, 6));
    zenc_normalize(wh, maxw, nw, L, S.norm[0]);
    const uint32_t nc = zenc_write_ncount(dst + 1, S.norm[0], maxw, L);
    ZEncFse &t = S.t[0];
    zenc_build(t, S.norm[0], maxw + 1, L, S.sym_at, S.cumul);
    uint8_t *bs = dst + 1 + nc;
    uint64_t bc = 0;
    int bn = 0;
    uint32_t o = 0;
    auto put = [&](uint32_t v, int n) {
        bc |= (uint64_t)(v & ((1u << n) - 1)) << bn;
        bn += n;
        while (bn >= 8) {
            bs[o++] = (uint8_t)bc;
            bc >>= 8;
            bn -= 8;
        }
    };
    auto init = [&](int sym) {
        const uint32_t nb = (uint32_t)(t.dnb[sym] + (1 << 15)) >> 16;
        const uint32_t v = (nb << 16) - (uint32_t)t.dnb[sym];
        return (uint32_t)t.state[(v >> nb) + t.dfs[sym]];
    };
    auto enc = [&](uint32_t &st, int sym) {
        const uint32_t nb = (st + (uint32_t)t.dnb[sym]) >> 16;
        put(st, (int)nb);
        st = t.state[(st >> nb) + t.dfs[sym]];
    };
    int i = (int)nw - 1;
    uint32_t s1, s2;
    if (nw & 1) {
        s1 = init(w[i]);
        s2 = init(w[i - 1]);
        enc(s1, w[i - 2]);
        i -= 3;
    } else {
        s2 = init(w[i]);
        s1 = init(w[i - 1]);
        i -= 2;
    }
    for (; i >= 0; --i) enc((i & 1) ? s2 : s1, w[i]);
    put(s2, L);
    put(s1, L);
    put(1, 1); // end mark
    if (bn > 0) bs[o++] = (uint8_t)bc;
    const uint32_t total = nc + o;
    if (total >= 128 || (nw <= 128 && total >= (nw + 1) / 2)) return 0;
    dst[0] = (uint8_t)total;
    return 1 + total;
}

// The literal section of lt[0, nlit) at dst: Huffman-compressed (4 streams from 256 literals, 1
// below; weights FSE-compressed, or in the direct 4-bit form when that is as small) when smaller,
// RLE when one byte value, raw otherwise.  All lanes; returns the section's bytes.  S: work space
// of the weight coder (its counts are left alone).
__device__ uint32_t literal_section(const uint8_t *lt, uint32_t nlit, uint8_t *dst, ZHufLds &H, ZSeqLds &S) {
    const uint32_t lane = __lane_id();
    if (nlit < 64) return raw_literals(lt, nlit, dst);
    for (uint32_t i = lane; i < 256; i += 64) H.hist[i] = 0;
    __syncthreads();
    for (uint32_t i = lane; i < nlit; i += 64) atomicAdd(&H.hist[lt[i]], 1u);
    __syncthreads();
    uint32_t present = 0, maxs = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t sy = lane + 64 * k;
        if (H.hist[sy]) {
            ++present;
            maxs = sy;
        }
    }
    const uint32_t nsym = ufl(wave_sum(present)), maxsym = ufl(wave_max(maxs));
    if (nsym == 1) { // RLE: 3-byte header (20-bit size) + the byte
        if (lane == 0) {
            dst[0] = (uint8_t)(0x0D | ((nlit & 0xF) << 4));
            dst[1] = (uint8_t)(nlit >> 4);
            dst[2] = (uint8_t)(nlit >> 12);
            dst[3] = (uint8_t)maxsym;
        }
        return 4;
    }
    // leaves in ascending (count, symbol) order
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t sy = lane + 64 * k, c = H.hist[sy];
        if (!c) continue;
        uint32_t rank = 0;
        for (uint32_t t = 0; t <= maxsym; ++t) {
            const uint32_t ct = H.hist[t];
            rank += ct && (ct < c || (ct == c && t < sy));
        }
        H.len[rank] = (int32_t)c;
        H.sym[rank] = (uint8_t)sy;
    }
    __syncthreads();
    if (lane == 0) {
        huf_lengths(H.len, (int)nsym);
        uint32_t mb = 0;
        for (uint32_t i = 0; i < nsym; ++i) mb = max(mb, (uint32_t)H.len[i]);
        for (uint32_t sy = 0; sy < 256; ++sy) H.code[sy] = 0;
        for (uint32_t i = 0; i < nsym; ++i) H.code[H.sym[i]] = (uint32_t)H.len[i] << 16;
        // canonical values (HUF_buildCTable): longest codes first from 0, symbol order within a length
        uint32_t per[ZHUF_MAXBITS + 2] = {0}, start[ZHUF_MAXBITS + 2] = {0};
        for (uint32_t i = 0; i < nsym; ++i) ++per[H.len[i]];
        uint32_t m = 0;
        for (uint32_t nb = mb; nb > 0; --nb) {
            start[nb] = m;
            m += per[nb];
            m >>= 1;
        }
        for (uint32_t sy = 0; sy <= maxsym; ++sy) {
            const uint32_t nb = H.code[sy] >> 16;
            if (nb) H.code[sy] |= start[nb]++;
        }
        H.maxbits = mb;
    }
    __syncthreads();
    const uint32_t mb = ufl(H.maxbits);
    // exact payload bits: is it worth it
    uint32_t tb = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t sy = lane + 64 * k;
        tb += H.hist[sy] * (H.code[sy] >> 16);
    }
    tb = ufl(wave_sum(tb));
    const bool four = nlit >= 256;
    const uint32_t hdr = four ? 5 : 3, nw = maxsym;
    __syncthreads(); // every lane has read H.hist
    uint32_t tree = 0;
    if (lane == 0) tree = huf_weights_fse(dst + hdr, H, S, nw, mb);
    tree = ufl(tree);
    const bool direct = tree == 0;
    if (direct) {
        if (nw > 128) return raw_literals(lt, nlit, dst);
        tree = 1 + (nw + 1) / 2;
    }
    const uint32_t est = hdr + tree + (four ? 6 : 0) + tb / 8 + 4;
    if (est >= 3 + nlit) return raw_literals(lt, nlit, dst);
    // direct tree description: header byte 127 + weights, then 4-bit weights (high nibble first)
    if (direct && lane == 0) dst[hdr] = (uint8_t)(127 + nw);
    for (uint32_t j = lane; direct && j < (nw + 1) / 2; j += 64) {
        uint32_t w2[2];
        for (uint32_t h = 0; h < 2; ++h) {
            const uint32_t sy = 2 * j + h, nb = sy < nw ? H.code[sy] >> 16 : 0;
            w2[h] = nb ? mb + 1 - nb : 0;
        }
        dst[hdr + 1 + j] = (uint8_t)((w2[0] << 4) | w2[1]);
    }
    uint32_t at = hdr + tree;
    uint32_t csz;
    if (four) {
        const uint32_t seg = (nlit + 3) / 4;
        uint32_t sz[4];
        at += 6;
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t a = k * seg, b = k == 3 ? nlit : a + seg;
            sz[k] = huf_stream(lt, a, b, dst + at, H);
            at += sz[k];
        }
        if (lane < 3) {
            dst[hdr + tree + 2 * lane] = (uint8_t)sz[lane == 0 ? 0 : lane == 1 ? 1 : 2];
            dst[hdr + tree + 2 * lane + 1] = (uint8_t)(sz[lane == 0 ? 0 : lane == 1 ? 1 : 2] >> 8);
        }
        csz = at - hdr;
        if (lane == 0) { // compressed, 4 streams, 18-bit sizes: 5-byte header
            const uint64_t v = 2u | (3u << 2) | ((uint64_t)nlit << 4) | ((uint64_t)csz << 22);
            for (int q = 0; q < 5; ++q) dst[q] = (uint8_t)(v >> (8 * q));
        }
    } else {
        at += huf_stream(lt, 0, nlit, dst + at, H);
        csz = at - hdr;
        if (lane == 0) { // compressed, 1 stream, 10-bit sizes: 3-byte header
            const uint32_t v = 2u | (nlit << 4) | (csz << 14);
            for (int q = 0; q < 3; ++q) dst[q] = (uint8_t)(v >> (8 * q));
        }
    }
    return at;
}

// LDS of one encode wave: the match finder's tables, then (dead by then) the coders' state
union ZEncLds {
    struct {
        uint16_t tpos[1 << ZE_HASH];
        uint32_t tseq[1 << ZE_HASH];
    } m;
    struct {
        ZHufLds H;
        ZSeqLds S;
    } c;
};

// The table of kind k for the nseq sequences counted in S.hist[k] (lane 0): RLE when one code is
// used, else a description of the counts when it costs fewer bits than the predefined
// distribution (FSE_optimalTableLog's accuracy log), else predefined (copied by the caller).
__device__ void zenc_choose(ZSeqLds &S, int k, uint32_t nseq) {
    const uint32_t *cnt = S.hist[k];
    int maxs = 0, present = 0;
    for (int c = 0; c < ZE_NSYM[k]; ++c)
        if (cnt[c]) {
            maxs = c;
            ++present;
        }
    if (present == 1) {
        S.mode[k] = 1;
        S.log[k] = 0;
        S.desc[k][0] = (uint8_t)maxs;
        S.desc_n[k] = 1;
        S.t[k].state[0] = 0;
        S.t[k].dnb[maxs] = 0;
        S.t[k].dfs[maxs] = 0;
        return;
    }
    S.mode[k] = 0;
    S.log[k] = (uint32_t)ZE_DEF_LOG[k];
    S.desc_n[k] = 0;
    if (nseq < ZE_CUSTOM_MIN) return;
    int L = ZE_MAX_LOG[k];
    const int max_src = zhb(nseq - 1) - 2, min_bits = min(zhb(nseq) + 1, zhb((uint32_t)maxs) + 2);
    if (max_src < L) L = max_src;
    if (min_bits > L) L = min_bits;
    L = max(5, min(L, ZE_MAX_LOG[k]));
    int16_t *norm = S.norm[k];
    zenc_normalize(cnt, maxs, nseq, L, norm);
    const uint32_t dn = zenc_write_ncount(S.desc[k], norm, maxs, L);
    uint64_t cost_def = 0, cost_cus = (uint64_t)dn * 8 * 256;
    for (int c = 0; c <= maxs; ++c) {
        if (!cnt[c]) continue;
        const int16_t d = zdef_norm(k, c);
        cost_def += (uint64_t)cnt[c] * (uint32_t)((ZE_DEF_LOG[k] << 8) - (int)lg256(d > 0 ? (uint32_t)d : 1u));
        cost_cus += (uint64_t)cnt[c] * (uint32_t)((L << 8) - (int)lg256((uint32_t)norm[c]));
    }
    if (cost_cus >= cost_def) return;
    S.mode[k] = 2;
    S.log[k] = (uint32_t)L;
    S.desc_n[k] = dn;
    zenc_build(S.t[k], norm, maxs + 1, L, S.sym_at, S.cumul);
}

#ifdef TFG_ZE_PROF // development: per-phase wall-clock totals over the frames (tools/zenc_probe.py)
__device__ unsigned long long g_zprof[8];
#define ZPROF(i)                                                                                   \
    do {                                                                                           \
        const uint64_t t1_ = wall_clock64();                                                       \
        if (lane == 0) atomicAdd(&g_zprof[i], (unsigned long long)(t1_ - t0_));                    \
        t0_ = t1_;                                                                                 \
    } while (0)
#else
#define ZPROF(i) ((void)0)
#endif

// One wave (= one workgroup) per frame: the packet frame (9-byte header + ZSTD frame) to
// out + f * ZE_SLOT, its size to sizes[f].  tmp: 2 * ZE_FRAME bytes per frame, the literal bytes
// from the front and the sequence list from the back (a sequence covers >= 4 bytes, so
// literals + 8 B per sequence <= 2 * ZE_FRAME).
__global__ void __launch_bounds__(64) zstd_encode_kernel(const uint8_t *src, uint64_t n, uint64_t nframes, uint8_t *out,
                                                         uint32_t *sizes, uint8_t *tmp, const ZEncTables *tabs) {
    __shared__ ZEncLds E;
    const uint64_t f = blockIdx.x;
    if (f >= nframes) return;
    const uint32_t lane = __lane_id();
#ifdef TFG_ZE_PROF
    uint64_t t0_ = wall_clock64();
#endif
    uint16_t *tpos = E.m.tpos;
    uint32_t *tseq = E.m.tseq;
    for (int i = lane; i < (1 << ZE_HASH); i += 64) {
        tpos[i] = 0xFFFF; // empty: never below a cursor position
        tseq[i] = 0;
    }
    __syncthreads();
    const uint8_t *s = src + f * ZE_FRAME;
    const uint32_t len = (uint32_t)min<uint64_t>(ZE_FRAME, n - f * ZE_FRAME);
    uint8_t *frame = out + f * ZE_SLOT;
    uint8_t *content = frame + 21;
    uint8_t *lt = tmp + f * (2ull * ZE_FRAME);
    uint2 *seq_end = (uint2 *)(lt + 2ull * ZE_FRAME); // sequence q at seq_end[-1 - q]

    // ---- matcher
    uint32_t nlit = 0, nseq = 0;
    uint32_t r1 = 1, r2 = 4, r3 = 8; // the repeat offsets (RFC 8878 §3.1.1.5: initial 1, 4, 8)
    auto copy_lits = [&](uint32_t a, uint32_t b) __attribute__((always_inline)) {
        for (uint32_t i = lane; i < b - a; i += 64) lt[nlit + i] = s[a + i];
        nlit += b - a;
    };
    uint32_t anchor = 0;
    if (len >= 8) {
        // 64 positions at a time, one a lane: every lane hashes the 4 bytes at its position and
        // reads its table slot at once; the candidates (4 bytes verified against the slot's
        // copy) are then taken in order, each extended 64 bytes per step by a ballot; the
        // chunk's positions enter the table after it is read (a match's source lies in an
        // earlier chunk, or is the repeat offset)
        const uint32_t last = len - 3; // positions with 4 readable bytes
        uint32_t ip = 0;               // the cursor: next position not yet covered
        uint32_t dry = 0;              // chunks since the last match
        for (uint32_t cbase = 0; cbase < last;) {
            const uint32_t pos = cbase + lane, cbase_ip0 = ip;
            const bool valid = pos < last;
            uint32_t w = 0;
            if (valid) w = (uint32_t)s[pos] | ((uint32_t)s[pos + 1] << 8) | ((uint32_t)s[pos + 2] << 16) | ((uint32_t)s[pos + 3] << 24);
            const uint32_t h = (w * 2654435761u) >> (32 - ZE_HASH);
            // candidates: the table slot, and the first of the three repeat offsets in force at
            // the chunk's start whose 4 bytes match (preferred: a repeat code costs a few bits)
            auto word_at = [&](uint32_t p) __attribute__((always_inline)) {
                return (uint32_t)s[p] | ((uint32_t)s[p + 1] << 8) | ((uint32_t)s[p + 2] << 16) | ((uint32_t)s[p + 3] << 24);
            };
            uint32_t roff = 0;
            if (valid && pos >= ip) {
                if (pos >= r1 && word_at(pos - r1) == w) roff = r1;
                else if (pos >= r2 && word_at(pos - r2) == w) roff = r2;
                else if (pos >= r3 && word_at(pos - r3) == w) roff = r3;
            }
            const uint32_t tref = tpos[h], rw = tseq[h];
            const bool by_rep = roff != 0;
            const bool by_tab = valid && pos >= ip && tref < pos && rw == w && (!by_rep || tref != pos - roff);
            const uint64_t mrep = __ballot(by_rep), mtab = __ballot(by_tab);
            uint64_t mask = mrep | mtab, covered = 0;
            auto extend = [&](uint32_t at, uint32_t from) __attribute__((always_inline)) {
                uint32_t ml = 4;
                for (;;) { // 64 bytes per step
                    const uint32_t x = at + ml + lane;
                    const bool eq = x < len && s[from + ml + lane] == s[x];
                    const uint64_t neq = ~__ballot(eq);
                    if (neq == 0) {
                        ml += 64;
                        continue;
                    }
                    return ml + (uint32_t)__builtin_ctzll(neq);
                }
            };
            while (mask) {
                const uint32_t j = (uint32_t)__builtin_ctzll(mask);
                const uint32_t at = cbase + j;
                // the longer of the two candidates; the repeat offset when within a byte
                const uint32_t rofj = (uint32_t)__builtin_amdgcn_readlane((int)roff, (int)j);
                const uint32_t ml_r = (mrep >> j) & 1 ? extend(at, at - rofj) : 0;
                const uint32_t tfrom = (uint32_t)__builtin_amdgcn_readlane((int)tref, (int)j);
                const uint32_t ml_t = (mtab >> j) & 1 ? extend(at, tfrom) : 0;
                const bool use_rep = ml_r >= ZE_MINMATCH && ml_r + 1 >= ml_t;
                const uint32_t ml = use_rep ? ml_r : ml_t, from = use_rep ? at - rofj : tfrom;
                if (ml < ZE_MINMATCH) {
                    mask &= mask - 1;
                    continue;
                }
                const uint32_t ll = at - anchor, off = at - from;
                copy_lits(anchor, at);
                // the offset value and the repeat-offset history (RFC 8878 §3.1.1.5): with
                // literals before it 1 / 2 / 3 are R1 / R2 / R3, without them R2 / R3 / R1 - 1;
                // any offset other than R1 becomes R1, the others shifting down behind it
                uint32_t ofv;
                if (ll > 0 && off == r1) {
                    ofv = 1;
                } else {
                    if (off == r2) ofv = ll > 0 ? 2 : 1;
                    else if (off == r3) ofv = ll > 0 ? 3 : 2;
                    else if (ll == 0 && off == r1 - 1) ofv = 3;
                    else ofv = off + 3;
                    if (off != r2) r3 = r2;
                    r2 = r1;
                    r1 = off;
                }
                if (lane == 0) seq_end[-1 - (int64_t)nseq] = make_uint2(ll | (ml << 16), ofv);
                ++nseq;
                ip = at + ml;
                anchor = ip;
                const uint64_t after = j == 63 ? 0ull : ~0ull << (j + 1); // lanes past the match start
                if (ip >= cbase + 64) {
                    covered |= after;
                    break;
                }
                covered |= after & ((1ull << (ip - cbase)) - 1);
                mask &= ~0ull << (ip - cbase); // candidates inside the match are covered
            }
            // the chunk's positions enter the table (one of the lanes sharing a slot wins), but
            // not those inside its matches (a slot keeps an older entry rather than a position
            // no search starts from); after chunks without a match only every stride-th, the
            // stride doubling every two dry chunks up to 64, so incompressible stretches do not
            // flush the older entries.  Measured (tools/zenc_probe.py, 4 MB, ratio): all
            // positions: k%08d 2.402, Int64 3.40, text 5.30; without those inside matches 2.392,
            // 3.75, 4.92 — Int64 columns weigh more in packets than prose.
            dry = ip > cbase_ip0 ? 0 : dry + 1;
            const uint32_t stride = 1u << min(6u, dry >> 1);
            if (valid && !((covered >> lane) & 1) && (pos & (stride - 1)) == 0) {
                tpos[h] = (uint16_t)pos;
                tseq[h] = w;
            }
            __builtin_amdgcn_wave_barrier();
            cbase = max(cbase + 64, ip);
        }
    }
    copy_lits(anchor, len);
    __syncthreads(); // the literal / list stores land before they are read back; the match tables are dead
    ZPROF(0);

    // ---- block: compressed when its size bound is below the raw size
    ZHufLds &H = E.c.H;
    ZSeqLds &S = E.c.S;
    uint32_t csize = 0;
    bool comp = false;
    if (3 + nlit / 4 < len) {
        // code counts and the extra bits of the sequences
        for (uint32_t i = lane; i < 3 * 64; i += 64) (&S.hist[0][0])[i] = 0;
        __syncthreads();
        uint32_t ex = 0;
        for (uint32_t q = lane; q < nseq; q += 64) {
            const uint2 v = seq_end[-1 - (int64_t)q];
            const uint32_t ll = v.x & 0xFFFF, ml = v.x >> 16, llc = zll_code(ll), mlc = zml_code(ml), ofc = zhb(v.y);
            atomicAdd(&S.hist[0][llc], 1u);
            atomicAdd(&S.hist[1][ofc], 1u);
            atomicAdd(&S.hist[2][mlc], 1u);
            ex += ll_bits((int)llc) + ml_bits((int)mlc) + ofc;
        }
        ex = ufl(wave_sum(ex));
        __syncthreads();
        ZPROF(1);
        const uint32_t lsz = literal_section(lt, nlit, content, H, S);
        __syncthreads();
        ZPROF(2);
        if (lane == 0)
            for (int k = 0; k < 3; ++k) zenc_choose(S, k, nseq);
        __syncthreads();
        for (int k = 0; k < 3; ++k)
            if (ufl(S.mode[k]) == 0)
                for (uint32_t i = lane; i < sizeof(ZEncFse) / 4; i += 64)
                    ((uint32_t *)&S.t[k])[i] = ((const uint32_t *)&tabs->t[k])[i];
        __syncthreads();
        ZPROF(3);
        const uint32_t nsh = nseq < 128 ? 1 : 2;
        const uint32_t d0 = ufl(S.desc_n[0]), d1 = ufl(S.desc_n[1]), d2 = ufl(S.desc_n[2]);
        const uint32_t lg0 = ufl(S.log[0]), lg1 = ufl(S.log[1]), lg2 = ufl(S.log[2]);
        const uint32_t hdr = nseq ? nsh + 1 + d0 + d1 + d2 : 1;
        const uint64_t bits = ex + (uint64_t)nseq * (lg0 + lg1 + lg2) + 1;
        const uint64_t bound = lsz + hdr + (nseq ? (bits + 7) / 8 : 0);
        if (bound < len && !nseq) { // literals only: the sequence section is its count
            comp = true;
            if (lane == 0) content[lsz] = 0;
            csize = lsz + 1;
        } else if (bound < len) {
            comp = true;
            uint8_t *h = content + lsz;
            if (lane == 0) {
                if (nsh == 1) {
                    h[0] = (uint8_t)nseq;
                } else {
                    h[0] = (uint8_t)((nseq >> 8) + 0x80);
                    h[1] = (uint8_t)nseq;
                }
                h[nsh] = (uint8_t)((S.mode[0] << 6) | (S.mode[1] << 4) | (S.mode[2] << 2));
            }
            uint8_t *dd = h + nsh + 1;
            for (uint32_t i = lane; i < d0 + d1 + d2; i += 64)
                dd[i] = i < d0 ? S.desc[0][i] : i < d0 + d1 ? S.desc[1][i - d0] : S.desc[2][i - d0 - d1];
            uint8_t *bs = h + hdr;
            uint64_t bc = 0;
            uint32_t bn = 0, wp = 0;
            auto add = [&](uint32_t v, uint32_t nb) __attribute__((always_inline)) {
                bc |= ((uint64_t)v & ((1ull << nb) - 1)) << bn; // nb <= 32
                bn += nb;
                if (bn >= 32) {
                    if (lane < 4) bs[wp + lane] = (uint8_t)(bc >> (8 * lane));
                    wp += 4;
                    bc >>= 32;
                    bn -= 32;
                }
            };
            // 64 sequences at a time, one a lane: codes, extra bits (LL, ML, OF packed low to
            // high) and the three codes' table entries, so the serial walk below only chains
            // the states and appends bits
            uint32_t vc = 0, velo = 0, vehi = 0;
            int32_t vdnb0 = 0, vdnb1 = 0, vdnb2 = 0, vdfs0 = 0, vdfs1 = 0, vdfs2 = 0;
            int64_t bbase = -1;
            auto load = [&](uint32_t q) __attribute__((always_inline)) {
                bbase = q & ~63u;
                const uint32_t i = (uint32_t)bbase + lane;
                const uint2 v = i < nseq ? seq_end[-1 - (int64_t)i] : make_uint2(3u << 16, 4);
                const uint32_t ll = v.x & 0xFFFF, ml = v.x >> 16, ofv = v.y;
                const uint32_t llc = zll_code(ll), mlc = zml_code(ml), ofc = (uint32_t)zhb(ofv);
                const uint32_t llb = (uint32_t)ll_bits((int)llc), mlb = (uint32_t)ml_bits((int)mlc);
                const uint64_t e = (uint64_t)(ll - ll_base((int)llc)) | ((uint64_t)(ml - ml_base((int)mlc)) << llb) |
                                   ((uint64_t)(ofv - (1u << ofc)) << (llb + mlb));
                velo = (uint32_t)e;
                vehi = (uint32_t)(e >> 32);
                vc = llc | (mlc << 8) | (ofc << 16) | ((llb + mlb + ofc) << 24);
                vdnb0 = S.t[0].dnb[llc];
                vdfs0 = S.t[0].dfs[llc];
                vdnb1 = S.t[1].dnb[ofc];
                vdfs1 = S.t[1].dfs[ofc];
                vdnb2 = S.t[2].dnb[mlc];
                vdfs2 = S.t[2].dfs[mlc];
            };
            auto rl = [&](int32_t v, int r) __attribute__((always_inline)) { return __builtin_amdgcn_readlane(v, r); };
            auto extras = [&](int r, uint32_t eb) __attribute__((always_inline)) {
                const uint32_t lo = (uint32_t)rl((int32_t)velo, r);
                if (eb <= 32) {
                    add(lo, eb);
                } else {
                    add(lo, 32);
                    add((uint32_t)rl((int32_t)vehi, r), eb - 32);
                }
            };
            auto init = [&](const ZEncFse &t, int32_t dnb, int32_t dfs) __attribute__((always_inline)) {
                const uint32_t nb = (uint32_t)(dnb + (1 << 15)) >> 16;
                const uint32_t v = (nb << 16) - (uint32_t)dnb;
                return ufl(t.state[(v >> nb) + dfs]);
            };
            auto enc = [&](const ZEncFse &t, uint32_t &st, int32_t dnb, int32_t dfs) __attribute__((always_inline)) {
                const uint32_t nb = (st + (uint32_t)dnb) >> 16;
                add(st, nb);
                st = ufl(t.state[(st >> nb) + dfs]);
            };
            load(nseq - 1);
            int r = (int)(nseq - 1 - (uint32_t)bbase);
            uint32_t s_ml = init(S.t[2], rl(vdnb2, r), rl(vdfs2, r));
            uint32_t s_of = init(S.t[1], rl(vdnb1, r), rl(vdfs1, r));
            uint32_t s_ll = init(S.t[0], rl(vdnb0, r), rl(vdfs0, r));
            extras(r, (uint32_t)rl((int32_t)vc, r) >> 24);
            for (int64_t q = (int64_t)nseq - 2; q >= 0; --q) {
                if (q < bbase) load((uint32_t)q);
                r = (int)(q - bbase);
                enc(S.t[1], s_of, rl(vdnb1, r), rl(vdfs1, r));
                enc(S.t[2], s_ml, rl(vdnb2, r), rl(vdfs2, r));
                enc(S.t[0], s_ll, rl(vdnb0, r), rl(vdfs0, r));
                extras(r, (uint32_t)rl((int32_t)vc, r) >> 24);
            }
            add(s_ml, lg2);
            add(s_of, lg1);
            add(s_ll, lg0);
            add(1, 1); // end mark
            const uint32_t tail = (bn + 7) / 8;
            if (lane < tail) bs[wp + lane] = (uint8_t)(bc >> (8 * lane));
            wp += tail;
            csize = lsz + hdr + wp;
            ZPROF(4);
        }
    }
    __syncthreads();
    if (!comp) {
        for (uint32_t i = lane; i < len; i += 64) content[i] = s[i];
        csize = len;
    }
    // ---- headers: block (last; compressed or raw), packet frame {0x90, frame bytes, raw bytes},
    // ZSTD magic, FHD 0xA0 (single segment, 4-byte content size), content size
    const uint32_t bh = 1u | ((comp ? 2u : 0u) << 1) | (csize << 3);
    const uint32_t fbytes = 21 + csize;
    if (lane < 4) {
        frame[1 + lane] = (uint8_t)(fbytes >> (8 * lane));
        frame[5 + lane] = (uint8_t)(len >> (8 * lane));
        frame[9 + lane] = (uint8_t)(0xFD2FB528u >> (8 * lane));
        frame[14 + lane] = (uint8_t)(len >> (8 * lane));
    }
    if (lane < 3) frame[18 + lane] = (uint8_t)(bh >> (8 * lane));
    if (lane == 0) {
        frame[0] = 0x90;
        frame[13] = 0xA0;
        sizes[f] = fbytes;
    }
    ZPROF(5);
}

} // namespace

size_t zstd_encode_tmp_bytes(uint64_t nframes) {
    return (size_t)nframes * 2 * ZE_FRAME + ((sizeof(ZEncTables) + 255) & ~size_t(255));
}

int zstd_encode_frames(Ctx *ctx, const uint8_t *body, uint64_t n, uint64_t nframes, uint8_t *slots, uint32_t *sizes,
                       void *tmp) {
    ZEncTables *tabs = (ZEncTables *)tmp;
    uint8_t *work = (uint8_t *)tmp + ((sizeof(ZEncTables) + 255) & ~size_t(255));
    hipLaunchKernelGGL(zenc_tables_kernel, dim3(1), dim3(64), 0, ctx->stream, tabs);
    TFG_LAUNCH_CHECK();
    {
        ProfScope _ps(ctx, "codec.zstd.compress");
        hipLaunchKernelGGL(zstd_encode_kernel, dim3((unsigned)nframes), dim3(64), 0, ctx->stream, body, n, nframes, slots,
                           sizes, work, (const ZEncTables *)tabs);
    }
    TFG_LAUNCH_CHECK();
    return TFG_OK;
}

#ifdef TFG_ZE_PROF
extern "C" int tfg_zenc_prof(unsigned long long *out) { // reads and clears the phase totals
    TFG_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_zprof), sizeof(g_zprof)));
    static const unsigned long long zero[8] = {0};
    TFG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_zprof), zero, sizeof(zero)));
    return 0;
}
#endif

} // namespace tfg
