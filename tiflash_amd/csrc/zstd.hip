// zstd.hip — ZSTD MPP packets on the device (§8 f1, HIGH_COMPRESSION mode): the stages of
// zstd_dec.h as kernels (the format and the stage split are described there).
//
//   scan     zstd_scan_kernel     one wave per packet frame, lanes in lockstep; the headers it
//                                 parses come through 512-byte LDS windows (one load each);
//                                 run twice: counts, then descriptors at exact bases
//   entropy  zstd_block_kernel    one 128-thread workgroup per block: the compressed block is
//                                 staged in LDS; wave 0 decodes the literals (the four Huffman
//                                 streams on lanes 0-3), wave 1 the sequences (FSE, lockstep,
//                                 records flushed 64 at a time) — the two halves are independent
//   resolve  zstd_resolve_kernel  one 1024-thread workgroup per packet frame: repeat offsets and
//                                 positions by scans (the repeat-offset updates compose), every check
//   execute  zstd_expand_kernel   every output byte: literal bytes copied, match bytes get their
//                                 source index and join a list; zstd_jump_kernel (src = src[src]
//                                 over the list, the still-unresolved bytes forming the next list:
//                                 log2 of the longest match chain rounds, each shorter than the
//                                 last); zstd_gather_kernel copies the match bytes
//   checksum zstd_check_kernel    one wave per ZSTD frame with a content checksum (XXH64)
// Every kernel is memory-safe on any input: a malformed frame raises the error flag and the later
// kernels keep every index inside the launch's buffers.
#include "common.h"
#include "codec_zstd.h"
#include "zstd_dec.h"

namespace tfg {
namespace {

constexpr int FRAME_HDR = 9;                              // COMPRESSED_BLOCK_HEADER_SIZE
constexpr uint64_t ZSTD_SCRATCH = (uint64_t)4 << 30;      // per launch group: descriptors, records, literals, sources
constexpr uint32_t ZCHUNK = 4096;                         // output bytes per expand workgroup
constexpr int ZMAX_ROUNDS = 40;                           // pointer-jumping rounds (chains < 2^40)

__device__ __forceinline__ void lds_order() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------- scan
// The scan's byte source on the device: a ZSCAN_WIN-byte LDS window, loaded by all lanes (8 bytes
// each) whenever a read leaves it.  Every lane runs the scan (uniform control flow).
struct ZSrcWin {
    const uint8_t *p;
    int64_t n;
    uint8_t *win;
    int64_t base;
    __device__ const uint8_t *at(int64_t off, int64_t k) {
        if (base < 0 || off < base || off + k > base + tfz::ZSCAN_WIN) {
            base = off;
            const uint32_t lane = threadIdx.x & 63;
            uint8_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int64_t i = off + lane * 8 + j;
                v[j] = i < n ? p[i] : 0;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) win[lane * 8 + j] = v[j];
            lds_order();
        }
        return win + (off - base);
    }
};

// pass 1 (bases null): counts[i] = the frame's ZCounts (blocks = ZNONE: malformed).  pass 2:
// descriptors at bases[4 i + 0 / 1 / 2] (blocks / frames / records of frames before i).
__global__ void __launch_bounds__(64) zstd_scan_kernel(const uint8_t *pkt, const uint64_t *foff, const uint64_t *roff,
                                                       uint64_t f0, tfz::ZCounts *counts, const uint32_t *bases,
                                                       tfz::ZBlockDesc *blocks, tfz::ZFrameDesc *frames, unsigned *err) {
    __shared__ uint8_t win[tfz::ZSCAN_WIN];
    const uint32_t i = blockIdx.x, lane = threadIdx.x;
    const uint64_t f = f0 + i;
    const uint64_t fb = foff[f + 1] - foff[f], raw = roff[f + 1] - roff[f];
    ZSrcWin S{pkt + foff[f] + FRAME_HDR, (int64_t)(fb - FRAME_HDR), win, -1};
    tfz::ZScan o;
    o.pframe = i;
    o.writer = lane == 0;
    if (bases) {
        o.blocks = blocks;
        o.frames = frames;
        o.block0 = bases[4 * i];
        o.frame0 = bases[4 * i + 1];
        o.rec0 = bases[4 * i + 2];
        o.lit0 = (uint32_t)(roff[f] - roff[f0]);
    }
    const bool ok = tfz::zstd_scan(S, (int64_t)(fb - FRAME_HDR), raw, o);
    if (lane == 0) {
        if (!bases) counts[i] = ok ? o.c : tfz::ZCounts{tfz::ZNONE, 0, 0, 0};
        if (!ok) atomicOr(err, 1u);
    }
}

// ---------------------------------------------------------------- entropy
// The tables of one block in LDS (~18.7 KB, so that two blocks of up to ~60 KB share a CU): the
// sequence tables and a two-symbol Huffman table built from the weights (sym1 | sym2 << 8 |
// len1 << 16 | (len1 + len2) << 20 | two << 25), with the symbols sorted by weight class.
struct ZBlockLds : tfz::ZSeqTables {
    uint32_t huf2[1 << tfz::ZHUF_MAXBITS];
    int huf_bits;
    uint16_t cstart[tfz::ZHUF_MAXBITS + 2], cbase[tfz::ZHUF_MAXBITS + 2]; // class k: first entry, first sorted symbol
    uint8_t syms[256];                                                      // symbols by (weight, symbol)
    // work space of the table builds (private arrays would live in scratch memory, ~1 us a
    // dependent access): the literal wave's Huffman weights, the sequence wave's FSE builds
    uint8_t weight[256];
    tfz::FseEntry hft[64];
    int16_t hnorm[16];
    uint16_t hnext[256];
    int16_t snorm[53];
    uint16_t snext[256];
};
// A lane's backward bitstream over the LDS-staged block (tfz::BitR's bits, 32-bit positions: a
// block is at most 128 KB).  `win` holds stream bits [wlo, wlo + 64); after a refill at least 57
// bits can be read.
struct LBits {
    const uint8_t *p; // LDS, 16 bytes of slack past the block
    int32_t n, pos, wlo;
    uint64_t win;
    __device__ __forceinline__ bool init(const uint8_t *buf, int32_t len) {
        p = buf;
        n = len;
        const uint32_t last = len > 0 ? buf[len - 1] : 0u;
        pos = last ? (len - 1) * 8 + (31 - __clz((int)last)) : 0;
        wlo = pos;
        win = 0;
        if (!last) return false;
        refill();
        return true;
    }
    __device__ __forceinline__ void refill() {
        const int32_t b0 = ((pos + 7) >> 3) - 8;
        wlo = b0 * 8;
        if (b0 >= 0 && b0 + 8 <= n) {
            typedef __attribute__((address_space(3))) const uint64_t lds_u64;
            const uint8_t *q = p + b0;
            const uint32_t sh = (uint32_t)((uintptr_t)q & 7) * 8;
            lds_u64 *w = (lds_u64 *)(q - ((uintptr_t)q & 7));
            const uint64_t lo = w[0], hi = w[1];
            win = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
        } else {
            uint64_t v = 0;
            for (int k = 0; k < 8; ++k)
                if (b0 + k >= 0 && b0 + k < n) v |= (uint64_t)p[b0 + k] << (8 * k);
            win = v;
        }
    }
    __device__ __forceinline__ uint32_t peek(int k) const { // 1 <= k <= 57
        return (uint32_t)((win >> (pos - k - wlo)) & ((1ull << k) - 1));
    }
};

// The four-lane Huffman decode of a block's literals: lane k < ns decodes stream k.
template <bool AL>
__device__ __forceinline__ bool huf_lanes(const ZBlockLds &T, const uint8_t *ls, int64_t lbytes, uint32_t lsize, int ns, uint8_t *lit,
                          uint32_t lane) {
    int64_t at = 0, len = lbytes, cnt = lsize, o = 0;
    if (ns == 4) {
        tfz::Huf4 h;
        if (!tfz::huf4_split(ls, lbytes, lsize, h)) return false;
        const int k = lane < 4 ? (int)lane : 0;
        at = h.at[k];
        len = h.len[k];
        cnt = h.cnt[k];
        o = k * h.seg;
    }
    bool ok = true;
    if (lane < (uint32_t)ns) {
        LBits bb;
        ok = bb.init(ls + at, (int32_t)len);
        const int mb = T.huf_bits;
        int64_t i = 0;
        for (; ok && i + 1 < cnt;) { // two symbols a lookup while two remain
            // the lanes refill together when one needs it: one refill every few lookups instead
            // of a masked refill in most iterations (the four streams consume at different rates)
            if (__ballot(bb.pos - mb < bb.wlo)) bb.refill();
            const uint32_t e = T.huf2[bb.peek(mb)];
            const bool two = (e >> 25) & 1u;
            lit[o + i] = (uint8_t)e;
            if (two) lit[o + i + 1] = (uint8_t)(e >> 8);
            bb.pos -= two ? (e >> 20) & 31u : (e >> 16) & 15u;
            i += two ? 2 : 1;
            ok = bb.pos >= 0;
        }
        if (ok && i < cnt) { // the last one: the entry's first symbol
            if (bb.pos - mb < bb.wlo) bb.refill();
            const uint32_t e = T.huf2[bb.peek(mb)];
            lit[o + i] = (uint8_t)e;
            bb.pos -= (e >> 16) & 15u;
            ok = bb.pos >= 0;
        }
        ok = ok && bb.pos == 0;
    }
    return __ballot(!ok) == 0;
}

// The Huffman table of a block from its tree description (all lanes of the wave): the weights
// (every lane, in lockstep), the symbols sorted by weight class (lane 0), then the two-symbol
// entries split over the lanes: entry u decodes its first code from the weight classes, and
// the second when its code lies wholly inside the index's remaining bits.
__device__ __forceinline__ bool huf2_read(const uint8_t *src, int64_t n, ZBlockLds &T, uint32_t lane) {
    int nw = 0, mb = 0;
    if (tfz::huf_weights(src, n, T.weight, nw, mb, T.hft, T.hnorm, T.hnext) < 0) return false;
    lds_order();
    // classes by ballots over the weights (64 symbols at a time): counts, starts, sorted symbols
    uint32_t run[tfz::ZHUF_MAXBITS + 2] = {}; // symbols of class k placed so far (wave-uniform)
    uint32_t cnt[tfz::ZHUF_MAXBITS + 2] = {};
    for (int i0 = 0; i0 < nw; i0 += 64) {
        const int i = i0 + (int)lane;
        const uint32_t w = i < nw ? T.weight[i] : 0u;
#pragma unroll
        for (int k = 1; k <= tfz::ZHUF_MAXBITS; ++k) cnt[k] += (uint32_t)__popcll(__ballot(w == (uint32_t)k));
    }
    uint32_t acc = 0, sacc = 0;
#pragma unroll
    for (int k = 1; k <= tfz::ZHUF_MAXBITS + 1; ++k) {
        const bool in = k <= mb;
        if (lane == 0) {
            T.cstart[k] = (uint16_t)(in ? acc : (1u << mb));
            T.cbase[k] = (uint16_t)sacc;
        }
        run[k] = sacc;
        if (in) {
            acc += cnt[k] << (k - 1);
            sacc += cnt[k];
        }
    }
    if (acc != (1u << mb)) return false;
    for (int i0 = 0; i0 < nw; i0 += 64) {
        const int i = i0 + (int)lane;
        const uint32_t w = i < nw ? T.weight[i] : 0u;
        const uint64_t below = (1ull << lane) - 1;
#pragma unroll
        for (int k = 1; k <= tfz::ZHUF_MAXBITS; ++k) {
            const uint64_t m = __ballot(w == (uint32_t)k);
            if (w == (uint32_t)k) T.syms[run[k] + (uint32_t)__popcll(m & below)] = (uint8_t)i;
            run[k] += (uint32_t)__popcll(m);
        }
    }
    if (lane == 0) T.huf_bits = mb;
    lds_order();
    const uint32_t mask = (1u << mb) - 1;
    auto first = [&](uint32_t u, uint32_t &len) -> uint32_t { // the code at the top of index u
        int k = 1;
        while (k < mb && T.cstart[k + 1] <= u) ++k;
        len = (uint32_t)(mb + 1 - k);
        return T.syms[T.cbase[k] + ((u - T.cstart[k]) >> (k - 1))];
    };
    for (uint32_t u = lane; u <= mask; u += 64) {
        uint32_t l1, l2;
        const uint32_t s1 = first(u, l1);
        uint32_t e = s1 | l1 << 16 | l1 << 20;
        if ((int)l1 < mb) {
            const uint32_t s2 = first((u << l1) & mask, l2);
            if ((int)(l1 + l2) <= mb) e = s1 | s2 << 8 | l1 << 16 | (l1 + l2) << 20 | 1u << 25;
        }
        T.huf2[u] = e;
    }
    lds_order();
    return true;
}

__device__ __forceinline__ uint32_t ufl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t ufl64(uint64_t v) {
    return (uint64_t)ufl((uint32_t)v) | ((uint64_t)ufl((uint32_t)(v >> 32)) << 32);
}

// The sequence bitstream reader of a wave decoding in lockstep: the same bits as tfz::BitR over
// the LDS-staged block, its state held in scalar registers (every LDS value is made wave-uniform
// with readfirstlane, so the bit arithmetic runs on the scalar unit).
struct UBits {
    const uint8_t *p; // LDS
    int32_t n, pos, wlo;
    uint64_t win;
    __device__ __forceinline__ bool init(const uint8_t *buf, int32_t len) {
        p = buf;
        n = len;
        if (len <= 0) return false;
        const uint32_t last = ufl(buf[len - 1]);
        if (!last) return false;
        pos = (len - 1) * 8 + (31 - __clz((int)last));
        refill();
        return true;
    }
    __device__ __forceinline__ void refill() {
        const int32_t b0 = ((pos + 7) >> 3) - 8;
        wlo = b0 * 8;
        if (b0 >= 0 && b0 + 8 <= n) { // two aligned LDS words (the stage has 16 bytes of slack)
            typedef __attribute__((address_space(3))) const uint64_t lds_u64;
            const uint8_t *q = p + b0;
            const uint32_t sh = (uint32_t)((uintptr_t)q & 7) * 8;
            lds_u64 *w = (lds_u64 *)(q - ((uintptr_t)q & 7));
            const uint64_t lo = w[0], hi = w[1];
            win = ufl64(sh ? (lo >> sh) | (hi << (64 - sh)) : lo);
        } else {
            uint64_t v = 0;
            for (int k = 0; k < 8; ++k)
                if (b0 + k >= 0 && b0 + k < n) v |= (uint64_t)p[b0 + k] << (8 * k);
            win = ufl64(v);
        }
    }
    __device__ __forceinline__ void need(int k) {
        if (pos - k < wlo) refill();
    }
    __device__ __forceinline__ uint32_t take(int k) { // k <= 32, after need
        if (k == 0) return 0;
        pos -= k;
        return (uint32_t)((win >> (pos - wlo)) & ((1ull << k) - 1));
    }
};

struct USeq { // one decoding-table entry, wave-uniform
    uint32_t value, base, bits, add;
};
__device__ __forceinline__ USeq useq(const tfz::ZSeqEntry *t, uint32_t s) {
    typedef __attribute__((address_space(3))) const uint64_t lds_u64;
    const uint64_t e = ufl64(*(lds_u64 *)(t + s));
    const uint32_t hi = (uint32_t)(e >> 32);
    return USeq{(uint32_t)e, hi & 0xFFFFu, (hi >> 16) & 0xFFu, hi >> 24};
}

// The sequences of one block (tfz::seq_decode's steps): records {ll, ml, offset value}, the
// block's trailing literal run last; record q kept by lane q % 64, 64 stored at a time.
__device__ __forceinline__ bool seq_wave(const ZBlockLds &T, const uint8_t *bits, int32_t n, uint32_t nseq, uint32_t lsize,
                                         tfz::ZRec *recs, uint32_t lane) {
    tfz::ZRec mine{0, 0, 0, 0};
    uint32_t lit_pos = 0;
    if (nseq) {
        UBits bb;
        if (!bb.init(bits, n)) return false;
        const int ll_log = (int)ufl((uint32_t)T.ll_log), of_log = (int)ufl((uint32_t)T.of_log),
                  ml_log = (int)ufl((uint32_t)T.ml_log);
        bb.need(ll_log + of_log + ml_log);
        uint32_t sll = bb.take(ll_log), sof = bb.take(of_log), sml = bb.take(ml_log);
        for (uint32_t q = 0; q < nseq; ++q) {
            const USeq el = useq(T.ll, sll), eo = useq(T.of, sof), em = useq(T.ml, sml);
            bb.need((int)eo.add);
            const uint32_t ofv = eo.value + bb.take((int)eo.add);
            bb.need(32);
            const uint32_t ml = em.value + bb.take((int)em.add);
            const uint32_t ll = el.value + bb.take((int)el.add);
            if (q + 1 < nseq) { // state updates: LL, ML, OF
                bb.need(26);
                sll = el.base + bb.take((int)el.bits);
                sml = em.base + bb.take((int)em.bits);
                sof = eo.base + bb.take((int)eo.bits);
            }
            if (bb.pos < 0 || lit_pos + ll > lsize) return false;
            if ((q & 63) == lane) mine = tfz::ZRec{ll, ml, ofv, 0};
            if ((q & 63) == 63) recs[q - 63 + lane] = mine; // 64 records, one coalesced store
            lit_pos += ll;
        }
        if (bb.pos != 0) return false;
    }
    if ((nseq & 63) == lane) mine = tfz::ZRec{lsize - lit_pos, 0, tfz::ZDIRECT, 0};
    const uint32_t total = nseq + 1, part = total & 63;
    if (part == 0) recs[nseq - 63 + lane] = mine;
    else if (lane < part) recs[total - part + lane] = mine;
    return true;
}

// One workgroup (2 waves) per block; LDS = ZBlockLds + the staged block (dynamic, stage_cap bytes + 16).
__global__ void __launch_bounds__(128) zstd_block_kernel(const uint8_t *pkt, const uint64_t *foff, uint64_t f0,
                                                         const tfz::ZBlockDesc *blocks, uint8_t *lits, tfz::ZRec *recs,
                                                         uint32_t stage_cap, unsigned *err) {
    extern __shared__ __attribute__((aligned(16))) uint8_t zl[];
    ZBlockLds &T = *reinterpret_cast<ZBlockLds *>(zl);
    uint8_t *stage = zl + ((sizeof(ZBlockLds) + 15) & ~size_t(15));
    const tfz::ZBlockDesc d = blocks[blockIdx.x];
    const uint8_t *body = pkt + foff[f0 + d.pframe] + FRAME_HDR;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (d.type == 0) { // raw: a literal run
        for (uint32_t i = tid; i < d.size; i += 128) lits[d.lit + i] = body[d.src + i];
        if (tid == 0) recs[d.rec] = tfz::ZRec{d.size, 0, tfz::ZDIRECT, 0};
        return;
    }
    if (d.type == 1) { // RLE: one literal, then an offset-1 copy
        if (tid == 0) {
            if (d.size) lits[d.lit] = body[d.src];
            recs[d.rec] = tfz::ZRec{d.size ? 1u : 0u, d.size ? d.size - 1 : 0u, tfz::ZDIRECT | (d.size > 1 ? 1u : 0u), 0};
        }
        return;
    }
    { // the block's bytes into LDS (stage_cap >= every compressed block of the launch), 16 loads
      // in flight a thread; 16 zero bytes of slack
        for (uint32_t i0 = tid * 16; i0 < d.size + 16; i0 += 128 * 16) {
            uint8_t v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = i0 + k < d.size ? body[d.src + i0 + k] : 0;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (i0 + k < d.size + 16) stage[i0 + k] = v[k];
        }
    }
    __syncthreads();
    bool ok = true;
    if (wave == 0) { // ---- literals
        uint8_t *lit = lits + d.lit;
        if (d.ltype == 0) {
            for (uint32_t i = lane; i < d.lsize; i += 64) lit[i] = body[d.lit_at + i];
        } else if (d.ltype == 1) {
            const uint8_t c = body[d.lit_at];
            for (uint32_t i = lane; i < d.lsize; i += 64) lit[i] = c;
        } else {
            ok = huf2_read(body + d.huf, d.huf_n, T, lane);
            if (ok) {
                ok = huf_lanes<true>(T, stage + (d.lit_at - d.src), d.lbytes, d.lsize, d.streams, lit, lane);
            }
        }
    } else { // ---- sequences
        if (d.nseq) {
            bool built = true;
            if (lane == 0)
                for (int k = 0; k < 3; ++k)
                    built = built && tfz::seq_table_build(T, k, d.tab[k], d.tab_n[k], body, T.snorm, T.snext);
            lds_order();
            ok = __ballot(lane == 0 && !built) == 0;
        }
        if (ok) {
            ok = seq_wave(T, stage + (ufl(d.seq_at) - ufl(d.src)), (int32_t)ufl(d.seq_n), ufl(d.nseq), ufl(d.lsize),
                          recs + ufl(d.rec), lane);
        }
    }
    if (lane == 0 && !ok) atomicOr(err, 1u);
}

// ---------------------------------------------------------------- resolve
// The repeat offsets as a scan.  A record maps the state (r0, r1, r2) to a new state whose every
// slot is an old slot plus a delta, or a constant (RFC 8878 §3.1.2.5: a new offset shifts the
// three; a repeat code moves one to the front, code 3 with no literals takes r0 - 1).  Such maps
// compose, so a wave scan gives every record the map from the batch's incoming state to the
// state before it, and its offset follows with no serial loop.
struct RepMap {
    uint32_t kinds; // slot k: bits 2k..2k+1 = the old slot it copies (0-2) or 3 = a constant
    uint32_t v[3];  // delta (slot) or value (constant)
};
__device__ __forceinline__ RepMap rep_identity() { return RepMap{0u | 1u << 2 | 2u << 4, {0, 0, 0}}; }
// b after a
__device__ __forceinline__ RepMap rep_compose(const RepMap &a, const RepMap &b) {
    RepMap c;
    c.kinds = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t kb = (b.kinds >> (2 * k)) & 3u;
        uint32_t kind, val;
        if (kb == 3) {
            kind = 3;
            val = b.v[k];
        } else {
            const uint32_t ka = (a.kinds >> (2 * kb)) & 3u;
            const uint32_t va = kb == 0 ? a.v[0] : kb == 1 ? a.v[1] : a.v[2];
            kind = ka;
            val = va + b.v[k];
        }
        c.kinds |= kind << (2 * k);
        c.v[k] = val;
    }
    return c;
}
__device__ __forceinline__ uint32_t rep_slot(const RepMap &m, int k, uint32_t r0, uint32_t r1, uint32_t r2) {
    const uint32_t kind = (m.kinds >> (2 * k)) & 3u;
    return kind == 3 ? m.v[k] : (kind == 0 ? r0 : kind == 1 ? r1 : r2) + m.v[k];
}
__device__ __forceinline__ RepMap rep_shfl_up(const RepMap &m, int d) {
    RepMap o;
    o.kinds = __shfl_up(m.kinds, d, 64);
    o.v[0] = __shfl_up(m.v[0], d, 64);
    o.v[1] = __shfl_up(m.v[1], d, 64);
    o.v[2] = __shfl_up(m.v[2], d, 64);
    return o;
}

// this record's map and its offset's expression: slot ekind of the state before it, plus eval
// (ekind 3: the constant eval)
__device__ __forceinline__ RepMap rec_map(uint32_t of, uint32_t ll, uint32_t &ekind, uint32_t &eval) {
    ekind = 3;
    eval = of & ~tfz::ZDIRECT;
    if (of & tfz::ZDIRECT) return rep_identity();
    if (of > 3) {
        eval = of - 3;
        return RepMap{3u | 0u << 2 | 1u << 4, {of - 3, 0, 0}};
    }
    const uint32_t idx = of - 1 + (ll == 0 ? 1u : 0u);
    eval = idx == 3 ? 0xFFFFFFFFu : 0u;
    ekind = idx == 3 ? 0u : idx;
    if (idx == 1) return RepMap{1u | 0u << 2 | 2u << 4, {0, 0, 0}};
    if (idx == 2) return RepMap{2u | 0u << 2 | 1u << 4, {0, 0, 0}};
    if (idx == 3) return RepMap{0u | 0u << 2 | 1u << 4, {0xFFFFFFFFu, 0, 0}};
    return rep_identity();
}

// One 1024-thread workgroup per packet frame, 1024 records a step (the next step's loaded while
// this one is resolved): every wave scans its 64 records (repeat-offset maps, output and literal
// positions), wave 0 scans the 16 wave totals, and every record gets its offset and positions
// from the step's carry.  Records are rewritten as {pos, ll, lpos, off}.
constexpr int RS_T = 1024;
__global__ void __launch_bounds__(RS_T) zstd_resolve_kernel(const uint64_t *roff, uint64_t f0, const uint32_t *bases,
                                                            tfz::ZFrameDesc *frames, tfz::ZRec *recs, unsigned *err) {
    constexpr int NW = RS_T / 64;
    __shared__ RepMap s_map[NW];      // wave totals, then the waves' exclusive prefixes
    __shared__ uint32_t s_sp[NW], s_ll[NW];
    __shared__ uint32_t s_carry[5];   // pos, lpos, r0, r1, r2 before the step
    __shared__ uint32_t s_next[5];    // ... after it
    __shared__ int s_bad;
    const uint32_t i = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t f = f0 + i, raw = roff[f + 1] - roff[f];
    if (tid == 0) {
        s_carry[0] = 0;
        s_carry[1] = (uint32_t)(roff[f] - roff[f0]);
        s_bad = 0;
    }
    __syncthreads();
    for (uint32_t z = bases[4 * i + 1]; z < bases[4 * i + 5]; ++z) {
        const tfz::ZFrameDesc fr = frames[z];
        const uint32_t zstart = s_carry[0];
        __syncthreads();
        if (tid == 0) { // every ZSTD frame starts from the initial repeat offsets
            s_carry[2] = 1;
            s_carry[3] = 4;
            s_carry[4] = 8;
        }
        tfz::ZRec nxt{0, 0, tfz::ZDIRECT, 0};
        if (fr.rec0 + tid < fr.rec1) nxt = recs[fr.rec0 + tid];
        __syncthreads();
        for (uint32_t q0 = fr.rec0; q0 < fr.rec1; q0 += RS_T) {
            const tfz::ZRec r = nxt;
            nxt = tfz::ZRec{0, 0, tfz::ZDIRECT, 0};
            if (q0 + RS_T + tid < fr.rec1) nxt = recs[q0 + RS_T + tid];
            const bool valid = q0 + tid < fr.rec1;
            const uint32_t ll = valid ? r.a : 0, ml = valid ? r.b : 0, of = valid ? r.c : tfz::ZDIRECT;
            uint32_t ekind, eval;
            RepMap inc = rec_map(of, ll, ekind, eval);
            uint32_t incl = ll + ml, linc = ll; // spans: a step covers at most 1024 x 128 KB + 128 KB
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const RepMap y = rep_shfl_up(inc, d);
                const uint32_t yp = __shfl_up(incl, d, 64), yl = __shfl_up(linc, d, 64);
                if (lane >= (uint32_t)d) {
                    inc = rep_compose(y, inc);
                    incl += yp;
                    linc += yl;
                }
            }
            if (lane == 63) {
                s_map[wave] = inc;
                s_sp[wave] = incl;
                s_ll[wave] = linc;
            }
            __syncthreads();
            if (wave == 0) { // exclusive scan of the wave totals (lanes < NW), and the step's carry out
                RepMap m = lane < NW ? s_map[lane] : rep_identity();
                uint32_t sp = lane < NW ? s_sp[lane] : 0u, sl = lane < NW ? s_ll[lane] : 0u;
#pragma unroll
                for (int d = 1; d < NW; d <<= 1) {
                    const RepMap y = rep_shfl_up(m, d);
                    const uint32_t yp = __shfl_up(sp, d, 64), yl = __shfl_up(sl, d, 64);
                    if (lane >= (uint32_t)d) {
                        m = rep_compose(y, m);
                        sp += yp;
                        sl += yl;
                    }
                }
                RepMap e = rep_shfl_up(m, 1);
                const uint32_t ep = __shfl_up(sp, 1, 64), el = __shfl_up(sl, 1, 64);
                if (lane < NW) {
                    s_map[lane] = lane == 0 ? rep_identity() : e;
                    s_sp[lane] = lane == 0 ? 0u : ep;
                    s_ll[lane] = lane == 0 ? 0u : el;
                }
                if (lane == NW - 1) {
                    const uint32_t c2 = s_carry[2], c3 = s_carry[3], c4 = s_carry[4];
                    const uint64_t np = (uint64_t)s_carry[0] + sp;
                    if (np > raw) s_bad = 1;
                    s_next[0] = (uint32_t)np;
                    s_next[1] = s_carry[1] + sl;
                    s_next[2] = rep_slot(m, 0, c2, c3, c4);
                    s_next[3] = rep_slot(m, 1, c2, c3, c4);
                    s_next[4] = rep_slot(m, 2, c2, c3, c4);
                }
            }
            __syncthreads();
            { // this wave's incoming state, then each record's
                const RepMap pw = s_map[wave];
                const uint32_t c2 = s_carry[2], c3 = s_carry[3], c4 = s_carry[4];
                const uint32_t w0 = rep_slot(pw, 0, c2, c3, c4), w1 = rep_slot(pw, 1, c2, c3, c4), w2 = rep_slot(pw, 2, c2, c3, c4);
                RepMap exc = rep_shfl_up(inc, 1);
                if (lane == 0) exc = rep_identity();
                const uint32_t s0 = rep_slot(exc, 0, w0, w1, w2), s1 = rep_slot(exc, 1, w0, w1, w2),
                               s2 = rep_slot(exc, 2, w0, w1, w2);
                const uint32_t myoff = ekind == 3 ? eval : (ekind == 0 ? s0 : ekind == 1 ? s1 : s2) + eval;
                const uint64_t mypos = (uint64_t)s_carry[0] + s_sp[wave] + incl - (ll + ml);
                const uint32_t mylpos = s_carry[1] + s_ll[wave] + linc - ll;
                if (valid) {
                    bool bad = false;
                    if (ml && (myoff == 0 || (uint64_t)myoff > mypos + ll - zstart)) bad = true;
                    if (mypos + ll + ml > raw) bad = true;
                    if (bad) s_bad = 1;
                    recs[q0 + tid] = tfz::ZRec{(uint32_t)mypos, ll, mylpos, myoff};
                }
            }
            __syncthreads();
            if (tid < 5) s_carry[tid] = s_next[tid];
            __syncthreads();
            if (s_bad) break;
        }
        if (tid == 0) {
            frames[z].out0 = zstart;
            frames[z].out1 = s_carry[0];
            if (fr.fcs != ~0ull && (uint64_t)(s_carry[0] - zstart) != fr.fcs) s_bad = 1;
        }
        __syncthreads();
        if (s_bad) break;
    }
    if (tid == 0 && (s_bad || s_carry[0] != raw)) atomicOr(err, 1u);
}

// ---------------------------------------------------------------- execute
// Worklists of byte indices (launch-relative): count + entries.  A block appends its threads'
// entries contiguously with ONE global atomic (per-wave atomics on one counter serialise: a
// first round of 25M entries spent 4.6 ms in them).  Every thread of the block calls it;
// entry k of a thread is vals[k] when bit k of mask is set.  s_w: (blockDim / 64 + 1) words.
template <int K>
__device__ __forceinline__ void block_append(uint32_t mask, const uint32_t (&vals)[K], uint32_t *list, unsigned *count,
                                             uint32_t *s_w) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t cnt = (uint32_t)__popc(mask);
    uint32_t x = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (uint32_t w = 0; w < nw; ++w) {
            const uint32_t v = s_w[w];
            s_w[w] = tot;
            tot += v;
        }
        s_w[nw] = tot ? atomicAdd(count, tot) : 0u;
    }
    __syncthreads();
    uint32_t pos = s_w[nw] + s_w[wave] + x - cnt;
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (mask & (1u << k)) list[pos++] = vals[k];
    __syncthreads(); // s_w is reused by the next call
}

// One workgroup per ZCHUNK output bytes of a packet frame (cbase: prefix of the frames' chunk
// counts); 16 bytes a thread.  Literal bytes are written to `out` and point at themselves
// (src[g] = g); a match byte points at its source byte (src[g] = g - off, or for byte j >= off of
// an overlapping match the byte j % off of the period before it) and joins the list of match
// bytes.
__global__ void __launch_bounds__(256) zstd_expand_kernel(const uint64_t *roff, uint64_t f0, uint32_t nf,
                                                          const uint32_t *cbase, const uint32_t *bases, const tfz::ZRec *recs,
                                                          const uint8_t *lits, uint64_t nlits, uint8_t *out, uint32_t *src,
                                                          uint32_t *mlist, unsigned *mcount, unsigned *err) {
    __shared__ uint32_t range[2];
    const uint32_t c = blockIdx.x;
    uint32_t lo = 0, hi = nf; // the frame: last i with cbase[i] <= c
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (cbase[mid] <= c) lo = mid;
        else hi = mid;
    }
    const uint32_t i = lo;
    const uint64_t f = f0 + i, raw = roff[f + 1] - roff[f], g0 = roff[f] - roff[f0];
    const uint32_t b0 = (c - cbase[i]) * ZCHUNK;
    const uint32_t b1 = (uint32_t)(b0 + ZCHUNK < raw ? b0 + ZCHUNK : raw);
    const uint32_t r0 = bases[4 * i + 2], r1 = bases[4 * i + 6]; // the frame's records
    if (r0 == r1) return;
    auto last_le = [&](uint32_t a, uint32_t z, uint32_t b) { // last record in [a, z) with pos <= b
        while (z - a > 1) {
            const uint32_t m = (a + z) / 2;
            if (recs[m].a <= b) a = m;
            else z = m;
        }
        return a;
    };
    if (threadIdx.x == 0) range[0] = last_le(r0, r1, b0);
    if (threadIdx.x == 1) range[1] = last_le(r0, r1, b1 ? b1 - 1 : 0) + 1;
    __syncthreads();
    const uint32_t s = b0 + threadIdx.x * 16;
    const uint32_t e = s < b1 ? (s + 16 < b1 ? s + 16 : b1) : s;
    bool bad = false;
    uint32_t sv[16];
    uint32_t mmask = 0;
    if (s < e) {
        uint32_t r = last_le(range[0], range[1], s);
        tfz::ZRec rec = recs[r];
        uint32_t end = r + 1 < r1 ? recs[r + 1].a : (uint32_t)raw;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t b = s + k;
            if (b >= e) break;
            while (b >= end && r + 1 < r1) {
                ++r;
                rec = recs[r];
                end = r + 1 < r1 ? recs[r + 1].a : (uint32_t)raw;
            }
            const uint64_t g = g0 + b;
            sv[k] = (uint32_t)g;
            if (b < rec.a) {
                bad = true; // inconsistent positions (a malformed frame)
            } else if (b - rec.a < rec.b) {
                const uint64_t li = (uint64_t)rec.c + (b - rec.a);
                if (li < nlits) out[g] = lits[li];
                else bad = true;
            } else if (rec.d == 0 || rec.d > rec.a + rec.b) {
                bad = true;
            } else {
                // an overlapping match (offset < length) repeats its first `off` bytes: byte j
                // of the match points into that period before the match, one hop instead of
                // j / off (long runs of one byte no longer make long chains)
                const uint32_t ms = rec.a + rec.b, j = b - ms;
                sv[k] = (uint32_t)(g0 + ms - rec.d + (j < rec.d ? j : j % rec.d));
                mmask |= 1u << k;
            }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (s + k < e) src[g0 + s + k] = sv[k];
    }
    // the match bytes into the list: one atomic per workgroup
    __shared__ uint32_t s_w[256 / 64 + 1];
    uint32_t gv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) gv[k] = (uint32_t)(g0 + s + k);
    block_append<16>(mmask, gv, mlist, mcount, s_w);
    if (bad) atomicOr(err, 1u);
}

// One pointer-jumping round over the bytes of list `in` (count *nin): src[g] = src[src[g]]; the
// bytes whose source is still not a literal go to list `out`.  Tiles of 4096 entries (16 a
// thread, all their loads in flight together), grid-stride over the count read on the device,
// so rounds are launched without a host read between them.
__global__ void __launch_bounds__(256) zstd_jump_kernel(uint32_t *src, const uint32_t *in, const unsigned *nin,
                                                        uint32_t *outl, unsigned *nout) {
    __shared__ uint32_t s_w[256 / 64 + 1];
    const uint32_t n = *nin;
    for (uint32_t t0 = blockIdx.x * 4096u; t0 < n; t0 += gridDim.x * 4096u) {
        uint32_t g[16], sv[16];
        uint32_t mask = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t i = t0 + (uint32_t)k * 256 + threadIdx.x;
            g[k] = i < n ? in[i] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) sv[k] = t0 + (uint32_t)k * 256 + threadIdx.x < n ? src[g[k]] : 0u;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (t0 + (uint32_t)k * 256 + threadIdx.x >= n) continue;
            const uint32_t t = src[sv[k]];
            if (t != sv[k]) {
                src[g[k]] = t;
                if (src[t] != t) mask |= 1u << k;
            }
        }
        block_append<16>(mask, g, outl, nout, s_w);
    }
}

// match bytes (list, count *n) take their source byte: a literal byte once the rounds are done
__global__ void __launch_bounds__(256) zstd_gather_kernel(const uint32_t *src, const uint32_t *list, const unsigned *n,
                                                          uint8_t *out) {
    const uint32_t cnt = *n, stride = gridDim.x * 256;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += stride) {
        const uint32_t g = list[i];
        out[g] = out[src[g]];
    }
}

__device__ __forceinline__ uint64_t load8_bytes(const uint8_t *p) {
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) v |= (uint64_t)p[k] << (8 * k);
    return v;
}

// XXH64 of p[0, len) by the wave: 16 stripes of 32 bytes loaded per step (lane 4s + k holds word
// k of stripe s), folded in order by lanes 0-3 (accumulator k), then lane 0 merges and hashes the
// tail.  Returns the low 32 bits (in every lane).
__device__ uint32_t wave_xxh64(const uint8_t *p, uint64_t len) {
    const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                   P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
    const uint32_t lane = threadIdx.x & 63, k = lane & 3;
    uint64_t h = 0;
    const uint64_t ns = len / 32;
    if (ns) {
        uint64_t v = k == 0 ? P1 + P2 : k == 1 ? P2 : k == 2 ? 0 : 0 - P1;
        for (uint64_t s0 = 0; s0 < ns; s0 += 16) {
            const uint64_t s = s0 + lane / 4;
            const uint64_t wd = s < ns ? load8_bytes(p + 32 * s + 8 * k) : 0;
            const int steps = (int)(ns - s0 < 16 ? ns - s0 : 16);
            for (int t = 0; t < steps; ++t) {
                const uint64_t x = __shfl(wd, 4 * t + (int)k, 64);
                v = tfz::rotl64(v + x * P2, 31) * P1;
            }
        }
        const uint64_t v1 = __shfl(v, 0, 64), v2 = __shfl(v, 1, 64), v3 = __shfl(v, 2, 64), v4 = __shfl(v, 3, 64);
        h = tfz::rotl64(v1, 1) + tfz::rotl64(v2, 7) + tfz::rotl64(v3, 12) + tfz::rotl64(v4, 18);
        const uint64_t vs[4] = {v1, v2, v3, v4};
        for (int q = 0; q < 4; ++q) h = (h ^ (tfz::rotl64(vs[q] * P2, 31) * P1)) * P1 + P4;
    } else {
        h = P5;
    }
    h += len;
    const uint8_t *e = p + len, *t = p + 32 * ns; // the tail: lane 0 (<= 31 bytes)
    if (lane == 0) {
        while (t + 8 <= e) {
            h ^= tfz::rotl64(load8_bytes(t) * P2, 31) * P1;
            h = tfz::rotl64(h, 27) * P1 + P4;
            t += 8;
        }
        if (t + 4 <= e) {
            h ^= (uint64_t)tfz::rd32(t) * P1;
            h = tfz::rotl64(h, 23) * P2 + P3;
            t += 4;
        }
        while (t < e) {
            h ^= (*t) * P5;
            h = tfz::rotl64(h, 11) * P1;
            ++t;
        }
        h ^= h >> 33;
        h *= P2;
        h ^= h >> 29;
        h *= P3;
        h ^= h >> 32;
    }
    return (uint32_t)__shfl(h, 0, 64);
}

// One wave per ZSTD frame: the content checksum over its output (frames without one return).
__global__ void __launch_bounds__(64) zstd_check_kernel(const uint64_t *roff, uint64_t f0, const tfz::ZFrameDesc *frames,
                                                        const uint8_t *out, unsigned *err) {
    const tfz::ZFrameDesc fr = frames[blockIdx.x];
    if (!fr.has_checksum) return;
    if (fr.out1 < fr.out0) {
        if (threadIdx.x == 0) atomicOr(err, 1u);
        return;
    }
    const uint8_t *p = out + (roff[f0 + fr.pframe] - roff[f0]) + fr.out0;
    if (wave_xxh64(p, fr.out1 - fr.out0) != fr.checksum && threadIdx.x == 0) atomicOr(err, 1u);
}

struct PoolBuf { // a call's work space from the context's call arena (common.h DevArena)
    Ctx *ctx;
    void *p = nullptr;
    uint64_t cap = 0;
    explicit PoolBuf(Ctx *c) : ctx(c) { arena_hold(ctx); }
    ~PoolBuf() { arena_drop(ctx); }
    PoolBuf(const PoolBuf &) = delete;
    PoolBuf &operator=(const PoolBuf &) = delete;
    int reserve(uint64_t bytes) { // a larger block when it grows (the smaller one returns with the call)
        if (bytes <= cap) return TFG_OK;
        if (int rc = arena_alloc(ctx, bytes, &p)) return rc;
        cap = bytes;
        return TFG_OK;
    }
};

} // namespace

int zstd_decode_frames(Ctx *ctx, const uint8_t *packet, uint64_t nf, const uint64_t *dfo, const uint64_t *dro,
                       const uint64_t *fo, const uint64_t *ro, uint8_t *dst, unsigned *err) {
    // ---- pass 1: counts of every frame (one read-back)
    PoolBuf cbuf(ctx), buf(ctx);
    if (int rc = cbuf.reserve(nf * sizeof(tfz::ZCounts) + 256)) return rc;
    tfz::ZCounts *dcounts = (tfz::ZCounts *)cbuf.p;
    {
        ProfScope _ps(ctx, "codec.zstd.scan");
        hipLaunchKernelGGL(zstd_scan_kernel, dim3((unsigned)nf), dim3(64), 0, ctx->stream, packet, dfo, dro, (uint64_t)0,
                           dcounts, (const uint32_t *)nullptr, (tfz::ZBlockDesc *)nullptr, (tfz::ZFrameDesc *)nullptr, err);
        TFG_LAUNCH_CHECK();
    }
    std::vector<tfz::ZCounts> counts(nf);
    TFG_HIP(hipMemcpyAsync(counts.data(), dcounts, nf * sizeof(tfz::ZCounts), hipMemcpyDeviceToHost, ctx->stream));
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    for (uint64_t f = 0; f < nf; ++f)
        TFG_CHECK(counts[f].blocks != tfz::ZNONE, TFG_ERR_INVALID_ARG, "corrupted ZSTD frame (Cannot decompress)");
    auto need = [&](uint64_t f) { // launch bytes of frame f: descriptors, records, literals, sources
        const uint64_t raw = ro[f + 1] - ro[f];
        return (uint64_t)counts[f].blocks * sizeof(tfz::ZBlockDesc) + (uint64_t)counts[f].frames * sizeof(tfz::ZFrameDesc) +
               (uint64_t)counts[f].recs * sizeof(tfz::ZRec) + raw * 17 + 64; // literals + src + 3 byte lists
    };
    for (uint64_t a = 0; a < nf;) {
        // ---- a launch group: frames [a, z) within ZSTD_SCRATCH and 32-bit indices
        uint64_t z = a, bytes = 0, raw = 0, recs = 0;
        while (z < nf) {
            const uint64_t nb = need(z), nr = ro[z + 1] - ro[z];
            if (z > a && (bytes + nb > ZSTD_SCRATCH || raw + nr >= (1ull << 31) || recs + counts[z].recs >= (1ull << 31))) break;
            bytes += nb;
            raw += nr;
            recs += counts[z].recs;
            ++z;
        }
        TFG_CHECK(raw < (1ull << 31) && recs < (1ull << 31), TFG_ERR_CAPACITY, "ZSTD frame of %llu bytes",
                  (unsigned long long)raw);
        const uint64_t g = z - a;
        std::vector<uint32_t> bases(4 * (g + 1)), cbase(g + 1);
        uint32_t nb = 0, nz = 0, nr = 0, nc = 0, max_comp = 0;
        for (uint64_t i = 0; i <= g; ++i) {
            bases[4 * i] = nb;
            bases[4 * i + 1] = nz;
            bases[4 * i + 2] = nr;
            cbase[i] = nc;
            if (i == g) break;
            const tfz::ZCounts &c = counts[a + i];
            nb += c.blocks;
            nz += c.frames;
            nr += c.recs;
            nc += (uint32_t)((ro[a + i + 1] - ro[a + i] + ZCHUNK - 1) / ZCHUNK);
            if (c.max_comp > max_comp) max_comp = c.max_comp;
        }
        Carver cv;
        const size_t o_blk = cv.take<tfz::ZBlockDesc>(nb + 1), o_frm = cv.take<tfz::ZFrameDesc>(nz + 1);
        const size_t o_rec = cv.take<tfz::ZRec>(nr + 1), o_lit = cv.take<uint8_t>(raw + 1);
        const size_t o_src = cv.take<uint32_t>(raw + 1), o_bas = cv.take<uint32_t>(bases.size());
        const size_t o_cb = cv.take<uint32_t>(cbase.size()), o_cnt = cv.take<unsigned>(4);
        const size_t o_l0 = cv.take<uint32_t>(raw + 1), o_l1 = cv.take<uint32_t>(raw + 1), o_l2 = cv.take<uint32_t>(raw + 1);
        if (int rc = buf.reserve(cv.off)) return rc;
        char *sb = (char *)buf.p;
        tfz::ZBlockDesc *blk = (tfz::ZBlockDesc *)(sb + o_blk);
        tfz::ZFrameDesc *frm = (tfz::ZFrameDesc *)(sb + o_frm);
        tfz::ZRec *rec = (tfz::ZRec *)(sb + o_rec);
        uint8_t *lit = (uint8_t *)(sb + o_lit);
        uint32_t *src = (uint32_t *)(sb + o_src), *dbases = (uint32_t *)(sb + o_bas), *dcb = (uint32_t *)(sb + o_cb);
        unsigned *lcount = (unsigned *)(sb + o_cnt); // [0] match bytes, [1] / [2] the round lists
        uint32_t *mlist = (uint32_t *)(sb + o_l0), *wl[2] = {(uint32_t *)(sb + o_l1), (uint32_t *)(sb + o_l2)};
        TFG_HIP(hipMemsetAsync(lcount, 0, 4 * sizeof(unsigned), ctx->stream));
        TFG_HIP(hipMemcpyAsync(dbases, bases.data(), bases.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        TFG_HIP(hipMemcpyAsync(dcb, cbase.data(), cbase.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        uint8_t *out = dst + ro[a];
        {
            ProfScope _ps(ctx, "codec.zstd.decompress");
            hipLaunchKernelGGL(zstd_scan_kernel, dim3((unsigned)g), dim3(64), 0, ctx->stream, packet, dfo, dro, a,
                               (tfz::ZCounts *)nullptr, (const uint32_t *)dbases, blk, frm, err);
            TFG_LAUNCH_CHECK();
            if (nb) {
                const uint32_t cap = (max_comp + 15) & ~15u;
                const size_t lds = ((sizeof(ZBlockLds) + 15) & ~size_t(15)) + cap + 16;
                // <= 18.7 KB of tables + a 128 KB block + slack: within gfx950's 160 KB of LDS (two
                // workgroups per CU while the launch's largest compressed block is under ~61 KB)
                TFG_CHECK(lds <= 160 * 1024, TFG_ERR_LOGICAL, "ZSTD block stage of %zu bytes", lds);
                hipLaunchKernelGGL(zstd_block_kernel, dim3(nb), dim3(128), lds, ctx->stream, packet, dfo, a,
                                   (const tfz::ZBlockDesc *)blk, lit, rec, cap, err);
                TFG_LAUNCH_CHECK();
            }
            hipLaunchKernelGGL(zstd_resolve_kernel, dim3((unsigned)g), dim3(RS_T), 0, ctx->stream, dro, a,
                               (const uint32_t *)dbases, frm, rec, err);
            TFG_LAUNCH_CHECK();
            if (nc) {
                hipLaunchKernelGGL(zstd_expand_kernel, dim3(nc), dim3(256), 0, ctx->stream, dro, a, (uint32_t)g,
                                   (const uint32_t *)dcb, (const uint32_t *)dbases, (const tfz::ZRec *)rec,
                                   (const uint8_t *)lit, raw, out, src, mlist, lcount, err);
                TFG_LAUNCH_CHECK();
            }
        }
        // pointer jumping over the match bytes: rounds go in batches of 4 without a host read
        // between them (an empty list costs one launch); the batch's last list count decides
        const unsigned jg = (unsigned)std::min<uint64_t>((raw + 4095) / 4096, 2048); // jump tiles of 4096
        const unsigned gg = (unsigned)std::min<uint64_t>((raw + 255) / 256, 16384);
        if (raw) {
            const uint32_t *in = mlist;
            const unsigned *nin = lcount;
            int round = 0;
            for (bool more = true; more;) {
                for (int k = 0; k < 4; ++k, ++round) {
                    TFG_CHECK(round < ZMAX_ROUNDS, TFG_ERR_INVALID_ARG, "corrupted ZSTD frame (Cannot decompress)");
                    uint32_t *o = wl[round & 1];
                    unsigned *no = lcount + 1 + (round & 1);
                    TFG_HIP(hipMemsetAsync(no, 0, sizeof(unsigned), ctx->stream));
                    ProfScope _ps(ctx, "codec.zstd.decompress");
                    hipLaunchKernelGGL(zstd_jump_kernel, dim3(jg), dim3(256), 0, ctx->stream, src, in, nin, o, no);
                    TFG_LAUNCH_CHECK();
                    in = o;
                    nin = no;
                }
                TFG_HIP(hipMemcpyAsync(ctx->host_pinned, nin, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
                TFG_HIP(hipStreamSynchronize(ctx->stream));
                more = *(const unsigned *)ctx->host_pinned != 0;
            }
            ProfScope _ps(ctx, "codec.zstd.decompress");
            hipLaunchKernelGGL(zstd_gather_kernel, dim3(gg), dim3(256), 0, ctx->stream, (const uint32_t *)src,
                               (const uint32_t *)mlist, (const unsigned *)lcount, out);
            TFG_LAUNCH_CHECK();
        }
        if (nz) {
            ProfScope _ps(ctx, "codec.zstd.decompress");
            hipLaunchKernelGGL(zstd_check_kernel, dim3(nz), dim3(64), 0, ctx->stream, dro, a, (const tfz::ZFrameDesc *)frm,
                               (const uint8_t *)out, err);
            TFG_LAUNCH_CHECK();
        }
        TFG_HIP(hipStreamSynchronize(ctx->stream)); // the host base tables stay alive until here
        a = z;
    }
    return TFG_OK;
}

} // namespace tfg
