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
//   resolve  zstd_resolve_kernel  one wave per packet frame: repeat offsets in order (readlane),
//                                 positions by wave scans, every check
//   execute  zstd_expand_kernel   every output byte: literal bytes copied, match bytes get their
//                                 source index; zstd_jump_kernel (src = src[src], repeated until no
//                                 byte points at a match byte: log2 of the longest match chain
//                                 rounds); zstd_gather_kernel copies the match bytes
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
__device__ __forceinline__ uint32_t rl32(uint32_t v, uint32_t j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j); }

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
// The four-lane Huffman decode of a block's literals: lane k < ns decodes stream k.
template <bool AL>
__device__ bool huf_lanes(const tfz::ZTables &T, const uint8_t *ls, int64_t lbytes, uint32_t lsize, int ns, uint8_t *lit,
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
        tfz::BitR<AL> bb;
        ok = bb.init(ls + at, len);
        const int mb = T.huf_bits;
        for (int64_t i = 0; ok && i < cnt; ++i) {
            bb.need(mb);
            const uint16_t e = T.huf[bb.peek(mb)];
            lit[o + i] = (uint8_t)e;
            bb.pos -= e >> 8;
            ok = bb.pos >= 0;
        }
        ok = ok && bb.pos == 0;
    }
    return __ballot(!ok) == 0;
}

template <bool AL>
__device__ bool seq_wave(const tfz::ZTables &T, const uint8_t *bits, int64_t n, const tfz::ZBlockDesc &d, tfz::ZRec *recs,
                         uint32_t lane) {
    tfz::ZRec mine{0, 0, 0, 0};
    const bool ok = tfz::seq_decode<AL>(T, bits, n, d.nseq, d.lsize, [&](uint32_t q, const tfz::ZRec &r) {
        if ((q & 63) == lane) mine = r;
        if ((q & 63) == 63) recs[d.rec + q - 63 + lane] = mine; // 64 records, one coalesced store
    });
    const uint32_t total = d.nseq + 1, part = total & 63;
    if (ok && part && lane < part) recs[d.rec + total - part + lane] = mine;
    return ok;
}

// One workgroup (2 waves) per block; LDS = ZTables + the staged block (dynamic, stage_cap bytes + 16).
__global__ void __launch_bounds__(128) zstd_block_kernel(const uint8_t *pkt, const uint64_t *foff, uint64_t f0,
                                                         const tfz::ZBlockDesc *blocks, uint8_t *lits, tfz::ZRec *recs,
                                                         uint32_t stage_cap, unsigned *err) {
    extern __shared__ __attribute__((aligned(16))) uint8_t zl[];
    tfz::ZTables &T = *reinterpret_cast<tfz::ZTables *>(zl);
    uint8_t *stage = zl + ((sizeof(tfz::ZTables) + 15) & ~size_t(15));
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
    const bool staged = d.size <= stage_cap;
    if (staged) { // the block's bytes into LDS, 16 loads in flight a thread; 16 zero bytes of slack
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
            ok = tfz::huf_read(body + d.huf, d.huf_n, T, lane, 64) >= 0;
            lds_order();
            if (ok) {
                if (staged) ok = huf_lanes<true>(T, stage + (d.lit_at - d.src), d.lbytes, d.lsize, d.streams, lit, lane);
                else ok = huf_lanes<false>(T, body + d.lit_at, d.lbytes, d.lsize, d.streams, lit, lane);
            }
        }
    } else { // ---- sequences
        if (d.nseq) {
            bool built = true;
            if (lane == 0)
                for (int k = 0; k < 3; ++k) built = built && tfz::seq_table_build(T, k, d.tab[k], d.tab_n[k], body);
            lds_order();
            ok = __ballot(lane == 0 && !built) == 0;
        }
        if (ok) {
            if (staged) ok = seq_wave<true>(T, stage + (d.seq_at - d.src), d.seq_n, d, recs, lane);
            else ok = seq_wave<false>(T, body + d.seq_at, d.seq_n, d, recs, lane);
        }
    }
    if (lane == 0 && !ok) atomicOr(err, 1u);
}

// ---------------------------------------------------------------- resolve
// One wave per packet frame.  Records go 64 at a time (the next batch loaded while this one is
// resolved): scans give positions, the repeat offsets run through the 64 in order.  Records are
// rewritten as {pos, ll, lpos, off}.
__global__ void __launch_bounds__(64) zstd_resolve_kernel(const uint64_t *roff, uint64_t f0, const uint32_t *bases,
                                                          tfz::ZFrameDesc *frames, tfz::ZRec *recs, unsigned *err) {
    const uint32_t i = blockIdx.x, lane = threadIdx.x;
    const uint64_t f = f0 + i, raw = roff[f + 1] - roff[f];
    uint32_t pos = 0, lpos = (uint32_t)(roff[f] - roff[f0]);
    bool bad = false;
    for (uint32_t z = bases[4 * i + 1]; z < bases[4 * i + 5] && !bad; ++z) {
        tfz::ZFrameDesc fr = frames[z];
        const uint32_t zstart = pos;
        uint32_t r0 = 1, r1 = 4, r2 = 8;
        tfz::ZRec nxt{0, 0, tfz::ZDIRECT, 0};
        if (fr.rec0 + lane < fr.rec1) nxt = recs[fr.rec0 + lane];
        for (uint32_t q0 = fr.rec0; q0 < fr.rec1; q0 += 64) {
            const tfz::ZRec r = nxt;
            const uint32_t cnt = fr.rec1 - q0 < 64 ? fr.rec1 - q0 : 64;
            nxt = tfz::ZRec{0, 0, tfz::ZDIRECT, 0};
            if (q0 + 64 + lane < fr.rec1) nxt = recs[q0 + 64 + lane];
            const uint32_t ll = lane < cnt ? r.a : 0, ml = lane < cnt ? r.b : 0;
            uint64_t span = (uint64_t)ll + ml, incl = span;
            uint32_t linc = ll;
#pragma unroll
            for (int k = 1; k < 64; k <<= 1) {
                const uint64_t y = __shfl_up(incl, k, 64);
                const uint32_t w = __shfl_up(linc, k, 64);
                if (lane >= (uint32_t)k) {
                    incl += y;
                    linc += w;
                }
            }
            const uint64_t mypos = pos + incl - span;
            const uint32_t mylpos = lpos + linc - ll;
            uint32_t myoff = 0;
            for (uint32_t j = 0; j < cnt; ++j) {
                const uint32_t off = tfz::rep_resolve(rl32(r.c, j), rl32(r.a, j), r0, r1, r2);
                myoff = lane == j ? off : myoff;
            }
            if (lane < cnt) {
                if (ml && (myoff == 0 || (uint64_t)myoff > mypos + ll - zstart)) bad = true;
                if (mypos + span > raw) bad = true;
                recs[q0 + lane] = tfz::ZRec{(uint32_t)mypos, ll, mylpos, myoff};
            }
            const uint64_t tot = __shfl(incl, 63, 64);
            const uint32_t ltot = __shfl(linc, 63, 64);
            if (pos + tot > raw) {
                bad = true;
                break;
            }
            pos += (uint32_t)tot;
            lpos += ltot;
            bad = __ballot(bad) != 0;
            if (bad) break;
        }
        if (lane == 0) {
            frames[z].out0 = zstart;
            frames[z].out1 = pos;
        }
        if (fr.fcs != ~0ull && (uint64_t)(pos - zstart) != fr.fcs) bad = true;
    }
    if (pos != raw) bad = true;
    if (lane == 0 && bad) atomicOr(err, 1u);
}

// ---------------------------------------------------------------- execute
// One workgroup per ZCHUNK output bytes of a packet frame (cbase: prefix of the frames' chunk
// counts); 16 bytes a thread.  Literal bytes are written to `out`; src[g] = g for them, g - off
// for match bytes (g: launch-relative output index).
__global__ void __launch_bounds__(256) zstd_expand_kernel(const uint64_t *roff, uint64_t f0, uint32_t nf,
                                                          const uint32_t *cbase, const uint32_t *bases, const tfz::ZRec *recs,
                                                          const uint8_t *lits, uint64_t nlits, uint8_t *out, uint32_t *src,
                                                          unsigned *err) {
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
    if (s >= b1) return;
    const uint32_t e = s + 16 < b1 ? s + 16 : b1;
    uint32_t r = last_le(range[0], range[1], s);
    tfz::ZRec rec = recs[r];
    uint32_t end = r + 1 < r1 ? recs[r + 1].a : (uint32_t)raw;
    bool bad = false;
    for (uint32_t b = s; b < e; ++b) {
        while (b >= end && r + 1 < r1) {
            ++r;
            rec = recs[r];
            end = r + 1 < r1 ? recs[r + 1].a : (uint32_t)raw;
        }
        const uint64_t g = g0 + b;
        uint32_t sv = (uint32_t)g;
        if (b < rec.a) {
            bad = true; // inconsistent positions (a malformed frame)
        } else if (b - rec.a < rec.b) {
            const uint64_t li = (uint64_t)rec.c + (b - rec.a);
            if (li < nlits) out[g] = lits[li];
            else bad = true;
        } else if (rec.d == 0 || rec.d > b) {
            bad = true;
        } else {
            sv = (uint32_t)(g - rec.d);
        }
        src[g] = sv;
    }
    if (bad) atomicOr(err, 1u);
}

// One pointer-jumping round over src[0, n): src[g] = src[src[g]]; *flag = 1 while some byte
// still points at a byte that is not a literal.
__global__ void __launch_bounds__(256) zstd_jump_kernel(uint32_t *src, uint64_t n, unsigned *flag) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    bool more = false;
    if (g < n) {
        const uint32_t s = src[g];
        if (s != (uint32_t)g) {
            const uint32_t t = src[s];
            if (t != s) {
                src[g] = t;
                more = src[t] != t;
            }
        }
    }
    if (__ballot(more) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

__global__ void __launch_bounds__(256) zstd_gather_kernel(const uint32_t *src, uint64_t n, uint8_t *out) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g < n) {
        const uint32_t s = src[g];
        if (s != (uint32_t)g) out[g] = out[s];
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

struct PoolBuf { // hipMallocAsync'd, hipFreeAsync'd on every exit
    hipStream_t st;
    void *p = nullptr;
    uint64_t cap = 0;
    ~PoolBuf() {
        if (p) (void)hipFreeAsync(p, st);
    }
    int reserve(uint64_t bytes) {
        if (bytes <= cap) return TFG_OK;
        if (p) TFG_HIP(hipFreeAsync(p, st));
        p = nullptr;
        TFG_HIP(hipMallocAsync(&p, bytes, st));
        cap = bytes;
        return TFG_OK;
    }
};

} // namespace

int zstd_decode_frames(Ctx *ctx, const uint8_t *packet, uint64_t nf, const uint64_t *dfo, const uint64_t *dro,
                       const uint64_t *fo, const uint64_t *ro, uint8_t *dst, unsigned *err) {
    // ---- pass 1: counts of every frame (one read-back)
    PoolBuf cbuf{ctx->stream}, buf{ctx->stream};
    if (int rc = cbuf.reserve(nf * sizeof(tfz::ZCounts) + 256)) return rc;
    tfz::ZCounts *dcounts = (tfz::ZCounts *)cbuf.p;
    {
        ProfScope _ps(ctx, "codec.zstd.scan");
        hipLaunchKernelGGL(zstd_scan_kernel, dim3((unsigned)nf), dim3(64), 0, ctx->stream, packet, dfo, dro, (uint64_t)0,
                           dcounts, (const uint32_t *)nullptr, (tfz::ZBlockDesc *)nullptr, (tfz::ZFrameDesc *)nullptr, err);
        TFG_LAUNCH_CHECK();
    }
    std::vector<tfz::ZCounts> counts(nf);
    if (int rc = read_back_u64(ctx, (const uint64_t *)dcounts, (uint64_t *)counts.data(), nf * 2)) return rc;
    for (uint64_t f = 0; f < nf; ++f)
        TFG_CHECK(counts[f].blocks != tfz::ZNONE, TFG_ERR_INVALID_ARG, "corrupted ZSTD frame (Cannot decompress)");
    auto need = [&](uint64_t f) { // launch bytes of frame f: descriptors, records, literals, sources
        const uint64_t raw = ro[f + 1] - ro[f];
        return (uint64_t)counts[f].blocks * sizeof(tfz::ZBlockDesc) + (uint64_t)counts[f].frames * sizeof(tfz::ZFrameDesc) +
               (uint64_t)counts[f].recs * sizeof(tfz::ZRec) + raw * 5 + 64;
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
        const size_t o_cb = cv.take<uint32_t>(cbase.size()), o_flag = cv.take<uint64_t>(1);
        if (int rc = buf.reserve(cv.off)) return rc;
        char *sb = (char *)buf.p;
        tfz::ZBlockDesc *blk = (tfz::ZBlockDesc *)(sb + o_blk);
        tfz::ZFrameDesc *frm = (tfz::ZFrameDesc *)(sb + o_frm);
        tfz::ZRec *rec = (tfz::ZRec *)(sb + o_rec);
        uint8_t *lit = (uint8_t *)(sb + o_lit);
        uint32_t *src = (uint32_t *)(sb + o_src), *dbases = (uint32_t *)(sb + o_bas), *dcb = (uint32_t *)(sb + o_cb);
        unsigned *flag = (unsigned *)(sb + o_flag);
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
                const size_t lds = ((sizeof(tfz::ZTables) + 15) & ~size_t(15)) + cap + 16;
                hipLaunchKernelGGL(zstd_block_kernel, dim3(nb), dim3(128), lds, ctx->stream, packet, dfo, a,
                                   (const tfz::ZBlockDesc *)blk, lit, rec, cap, err);
                TFG_LAUNCH_CHECK();
            }
            hipLaunchKernelGGL(zstd_resolve_kernel, dim3((unsigned)g), dim3(64), 0, ctx->stream, dro, a,
                               (const uint32_t *)dbases, frm, rec, err);
            TFG_LAUNCH_CHECK();
            if (nc) {
                hipLaunchKernelGGL(zstd_expand_kernel, dim3(nc), dim3(256), 0, ctx->stream, dro, a, (uint32_t)g,
                                   (const uint32_t *)dcb, (const uint32_t *)dbases, (const tfz::ZRec *)rec,
                                   (const uint8_t *)lit, raw, out, src, err);
                TFG_LAUNCH_CHECK();
            }
        }
        const unsigned jg = (unsigned)((raw + 255) / 256);
        if (raw) {
            int round = 0;
            for (;; ++round) {
                TFG_CHECK(round < ZMAX_ROUNDS, TFG_ERR_INVALID_ARG, "corrupted ZSTD frame (Cannot decompress)");
                TFG_HIP(hipMemsetAsync(flag, 0, sizeof(unsigned), ctx->stream));
                {
                    ProfScope _ps(ctx, "codec.zstd.decompress");
                    hipLaunchKernelGGL(zstd_jump_kernel, dim3(jg), dim3(256), 0, ctx->stream, src, raw, flag);
                    TFG_LAUNCH_CHECK();
                }
                uint64_t more = 0;
                TFG_HIP(hipMemcpyAsync(ctx->host_pinned, flag, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
                TFG_HIP(hipStreamSynchronize(ctx->stream));
                more = *(const unsigned *)ctx->host_pinned;
                if (!more) break;
            }
            ProfScope _ps(ctx, "codec.zstd.decompress");
            hipLaunchKernelGGL(zstd_gather_kernel, dim3(jg), dim3(256), 0, ctx->stream, (const uint32_t *)src, raw, out);
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
