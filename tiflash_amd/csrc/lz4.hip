// lz4.hip — LZ4-compressed MPP packets (§8 f1): CHBlockChunkCodecV1 with CompressionMethod::LZ4.
//
// Reference framing: CHBlockChunkCodecV1::encode (Flash/Coprocessor/CHBlockChunkCodecV1.cpp:
// 391-429, 555-565) writes the packet body (header + columns, i.e. the NONE packet without its
// 0x02 byte) through CompressedCHBlockChunkWriteBuffer = CompressedWriteBuffer<false>, and
// decode (:567-581) reads it back through CompressedReadBuffer<false>: a sequence of frames
//     0x82 | UInt32 frame bytes (9-byte header included) | UInt32 raw bytes | LZ4 block
// (IO/Compression/CompressionInfo.h: COMPRESSED_BLOCK_HEADER_SIZE = 9, CompressionMethodByte::LZ4
// = 0x82; no CityHash checksum in the <false> instantiation).  The LZ4 block is the published
// LZ4 block format (lz4 1.9.x, lz4_Block_format.md; the library is a third-party dependency of
// the reference, not vendored under /root/reference): sequences of a token (literal length << 4
// | match length - 4), 255-step length extensions, the literals, a 2-byte little-endian offset;
// the last 5 bytes of a block are literals and the last match starts at least 12 bytes before
// the end.  Any LZ4 encoder's frames decode here; the reference writes one frame per packet (the
// write buffer is sized to the whole packet), this encoder writes 64 KB frames so that frames
// compress and decompress in parallel — the reference's CompressedReadBuffer reads either.
//
// GPU design: one wave per frame for both directions, control flow uniform across the wave.
//  * encode: 64 positions per step, one a lane: each lane hashes the 4 bytes at its position and
//    reads its slot of a single-probe hash table ({position, sequence} entries in LDS, so a
//    candidate is verified without a global load); the candidates are taken greedily in order,
//    match extension compares 64 bytes per step with a ballot; the chunk's positions outside its
//    matches then enter the table (sparser after chunks without a match, as LZ4's skip
//    acceleration); literals are copied by all lanes.
//  * decode: the token stream goes through the same register window; literal runs are copied by
//    all lanes; a match copies lane i's byte from out[start - offset + i % offset], bytes written
//    before the match began (other lanes' stores are drained and the loads bypass the L1).
//  * the frame table of a packet comes from one thread walking the 9-byte headers.
#include "common.h"
#include "codec_zstd.h"

namespace tfg {
namespace {

constexpr uint8_t LZ4_METHOD = 0x82;       // CompressionMethodByte::LZ4
constexpr uint8_t ZSTD_METHOD = 0x90;      // CompressionMethodByte::ZSTD (zstd_dec.h)
constexpr uint8_t NONE_METHOD = 0x02;      // CompressionMethodByte::NONE
constexpr int FRAME_HDR = 9;               // COMPRESSED_BLOCK_HEADER_SIZE
constexpr uint64_t MAX_FRAME_RAW = 0x40000000ull; // DBMS_MAX_COMPRESSED_SIZE
constexpr uint32_t ENC_FRAME = 64 * 1024;  // raw bytes per frame this encoder writes
// match-finder table: 2^HASH_LOG x 6 B of LDS per frame.  Measured on 256 MB of k%08d rows
// (tools/lz4_probe.py) with the serial matcher (one position a step): 12 bits 8.6 GB/s at ratio
// 1.371, 11 bits 12.1 GB/s at 1.320, 10 bits 17.8 GB/s at 1.266; with 64 positions a step: 11
// bits 23.6 GB/s at 1.320, 10 bits 38.9 GB/s at 1.267 (6 KB: every frame of 256 MB resident).
#ifndef TFG_LZ4_HASH_LOG
#define TFG_LZ4_HASH_LOG 10
#endif
constexpr int HASH_LOG = TFG_LZ4_HASH_LOG;
constexpr uint64_t ENC_SLOT = FRAME_HDR + ENC_FRAME + ENC_FRAME / 255 + 16; // header + LZ4_COMPRESSBOUND
constexpr int MIN_MATCH = 4, LAST_LITERALS = 5, MF_LIMIT = 12;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Register window over a byte stream: lane l holds src[base + l] (0 past `end`).
struct Window {
    const uint8_t *src;
    uint64_t end;
    uint64_t base = ~0ull;
    uint32_t v = 0;
    __device__ __forceinline__ void load(uint64_t p) {
        base = p;
        const uint64_t q = p + lane_id();
        v = q < end ? src[q] : 0u;
    }
    // byte at p (p uniform); reloads when p is outside the window
    __device__ __forceinline__ uint32_t byte(uint64_t p) {
        if (p < base || p >= base + 64) load(p);
        return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(p - base));
    }
    // 4 bytes at p, little-endian
    __device__ __forceinline__ uint32_t word(uint64_t p) {
        if (p < base || p + 4 > base + 64) load(p);
        const int r = (int)(p - base);
        return (uint32_t)__builtin_amdgcn_readlane((int)v, r) | ((uint32_t)__builtin_amdgcn_readlane((int)v, r + 1) << 8) |
               ((uint32_t)__builtin_amdgcn_readlane((int)v, r + 2) << 16) |
               ((uint32_t)__builtin_amdgcn_readlane((int)v, r + 3) << 24);
    }
};

// One wave (= one workgroup) per frame.  Writes the frame (header + block) to out + f * ENC_SLOT
// and its size to sizes[f].
__global__ void __launch_bounds__(64) lz4_encode_kernel(const uint8_t *src, uint64_t n, uint64_t nframes, uint8_t *out,
                                                        uint32_t *sizes) {
    __shared__ uint16_t tpos[1 << HASH_LOG];
    __shared__ uint32_t tseq[1 << HASH_LOG];
    const uint64_t f = blockIdx.x;
    if (f >= nframes) return;
    const uint32_t lane = lane_id();
    for (int i = lane; i < (1 << HASH_LOG); i += 64) {
        tpos[i] = 0xFFFF; // empty: never below a cursor position (those stay under 65524)
        tseq[i] = 0;
    }
    __syncthreads();
    const uint8_t *s = src + f * ENC_FRAME;
    const uint32_t len = (uint32_t)min<uint64_t>(ENC_FRAME, n - f * ENC_FRAME);
    uint8_t *frame = out + f * ENC_SLOT;
    uint8_t *o = frame + FRAME_HDR;
    uint32_t op = 0; // uniform output cursor
    auto put_len = [&](uint32_t v) __attribute__((always_inline)) { // extension of a length field at 15
        v -= 15;
        while (v >= 255) {
            if (lane == 0) o[op] = 255;
            ++op;
            v -= 255;
        }
        if (lane == 0) o[op] = (uint8_t)v;
        ++op;
    };
    // literals [anchor, lit_end) followed by a match (ml == 0: the last sequence)
    auto emit = [&](uint32_t anchor, uint32_t lit_end, uint32_t off, uint32_t ml) __attribute__((always_inline)) {
        const uint32_t lit = lit_end - anchor;
        const uint32_t mcode = ml ? ml - MIN_MATCH : 0;
        if (lane == 0) o[op] = (uint8_t)((min(lit, 15u) << 4) | min(mcode, 15u));
        ++op;
        if (lit >= 15) put_len(lit);
        for (uint32_t i = lane; i < lit; i += 64) o[op + i] = s[anchor + i];
        op += lit;
        if (!ml) return;
        if (lane == 0) {
            o[op] = (uint8_t)off;
            o[op + 1] = (uint8_t)(off >> 8);
        }
        op += 2;
        if (mcode >= 15) put_len(mcode);
    };
    uint32_t anchor = 0;
    if (len >= MF_LIMIT + 1) {
        // 64 positions per step, one a lane (as the ZSTD sender, zstd_enc.hip): every lane hashes
        // the 4 bytes at its position and reads its table slot at once; the verified candidates
        // are taken in order, each extended 64 bytes per step by a ballot; then the chunk's
        // positions outside its matches enter the table (every stride-th after chunks without
        // a match, so incompressible stretches keep older entries)
        const uint32_t mflimit = len - MF_LIMIT, matchlimit = len - LAST_LITERALS;
        uint32_t ip = 0, dry = 0;
        for (uint32_t cbase = 0; cbase < mflimit;) {
            const uint32_t pos = cbase + lane, ip0 = ip;
            const bool valid = pos < mflimit;
            uint32_t w = 0;
            if (valid) w = (uint32_t)s[pos] | ((uint32_t)s[pos + 1] << 8) | ((uint32_t)s[pos + 2] << 16) | ((uint32_t)s[pos + 3] << 24);
            const uint32_t h = (w * 2654435761u) >> (32 - HASH_LOG);
            const uint32_t ref = tpos[h], rw = tseq[h];
            uint64_t mask = __ballot(valid && pos >= ip && ref < pos && rw == w), covered = 0;
            while (mask) {
                const uint32_t j = (uint32_t)__builtin_ctzll(mask);
                const uint32_t at = cbase + j, from = (uint32_t)__builtin_amdgcn_readlane((int)ref, (int)j);
                uint32_t ml = MIN_MATCH;
                for (;;) { // extend 64 bytes per step
                    const uint32_t x = at + ml + lane;
                    const bool eq = x < matchlimit && s[from + ml + lane] == s[x];
                    const uint64_t neq = ~__ballot(eq);
                    if (neq == 0) {
                        ml += 64;
                        continue;
                    }
                    ml += (uint32_t)__builtin_ctzll(neq);
                    break;
                }
                emit(anchor, at, at - from, ml);
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
            dry = ip > ip0 ? 0 : dry + 1;
            const uint32_t stride = 1u << min(6u, dry >> 1);
            __builtin_amdgcn_wave_barrier();
            if (valid && !((covered >> lane) & 1) && (pos & (stride - 1)) == 0) { // one of a slot's lanes wins
                tpos[h] = (uint16_t)pos;
                tseq[h] = w;
            }
            __builtin_amdgcn_wave_barrier();
            cbase = max(cbase + 64, ip);
        }
    }
    emit(anchor, len, 0, 0); // last literals
    const uint32_t fbytes = FRAME_HDR + op;
    if (lane == 0) frame[0] = LZ4_METHOD;
    if (lane < 4) {
        frame[1 + lane] = (uint8_t)(fbytes >> (8 * lane));
        frame[5 + lane] = (uint8_t)(len >> (8 * lane));
    }
    if (lane == 0) sizes[f] = fbytes;
}

// exclusive prefix of the frame sizes (nframes is small: one thread)
__global__ void lz4_offsets_kernel(const uint32_t *sizes, uint64_t nframes, uint64_t *offs) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t acc = 0;
    for (uint64_t f = 0; f < nframes; ++f) {
        offs[f] = acc;
        acc += sizes[f];
    }
    offs[nframes] = acc;
}

// frame f's bytes -> dst + offs[f]
__global__ void lz4_pack_kernel(const uint8_t *frames, uint64_t slot, const uint32_t *sizes, const uint64_t *offs,
                                uint64_t nframes, uint8_t *dst) {
    const uint64_t f = blockIdx.x;
    if (f >= nframes) return;
    const uint8_t *s = frames + f * slot;
    const uint32_t sz = sizes[f];
    uint8_t *d = dst + offs[f];
    for (uint32_t i = threadIdx.x; i < sz; i += blockDim.x) d[i] = s[i];
}

// one thread walks the frame headers: foff / roff get frame and raw offsets (exclusive sums, up
// to max_frames entries); out = {frames, raw bytes, malformed}
__global__ void lz4_frames_kernel(const uint8_t *pkt, uint64_t bytes, uint8_t method, uint64_t *foff, uint64_t *roff,
                                  uint64_t max_frames, uint64_t *out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t pos = 0, raw = 0, k = 0, bad = 0;
    while (pos < bytes) {
        if (pos + FRAME_HDR > bytes || pkt[pos] != method) {
            bad = 1;
            break;
        }
        uint32_t fb = 0, rb = 0;
        for (int b = 0; b < 4; ++b) {
            fb |= (uint32_t)pkt[pos + 1 + b] << (8 * b);
            rb |= (uint32_t)pkt[pos + 5 + b] << (8 * b);
        }
        // a frame may not claim more raw bytes than its codec can expand its block to (LZ4: one
        // token byte yields at most 255 + 16 raw bytes; ZSTD: a 4-byte RLE block 128 KB), nor
        // more than DBMS_MAX_COMPRESSED_SIZE (IO/Compression/CompressionInfo.h:21), so a forged
        // header cannot size the output
        const uint64_t expand = method == LZ4_METHOD ? 255 : 32768;
        if (fb <= FRAME_HDR || pos + fb > bytes || rb > MAX_FRAME_RAW ||
            (uint64_t)rb > (uint64_t)(fb - FRAME_HDR) * expand + 16) {
            bad = 1;
            break;
        }
        if (k < max_frames) {
            foff[k] = pos;
            roff[k] = raw;
        }
        ++k;
        pos += fb;
        raw += rb;
    }
    if (k <= max_frames) {
        foff[k] = pos;
        roff[k] = raw;
    }
    out[0] = k;
    out[1] = raw;
    out[2] = bad;
}

// One wave per frame: decodes the LZ4 block of frame f into dst + roff[f].  err |= 1 when the
// block is malformed or does not produce exactly its declared raw size (the checks of
// LZ4_decompress_safe and of the codec's decompressed-size comparison).
__global__ void __launch_bounds__(64) lz4_decode_kernel(const uint8_t *pkt, const uint64_t *foff, const uint64_t *roff,
                                                        uint64_t nframes, uint8_t *dst, unsigned *err) {
    const uint64_t f = blockIdx.x;
    if (f >= nframes) return;
    const uint32_t lane = lane_id();
    const uint8_t *s = pkt + foff[f];
    const uint64_t src_end = foff[f + 1] - foff[f];
    const uint64_t raw = roff[f + 1] - roff[f];
    uint8_t *o = dst + roff[f];
    volatile const uint8_t *ov = o; // L1-bypassing reads of bytes other lanes wrote
    Window win{s, src_end};
    uint64_t ip = FRAME_HDR, op = 0;
    bool bad = false;
    auto ext = [&](uint64_t &v) __attribute__((always_inline)) { // 255-step extension
        uint32_t b;
        do {
            if (ip >= src_end) {
                bad = true;
                return;
            }
            b = win.byte(ip++);
            v += b;
        } while (b == 255);
    };
    while (!bad) {
        if (ip >= src_end) {
            bad = true; // a block ends with a literal-only sequence, never between sequences
            break;
        }
        const uint32_t token = win.byte(ip++);
        uint64_t lit = token >> 4;
        if (lit == 15) ext(lit);
        if (bad || ip + lit > src_end || op + lit > raw) {
            bad = true;
            break;
        }
        for (uint64_t i = lane; i < lit; i += 64) o[op + i] = s[ip + i];
        ip += lit;
        op += lit;
        if (ip == src_end) break; // the last sequence: literals only
        if (ip + 2 > src_end) {
            bad = true;
            break;
        }
        const uint32_t off = win.byte(ip) | (win.byte(ip + 1) << 8);
        ip += 2;
        uint64_t ml = (token & 15) + MIN_MATCH;
        if ((token & 15) == 15) ext(ml);
        if (bad || off == 0 || off > op || op + ml > raw) {
            bad = true;
            break;
        }
        // every lane's earlier stores have completed before any lane reads them back
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        if (off >= ml) { // no overlap: a straight copy of bytes written before this match
            for (uint64_t i = lane; i < ml; i += 64) o[op + i] = ov[op - off + i];
        } else { // overlapping: the off-byte pattern repeats (frame raw sizes fit 32 bits)
            const uint32_t ml32 = (uint32_t)ml;
            for (uint32_t i = lane; i < ml32; i += 64) o[op + i] = ov[op - off + (i % off)];
        }
        op += ml;
    }
    if (lane == 0 && (bad || op != raw)) atomicOr(err, 1u);
}

// ---- the frame table in parallel: the packet in 64 KB segments, one wave each, finds the first
// plausible frame start of its segment (two chained headers with sane sizes, then the method byte
// again) and walks the frames from there past its end; a second
// kernel keeps the segments the true chain runs through — entering position = the prefix max of
// the earlier segments' exits, a segment in use must have started exactly there — and writes the
// table. Any disagreement, a malformed header or more than FSEG_CAP frames in a segment makes the
// host run lz4_frames_kernel instead (which also gives malformed packets their error).
constexpr uint64_t FSEG = 64 * 1024;
constexpr uint32_t FSEG_CAP = 256; // a 64 KB frame of one repeated byte compresses to ~270 B
struct FSeg {
    uint64_t first, exit, raw;
    uint32_t n, flags; // flags: 1 = a start was found, 2 = give up (bad header / overflow)
};

__device__ __forceinline__ uint32_t pkt_u32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
// the serial walk's header checks at pos (frame bytes / raw bytes out)
__device__ __forceinline__ bool frame_ok(const uint8_t *pkt, uint64_t bytes, uint8_t method, uint64_t pos, uint32_t &fb,
                                         uint32_t &rb) {
    if (pos + FRAME_HDR > bytes || pkt[pos] != method) return false;
    fb = pkt_u32(pkt + pos + 1);
    rb = pkt_u32(pkt + pos + 5);
    const uint64_t expand = method == LZ4_METHOD ? 255 : 32768;
    return fb > FRAME_HDR && pos + fb <= bytes && rb <= MAX_FRAME_RAW &&
           (uint64_t)rb <= (uint64_t)(fb - FRAME_HDR) * expand + 16;
}

__global__ void __launch_bounds__(64) frames_seg_kernel(const uint8_t *pkt, uint64_t bytes, uint8_t method, uint64_t nseg,
                                                        FSeg *seg, uint64_t *sfo, uint32_t *srb) {
    const uint64_t g = blockIdx.x;
    if (g >= nseg) return;
    const uint32_t lane = __lane_id();
    const uint64_t s0 = g * FSEG, s1 = min(bytes, s0 + FSEG);
    uint64_t first = g == 0 ? 0 : ~0ull;
    for (uint64_t base = s0; g > 0 && base < s1; base += 64 * 16) {
        const uint64_t q0 = base + lane * 16;
        uint64_t found = ~0ull;
        for (uint32_t b = 0; b < 16 && q0 + b < s1; ++b) {
            const uint64_t q = q0 + b;
            uint32_t fb, rb, fb2, rb2;
            // two chained headers, then the method byte (or the end): a false start inside
            // compressed bytes passes one header check about once per few MB, not two
            if (pkt[q] == method && frame_ok(pkt, bytes, method, q, fb, rb) &&
                (q + fb == bytes || (frame_ok(pkt, bytes, method, q + fb, fb2, rb2) &&
                                     (q + fb + fb2 == bytes || pkt[q + fb + fb2] == method)))) {
                found = q;
                break;
            }
        }
        const uint64_t any = __ballot(found != ~0ull);
        if (any) {
            first = (uint64_t)__shfl((long long)found, (int)__builtin_ctzll(any), 64);
            break;
        }
    }
    FSeg out{first, 0, 0, 0, 0};
    if (first != ~0ull) {
        out.flags = 1;
        uint64_t pos = first;
        while (pos < s1) {
            uint32_t fb, rb;
            if (!frame_ok(pkt, bytes, method, pos, fb, rb) || out.n >= FSEG_CAP) {
                out.flags |= 2;
                break;
            }
            if (lane == 0) {
                sfo[g * FSEG_CAP + out.n] = pos;
                srb[g * FSEG_CAP + out.n] = rb;
            }
            ++out.n;
            out.raw += rb;
            pos += fb;
        }
        out.exit = pos;
    }
    if (lane == 0) seg[g] = out;
}

// one 1024-thread workgroup; out = {frames, raw bytes, 0, fall back to the serial walk}
__global__ void __launch_bounds__(1024) frames_join_kernel(const FSeg *seg, const uint64_t *sfo, const uint32_t *srb,
                                                           uint64_t nseg, uint64_t bytes, uint64_t *foff, uint64_t *roff,
                                                           uint64_t max_frames, uint64_t *out) {
    __shared__ uint64_t a[1024], b[1024], c[1024];
    __shared__ uint64_t carry_ent, carry_k, carry_raw;
    __shared__ int fail;
    const uint32_t t = threadIdx.x;
    if (t == 0) {
        carry_ent = 0;
        carry_k = 0;
        carry_raw = 0;
        fail = 0;
    }
    __syncthreads();
    for (uint64_t c0 = 0; c0 < nseg; c0 += 1024) {
        const uint64_t g = c0 + t;
        const bool in = g < nseg;
        FSeg sg{};
        if (in) sg = seg[g];
        // exclusive prefix max of the exits (segments without a start exit at 0)
        a[t] = in && (sg.flags & 1) ? sg.exit : 0;
        __syncthreads();
        for (uint32_t d = 1; d < 1024; d <<= 1) {
            const uint64_t v = t >= d ? a[t - d] : 0;
            __syncthreads();
            a[t] = max(a[t], v);
            __syncthreads();
        }
        const uint64_t ent = max(carry_ent, t ? a[t - 1] : 0);
        const uint64_t s1 = min(bytes, g * FSEG + FSEG);
        const bool used = in && ent < s1;
        if (in && (sg.flags & 2)) fail = 1;
        if (used && sg.first != ent) fail = 1;                     // started somewhere else
        if (in && !used && (sg.flags & 1) && sg.exit > ent) fail = 1; // a false start ran past the chain
        b[t] = used ? sg.n : 0;
        c[t] = used ? sg.raw : 0;
        __syncthreads();
        for (uint32_t d = 1; d < 1024; d <<= 1) { // inclusive prefix sums
            const uint64_t vb = t >= d ? b[t - d] : 0, vc = t >= d ? c[t - d] : 0;
            __syncthreads();
            b[t] += vb;
            c[t] += vc;
            __syncthreads();
        }
        if (used) {
            uint64_t k = carry_k + b[t] - sg.n, r = carry_raw + c[t] - sg.raw;
            for (uint32_t i = 0; i < sg.n; ++i, ++k) {
                if (k < max_frames) {
                    foff[k] = sfo[g * FSEG_CAP + i];
                    roff[k] = r;
                }
                r += srb[g * FSEG_CAP + i];
            }
        }
        __syncthreads();
        if (t == 1023) {
            carry_ent = max(carry_ent, a[1023]);
            carry_k += b[1023];
            carry_raw += c[1023];
        }
        __syncthreads();
    }
    if (t == 0) {
        const uint64_t k = carry_k;
        const bool ok = !fail && carry_ent == bytes;
        if (ok && k <= max_frames) {
            foff[k] = bytes;
            roff[k] = carry_raw;
        }
        out[0] = k;
        out[1] = carry_raw;
        out[2] = 0;
        out[3] = ok ? 0 : 1;
    }
}

int read_method(Ctx *ctx, const uint8_t *packet, uint8_t *m) {
    TFG_HIP(hipMemcpyAsync(ctx->host_pinned, packet, 1, hipMemcpyDeviceToHost, ctx->stream));
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    *m = *(const uint8_t *)ctx->host_pinned;
    return TFG_OK;
}

} // namespace
} // namespace tfg

using namespace tfg;

extern "C" {

size_t tfg_codec_compress_bound(size_t bytes) {
    if (bytes <= 1) return 0;
    const uint64_t n = bytes - 1, nframes = (n + ENC_FRAME - 1) / ENC_FRAME;
    return (size_t)(nframes * (uint64_t)(FRAME_HDR + 16) + n + n / 255);
}

int tfg_codec_compress(tfg_ctx *ctx, int method, const uint8_t *packet, size_t bytes, uint8_t *out, size_t capacity,
                       size_t *out_bytes_host) {
    TFG_CHECK(ctx && out_bytes_host && (bytes == 0 || packet), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(method == TFG_COMPRESSION_LZ4 || method == TFG_COMPRESSION_LZ4HC || method == TFG_COMPRESSION_ZSTD,
              TFG_ERR_NOT_IMPLEMENTED, "compression method %d: LZ4 / LZ4HC / ZSTD", method);
    if (int rc = set_device(ctx)) return rc;
    *out_bytes_host = 0;
    if (bytes == 0) return TFG_OK; // the empty Block: no packet body
    uint8_t m = 0;
    if (int rc = read_method(ctx, packet, &m)) return rc;
    TFG_CHECK(m == NONE_METHOD, TFG_ERR_INVALID_ARG, "not an uncompressed V1 packet (method byte 0x%02x)", m);
    if (bytes == 1) return TFG_OK;
    if (!out) {
        *out_bytes_host = tfg_codec_compress_bound(bytes);
        return TFG_OK;
    }
    const uint8_t *body = packet + 1;
    static_assert(ZE_FRAME == ENC_FRAME, "both senders frame the body in 64 KB units");
    const bool zstd = method == TFG_COMPRESSION_ZSTD;
    const uint64_t n = bytes - 1, nframes = (n + ENC_FRAME - 1) / ENC_FRAME;
    const uint64_t slot = zstd ? ZE_SLOT : ENC_SLOT;
    TFG_CHECK(nframes < (1ull << 31), TFG_ERR_INVALID_ARG, "packet of %llu bytes", (unsigned long long)bytes);
    Carver cv;
    const size_t o_frames = cv.take<uint8_t>(nframes * slot), o_sizes = cv.take<uint32_t>(nframes);
    const size_t o_offs = cv.take<uint64_t>(nframes + 1);
    const size_t o_tmp = cv.take<uint8_t>(zstd ? zstd_encode_tmp_bytes(nframes) : 0);
    void *sp;
    if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
    char *sb = (char *)sp;
    uint8_t *frames = (uint8_t *)(sb + o_frames);
    uint32_t *sizes = (uint32_t *)(sb + o_sizes);
    uint64_t *offs = (uint64_t *)(sb + o_offs);
    if (zstd) {
        if (int rc = zstd_encode_frames(ctx, body, n, nframes, frames, sizes, sb + o_tmp)) return rc;
    } else {
        ProfScope _ps(ctx, "codec.lz4.compress");
        hipLaunchKernelGGL(lz4_encode_kernel, dim3((unsigned)nframes), dim3(64), 0, ctx->stream, body, n, nframes, frames,
                           sizes);
        TFG_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(lz4_offsets_kernel, dim3(1), dim3(64), 0, ctx->stream, (const uint32_t *)sizes, nframes, offs);
    TFG_LAUNCH_CHECK();
    uint64_t total = 0;
    if (int rc = read_back_u64(ctx, offs + nframes, &total, 1)) return rc;
    *out_bytes_host = total;
    TFG_CHECK(capacity >= total, TFG_ERR_CAPACITY, "compressed packet needs %llu bytes, capacity %llu",
              (unsigned long long)total, (unsigned long long)capacity);
    hipLaunchKernelGGL(lz4_pack_kernel, dim3((unsigned)nframes), dim3(256), 0, ctx->stream, (const uint8_t *)frames, slot,
                       (const uint32_t *)sizes, (const uint64_t *)offs, nframes, out);
    TFG_LAUNCH_CHECK();
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    return TFG_OK;
}

int tfg_codec_decompress(tfg_ctx *ctx, const uint8_t *packet, size_t bytes, uint8_t *out, size_t capacity,
                         size_t *out_bytes_host) {
    TFG_CHECK(ctx && out_bytes_host && (bytes == 0 || packet), TFG_ERR_INVALID_ARG, "null argument");
    if (int rc = set_device(ctx)) return rc;
    *out_bytes_host = 0;
    if (bytes == 0) return TFG_OK;
    uint8_t m = 0;
    if (int rc = read_method(ctx, packet, &m)) return rc;
    TFG_CHECK(m == LZ4_METHOD || m == ZSTD_METHOD, m == NONE_METHOD ? TFG_ERR_INVALID_ARG : TFG_ERR_NOT_IMPLEMENTED,
              "method byte 0x%02x: only LZ4 and ZSTD frames decompress", m);
    uint64_t max_frames = bytes / (ENC_SLOT / 4) + 16; // grown below when the packet has more
    uint64_t res[3] = {0, 0, 0};
    char *sb = nullptr;
    size_t o_foff = 0, o_roff = 0;
    const uint64_t nseg = (bytes + FSEG - 1) / FSEG;
    const bool parallel = nseg >= 4 && nseg < (1ull << 31);
    for (int attempt = 0; attempt < 2; ++attempt) {
        Carver cv;
        o_foff = cv.take<uint64_t>(max_frames + 1);
        o_roff = cv.take<uint64_t>(max_frames + 1);
        const size_t o_res = cv.take<uint64_t>(4);
        const size_t o_seg = cv.take<FSeg>(parallel ? nseg : 0), o_sfo = cv.take<uint64_t>(parallel ? nseg * FSEG_CAP : 0);
        const size_t o_srb = cv.take<uint32_t>(parallel ? nseg * FSEG_CAP : 0);
        void *sp;
        if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
        sb = (char *)sp;
        uint64_t *dres = (uint64_t *)(sb + o_res);
        bool serial = !parallel;
        if (parallel) { // the segmented parse; the serial walk when it does not agree with itself
            ProfScope _ps(ctx, "codec.frames");
            hipLaunchKernelGGL(frames_seg_kernel, dim3((unsigned)nseg), dim3(64), 0, ctx->stream, packet, (uint64_t)bytes, m,
                               nseg, (FSeg *)(sb + o_seg), (uint64_t *)(sb + o_sfo), (uint32_t *)(sb + o_srb));
            TFG_LAUNCH_CHECK();
            hipLaunchKernelGGL(frames_join_kernel, dim3(1), dim3(1024), 0, ctx->stream, (const FSeg *)(sb + o_seg),
                               (const uint64_t *)(sb + o_sfo), (const uint32_t *)(sb + o_srb), nseg, (uint64_t)bytes,
                               (uint64_t *)(sb + o_foff), (uint64_t *)(sb + o_roff), max_frames, dres);
            TFG_LAUNCH_CHECK();
            uint64_t r4[4] = {0, 0, 0, 0};
            if (int rc = read_back_u64(ctx, dres, r4, 4)) return rc;
            serial = r4[3] != 0;
            for (int q = 0; q < 3; ++q) res[q] = r4[q];
        }
        if (serial) {
            hipLaunchKernelGGL(lz4_frames_kernel, dim3(1), dim3(64), 0, ctx->stream, packet, (uint64_t)bytes, m,
                               (uint64_t *)(sb + o_foff), (uint64_t *)(sb + o_roff), max_frames, dres);
            TFG_LAUNCH_CHECK();
            if (int rc = read_back_u64(ctx, dres, res, 3)) return rc;
        }
        TFG_CHECK(!res[2], TFG_ERR_INVALID_ARG, "malformed %s packet (frame headers)", m == LZ4_METHOD ? "LZ4" : "ZSTD");
        if (res[0] <= max_frames) break;
        max_frames = res[0];
    }
    TFG_CHECK(res[0] <= max_frames && res[0] < (1ull << 31), TFG_ERR_LOGICAL, "frame table of %llu frames",
              (unsigned long long)res[0]);
    *out_bytes_host = res[1] + 1; // the NONE method byte + the raw body
    if (!out) return TFG_OK;
    TFG_CHECK(capacity >= res[1] + 1, TFG_ERR_CAPACITY, "decompressed packet needs %llu bytes, capacity %llu",
              (unsigned long long)(res[1] + 1), (unsigned long long)capacity);
    TFG_HIP(hipMemsetAsync(out, NONE_METHOD, 1, ctx->stream));
    unsigned *err = (unsigned *)ctx->dev_counter;
    TFG_HIP(hipMemsetAsync(err, 0, sizeof(unsigned), ctx->stream));
    if (res[0] && m == ZSTD_METHOD) {
        // zstd.hip: scan, per-block entropy, resolve, parallel execution (frame tables read once)
        const uint64_t nf = res[0];
        std::vector<uint64_t> fo(nf + 1), ro(nf + 1);
        TFG_HIP(hipMemcpyAsync(fo.data(), sb + o_foff, (nf + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
        TFG_HIP(hipMemcpyAsync(ro.data(), sb + o_roff, (nf + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
        if (int rc = zstd_decode_frames(ctx, packet, nf, (const uint64_t *)(sb + o_foff), (const uint64_t *)(sb + o_roff),
                                        fo.data(), ro.data(), out + 1, err))
            return rc;
        TFG_HIP(hipMemcpyAsync(ctx->host_pinned, err, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
    } else if (res[0]) {
        ProfScope _ps(ctx, "codec.lz4.decompress");
        hipLaunchKernelGGL(lz4_decode_kernel, dim3((unsigned)res[0]), dim3(64), 0, ctx->stream, packet,
                           (const uint64_t *)(sb + o_foff), (const uint64_t *)(sb + o_roff), res[0], out + 1, err);
        TFG_LAUNCH_CHECK();
        TFG_HIP(hipMemcpyAsync(ctx->host_pinned, err, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
    } else {
        TFG_HIP(hipMemcpyAsync(ctx->host_pinned, err, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
    }
    const unsigned e = *(const unsigned *)ctx->host_pinned;
    TFG_CHECK(!e, TFG_ERR_INVALID_ARG, "corrupted %s frame (Cannot decompress)", m == LZ4_METHOD ? "LZ4" : "ZSTD");
    return TFG_OK;
}

} // extern "C"
