// codec.hip — the MPP wire format of Blocks (§8 f1): CHBlockChunkCodec and CHBlockChunkCodecV1
// (compression NONE), encoded from and decoded into device-resident columns.
//
// Reference: CHBlockChunkCodecStream::encode / CHBlockChunkCodec::decodeImpl
// (Flash/Coprocessor/CHBlockChunkCodec.cpp:134-208), EncodeHeader / DecodeHeader /
// decodeColumnsByBlock and the V1 packet layout (Flash/Coprocessor/CHBlockChunkCodecV1.cpp:45-147,
// 370-432, 567-583), the bulk serialisations of the column types: DataTypeNumberBase
// (DataTypes/DataTypeNumberBase.cpp:220-245), DataTypeDecimal (DataTypes/DataTypeDecimal.cpp:93-125),
// DataTypeNullable (null map, then the nested data: DataTypes/DataTypeNullable.cpp:66-117),
// DataTypeString legacy size-prefixed rows (DataTypes/DataTypeString.cpp:93-232) and StringV2
// sizes-then-chars (:339-430), writeVarUInt (IO/VarInt.h:224-240).
//
// Layout of a packet:
//   V1:       0x02 (CompressionMethodByte::NONE) | varuint cols | varuint rows | per column
//             (varuint len, name, varuint len, type name) | per part: varuint part_rows, then
//             every column's bulk data for the part.
//   CHBlock:  varuint cols | varuint rows | per column: name, type name, bulk data (if rows).
// Bulk data: fixed-width values little-endian (Int128 for Decimal(p<=38)); Nullable(T): rows null
// bytes then T's data; String: per row varuint(size) + size bytes (no terminator); StringV2:
// rows UInt64 sizes (terminator included), then the chars (terminators included).
//
// GPU design.  The header is a few bytes: the host builds it (encode) or parses it from small
// windows read back from the device (decode).  The bulk data never leaves HBM: fixed-width
// columns and StringV2 chars are device-to-device copies; StringV2 sizes are a difference /
// scan kernel; legacy String rows are a length scan + one-row-per-thread writer (encode) and a
// chunk-speculative parse (decode, below).
//
// Legacy String decode: record i starts where record i-1 ends, a serial chain.  The byte range
// is cut into chunks of CH bytes; for every chunk and every entry offset e < L (the position of
// its first record start relative to the chunk), one lane walks the records in LDS and yields
// (exit offset into the next chunk, records started in the chunk).  Composing these maps from
// chunk 0 (entry 0) — 64 chunks per group, then groups sequentially, then chunks inside each
// group — gives every chunk its true entry and first row; a final walk per chunk writes the row
// start positions.  A record that crosses a chunk boundary by >= L bytes makes the map
// undefined; the path then falls back to one device thread walking the rows (still exact).
#include <cstdio>

#include "common.h"

namespace tfg {

constexpr uint8_t COMP_NONE = 0x02; // CompressionMethodByte::NONE (IO/Compression/CompressionInfo.h:55)
constexpr uint8_t COMP_LZ4 = 0x82;  // CompressionMethodByte::LZ4 (frames decompressed by lz4.hip)
constexpr uint8_t COMP_ZSTD = 0x90; // CompressionMethodByte::ZSTD (frames decompressed by lz4.hip + zstd_dec.h)
constexpr int LCH = 32768;          // legacy parse chunk bytes
constexpr int LENT = 256;           // entry offsets per chunk (threads of the map kernel)
constexpr int LGRP = 64;            // chunks per resolution group
constexpr uint16_t LONG_EXIT = 0xFFFF;

// ------------------------------------------------------------------------------------ types
struct CType {
    int type = 0;       // tfg_type of the payload
    int width = 0;      // bytes per value (0 for strings)
    bool nullable = false;
    bool string = false;
    bool v2 = false;    // StringV2 (SeparateSizeAndChars)
    std::string name;   // the type name as written on the wire
};

static bool parse_type_name(const std::string &s, CType &t) {
    t = CType{};
    t.name = s;
    std::string x = s;
    if (x.rfind("Nullable(", 0) == 0 && x.back() == ')') {
        t.nullable = true;
        x = x.substr(9, x.size() - 10);
    }
    static const struct {
        const char *n;
        int type;
    } fixed[] = {{"Int8", TFG_INT8},       {"Int16", TFG_INT16},     {"Int32", TFG_INT32},   {"Int64", TFG_INT64},
                 {"UInt8", TFG_UINT8},     {"UInt16", TFG_UINT16},   {"UInt32", TFG_UINT32}, {"UInt64", TFG_UINT64},
                 {"Float32", TFG_FLOAT32}, {"Float64", TFG_FLOAT64}, {"MyDate", TFG_UINT64}};
    for (const auto &f : fixed)
        if (x == f.n) {
            t.type = f.type;
            t.width = (int)type_width(f.type);
            return true;
        }
    // MyDateTime(fsp) is a packed UInt64, MyDuration(fsp) an Int64 of nanoseconds
    if (x.rfind("MyDateTime(", 0) == 0) {
        t.type = TFG_UINT64;
        t.width = 8;
        return true;
    }
    if (x.rfind("MyDuration(", 0) == 0) {
        t.type = TFG_INT64;
        t.width = 8;
        return true;
    }
    if (x == "String" || x == "StringV2") {
        t.type = TFG_STRING;
        t.string = true;
        t.v2 = x == "StringV2";
        return true;
    }
    int p = 0, sc = 0;
    if (sscanf(x.c_str(), "Decimal(%d,%d)", &p, &sc) == 2 || sscanf(x.c_str(), "Decimal(%d, %d)", &p, &sc) == 2) {
        if (p <= 0 || p > 38) return false; // Decimal256 (boost multiprecision) is out of scope
        t.type = p <= 9 ? TFG_DECIMAL32 : p <= 18 ? TFG_DECIMAL64 : TFG_DECIMAL128;
        t.width = (int)type_width(t.type);
        return true;
    }
    return false;
}

static void put_varuint(std::string &o, uint64_t x) { // IO/VarInt.h:224-240 (at most 9 bytes)
    for (int i = 0; i < 9; ++i) {
        uint8_t b = x & 0x7F;
        if (x > 0x7F) b |= 0x80;
        o.push_back((char)b);
        x >>= 7;
        if (!x) return;
    }
}
static void put_string(std::string &o, const std::string &s) { // writeStringBinary
    put_varuint(o, s.size());
    o += s;
}
static int varuint_len_host(uint64_t x) {
    int n = 1;
    while (x > 0x7F && n < 10) {
        x >>= 7;
        ++n;
    }
    return n;
}

__device__ __forceinline__ int varuint_len(uint64_t x) {
    int n = 1;
    while (x > 0x7F && n < 10) {
        x >>= 7;
        ++n;
    }
    return n;
}

// readVarUInt over a byte array; returns bytes consumed (0 = ran past `avail`)
__device__ __forceinline__ int read_varuint(const uint8_t *p, uint64_t avail, uint64_t &x) {
    x = 0;
    for (int i = 0; i < 10; ++i) {
        if ((uint64_t)i >= avail) return 0;
        const uint8_t b = p[i];
        x |= (uint64_t)(b & 0x7F) << (7 * i);
        if (!(b & 0x80)) return i + 1;
    }
    return 10;
}

// ------------------------------------------------------------------------------------ kernels
// legacy String encode: record bytes per row (varuint(size) + size, size = offsets diff - 1)
__global__ void str_legacy_len_kernel(const uint64_t *off, int64_t n, uint64_t *rec) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t sz = off[i] - (i ? off[i - 1] : 0) - 1;
        rec[i] = (uint64_t)varuint_len(sz) + sz;
    }
}

__global__ void str_legacy_write_kernel(const uint8_t *chars, const uint64_t *off, const uint64_t *pos, int64_t n,
                                        uint8_t *dst) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t b = i ? off[i - 1] : 0;
        uint64_t sz = off[i] - b - 1;
        uint8_t *d = dst + pos[i];
        for (;;) {
            uint8_t c = sz & 0x7F;
            if (sz > 0x7F) c |= 0x80;
            *d++ = c;
            sz >>= 7;
            if (!sz) break;
        }
        const uint64_t len = off[i] - b - 1;
        for (uint64_t k = 0; k < len; ++k) d[k] = chars[b + k];
    }
}

// StringV2 encode: sizes (terminator included)
__global__ void str_v2_sizes_kernel(const uint64_t *off, int64_t n, uint64_t *sizes) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        sizes[i] = off[i] - (i ? off[i - 1] : 0);
}

// legacy decode, step 1: per chunk and entry offset e, walk the records inside the chunk
__global__ void __launch_bounds__(LENT) str_map_kernel(const uint8_t *pkt, uint64_t s0, uint64_t wend, uint64_t pend,
                                                      uint16_t *exit_, uint32_t *cnt) {
    __shared__ uint8_t buf[LCH + 16];
    const uint64_t base = s0 + (uint64_t)blockIdx.x * LCH;
    for (int i = threadIdx.x; i < LCH + 16; i += LENT) buf[i] = base + i < pend ? pkt[base + i] : 0;
    __syncthreads();
    const uint64_t lim = wend - base < (uint64_t)LCH ? wend - base : (uint64_t)LCH; // bytes of this chunk
    uint64_t pos = threadIdx.x;
    uint32_t c = 0;
    while (pos < lim) {
        uint64_t sz;
        const int vl = read_varuint(buf + pos, pend - (base + pos), sz);
        if (vl == 0) { // truncated varint at the packet end: no further records
            pos = ~0ull >> 1;
            break;
        }
        ++c;
        pos += (uint64_t)vl + sz;
        if (pos < (uint64_t)vl) { // overflow from a corrupt size
            pos = ~0ull >> 1;
            break;
        }
    }
    const uint64_t ex = pos >= (uint64_t)LCH ? pos - LCH : 0; // pos < LCH only past the window end
    exit_[(size_t)blockIdx.x * LENT + threadIdx.x] = ex < (uint64_t)LENT ? (uint16_t)ex : LONG_EXIT;
    cnt[(size_t)blockIdx.x * LENT + threadIdx.x] = c;
}

// step 2: compose LGRP consecutive chunk maps per entry
__global__ void __launch_bounds__(LENT) str_group_kernel(const uint16_t *exit_, const uint32_t *cnt, int64_t nchunks,
                                                        uint16_t *gexit, uint64_t *gcnt) {
    const int64_t c0 = (int64_t)blockIdx.x * LGRP;
    uint32_t x = threadIdx.x;
    uint64_t tot = 0;
    for (int64_t c = c0; c < c0 + LGRP && c < nchunks; ++c) {
        if (x == LONG_EXIT) break;
        tot += cnt[(size_t)c * LENT + x];
        x = exit_[(size_t)c * LENT + x];
    }
    gexit[(size_t)blockIdx.x * LENT + threadIdx.x] = (uint16_t)x;
    gcnt[(size_t)blockIdx.x * LENT + threadIdx.x] = tot;
}

// step 3: groups in order from entry 0 (one thread); res[0] = records found, res[1] = long flag.
// Past the column's last row the walk runs through the bytes of the columns that follow; what
// it finds there (including undefined maps) is ignored.
__global__ void str_resolve_groups_kernel(const uint16_t *gexit, const uint64_t *gcnt, int64_t ngroups, uint64_t nrows,
                                          uint16_t *gentry, uint64_t *gbase, uint64_t *res) {
    uint32_t x = 0;
    uint64_t base = 0, lng = 0;
    int64_t g = 0;
    for (; g < ngroups && base < nrows; ++g) {
        if (x == LONG_EXIT) {
            lng = 1;
            break;
        }
        gentry[g] = (uint16_t)x;
        gbase[g] = base;
        base += gcnt[(size_t)g * LENT + x];
        x = gexit[(size_t)g * LENT + x];
    }
    for (; g < ngroups; ++g) gentry[g] = LONG_EXIT; // not needed (or undefined): skipped
    if (x == LONG_EXIT && base < nrows) lng = 1;
    res[0] = base;
    res[1] = lng;
}

// step 4: chunks of every group from the group's entry
__global__ void str_resolve_chunks_kernel(const uint16_t *exit_, const uint32_t *cnt, int64_t nchunks,
                                          const uint16_t *gentry, const uint64_t *gbase, int64_t ngroups,
                                          uint16_t *centry, uint64_t *cbase) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ngroups) return;
    uint32_t x = gentry[g];
    uint64_t base = x == LONG_EXIT ? 0 : gbase[g];
    for (int64_t c = g * LGRP; c < (g + 1) * LGRP && c < nchunks; ++c) {
        centry[c] = (uint16_t)x;
        cbase[c] = base;
        if (x == LONG_EXIT) {
            for (int64_t d = c + 1; d < (g + 1) * LGRP && d < nchunks; ++d) centry[d] = LONG_EXIT;
            return;
        }
        base += cnt[(size_t)c * LENT + x];
        x = exit_[(size_t)c * LENT + x];
    }
}

// step 5: one lane per chunk writes the start of every record (rows < nrows) and the end of
// the last one
__global__ void str_emit_kernel(const uint8_t *pkt, uint64_t s0, uint64_t wend, uint64_t pend, const uint16_t *centry,
                                const uint64_t *cbase, uint64_t nrows, uint64_t *starts, uint64_t *seg_end) {
    const int64_t c = blockIdx.x;
    if (threadIdx.x != 0 || centry[c] == LONG_EXIT) return;
    const uint64_t base = s0 + (uint64_t)c * LCH;
    uint64_t r = cbase[c];
    if (r >= nrows) return;
    const uint64_t lim = wend - base < (uint64_t)LCH ? wend - base : (uint64_t)LCH;
    uint64_t pos = centry[c];
    while (pos < lim && r < nrows) {
        uint64_t sz;
        const int vl = read_varuint(pkt + base + pos, pend - (base + pos), sz);
        if (vl == 0) return;
        starts[r++] = base + pos;
        pos += (uint64_t)vl + sz;
        if (r == nrows) *seg_end = base + pos;
    }
}

// fallback (records longer than LENT bytes across chunk boundaries): one thread walks the rows
__global__ void str_seq_kernel(const uint8_t *pkt, uint64_t s0, uint64_t pend, uint64_t nrows, uint64_t *starts,
                               uint64_t *res) {
    uint64_t pos = s0, r = 0;
    while (r < nrows && pos < pend) {
        uint64_t sz;
        const int vl = read_varuint(pkt + pos, pend - pos, sz);
        if (vl == 0) break;
        starts[r++] = pos;
        pos += (uint64_t)vl + sz;
    }
    res[0] = r;
    res[1] = pos;
}

// legacy decode, rows -> sizes with terminator
__global__ void str_legacy_sizes_kernel(const uint8_t *pkt, uint64_t pend, const uint64_t *starts, int64_t n,
                                        uint64_t *sizes) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t sz;
        read_varuint(pkt + starts[i], pend - starts[i], sz);
        sizes[i] = sz + 1;
    }
}

__global__ void str_legacy_copy_kernel(const uint8_t *pkt, const uint64_t *starts, const uint64_t *excl, int64_t n,
                                       uint64_t chars_base, uint64_t *out_off, uint8_t *out_chars) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t sz;
        const int vl = read_varuint(pkt + starts[i], 10, sz);
        const uint8_t *src = pkt + starts[i] + vl;
        uint8_t *d = out_chars + chars_base + excl[i];
        for (uint64_t k = 0; k < sz; ++k) d[k] = src[k];
        d[sz] = 0;
        out_off[i] = chars_base + excl[i] + sz + 1;
    }
}

// StringV2 decode: offsets = base + inclusive prefix of the sizes
__global__ void str_v2_offsets_kernel(const uint64_t *excl, const uint64_t *sizes, int64_t n, uint64_t base,
                                      uint64_t *out_off) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out_off[i] = base + excl[i] + sizes[i];
}

// ------------------------------------------------------------------------------------ host side
struct Seg { // one column's data inside one part of a packet
    int64_t rows = 0;
    uint64_t null_off = 0; // nullable: packet offset of the null map
    uint64_t data_off = 0; // fixed: values; V2: sizes; legacy: first record
    uint64_t chars_off = 0;   // V2: packet offset of the chars
    uint64_t chars_bytes = 0; // strings: decoded chars (terminators included)
    uint64_t *starts = nullptr; // legacy: device row start positions (owned)
};

} // namespace tfg

struct tfg_codec_packet {
    tfg::Ctx *ctx = nullptr;
    const uint8_t *pkt = nullptr;
    uint64_t bytes = 0;
    int64_t rows = 0;
    std::vector<std::string> names;
    std::vector<tfg::CType> types;
    std::vector<std::vector<tfg::Seg>> segs; // [column][part]
    uint8_t *owned = nullptr;                // LZ4 packets: the decompressed NONE packet
    ~tfg_codec_packet() {
        if (owned) (void)hipFree(owned);
        for (auto &c : segs)
            for (auto &s : c)
                if (s.starts) (void)hipFree(s.starts);
    }
};

namespace tfg {

// Host view of the device packet: windows read back on demand (the header is small).
struct PacketReader {
    Ctx *ctx;
    const uint8_t *pkt;
    uint64_t bytes;
    uint64_t pos = 0;
    std::vector<uint8_t> win;
    uint64_t win_off = 0;
    int fetch(uint64_t at, uint64_t len) {
        if (at >= win_off && at + len <= win_off + win.size()) return TFG_OK;
        const uint64_t n = std::min<uint64_t>(bytes - at, std::max<uint64_t>(len, 65536));
        win.resize(n);
        win_off = at;
        TFG_HIP(hipMemcpyAsync(win.data(), pkt + at, n, hipMemcpyDeviceToHost, ctx->stream));
        TFG_HIP(hipStreamSynchronize(ctx->stream));
        return TFG_OK;
    }
    int byte(uint8_t &b) {
        TFG_CHECK(pos < bytes, TFG_ERR_INVALID_ARG, "packet truncated at byte %llu", (unsigned long long)pos);
        if (int rc = fetch(pos, 1)) return rc;
        b = win[pos - win_off];
        ++pos;
        return TFG_OK;
    }
    int varuint(uint64_t &x) {
        x = 0;
        for (int i = 0; i < 10; ++i) {
            uint8_t b;
            if (int rc = byte(b)) return rc;
            x |= (uint64_t)(b & 0x7F) << (7 * i);
            if (!(b & 0x80)) return TFG_OK;
        }
        return TFG_OK;
    }
    int str(std::string &s) {
        uint64_t n;
        if (int rc = varuint(n)) return rc;
        TFG_CHECK(n <= bytes - pos, TFG_ERR_INVALID_ARG, "string of %llu bytes past the packet end", (unsigned long long)n);
        if (int rc = fetch(pos, n)) return rc;
        s.assign((const char *)win.data() + (pos - win_off), n);
        pos += n;
        return TFG_OK;
    }
    int skip(uint64_t n) {
        TFG_CHECK(n <= bytes - pos, TFG_ERR_INVALID_ARG, "column data past the packet end");
        pos += n;
        return TFG_OK;
    }
};

static int read_u64_host(Ctx *ctx, const uint64_t *dev, uint64_t *host, size_t n) { return read_back_u64(ctx, dev, host, n); }

// Locates the `rows` legacy String records starting at s0 (device parse); fills seg.starts and
// returns the end position.
static int parse_legacy_strings(Ctx *ctx, const uint8_t *pkt, uint64_t pend, uint64_t s0, int64_t rows, Seg &seg,
                                uint64_t &end) {
    TFG_HIP(hipMalloc(&seg.starts, (size_t)std::max<int64_t>(rows, 1) * 8));
    uint64_t window = std::min<uint64_t>(pend - s0, (uint64_t)rows * 16 + 4096);
    for (;;) {
        const int64_t nch = (int64_t)((window + LCH - 1) / LCH);
        const int64_t ngr = (nch + LGRP - 1) / LGRP;
        Carver cv;
        const size_t o_exit = cv.take<uint16_t>((size_t)nch * LENT), o_cnt = cv.take<uint32_t>((size_t)nch * LENT);
        const size_t o_gexit = cv.take<uint16_t>((size_t)ngr * LENT), o_gcnt = cv.take<uint64_t>((size_t)ngr * LENT);
        const size_t o_gent = cv.take<uint16_t>(ngr), o_gbase = cv.take<uint64_t>(ngr);
        const size_t o_cent = cv.take<uint16_t>(nch), o_cbase = cv.take<uint64_t>(nch), o_res = cv.take<uint64_t>(4);
        void *sp;
        if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
        char *sb = (char *)sp;
        uint16_t *ex = (uint16_t *)(sb + o_exit), *gex = (uint16_t *)(sb + o_gexit);
        uint32_t *cn = (uint32_t *)(sb + o_cnt);
        uint64_t *gcn = (uint64_t *)(sb + o_gcnt), *gbase = (uint64_t *)(sb + o_gbase), *cbase = (uint64_t *)(sb + o_cbase);
        uint16_t *gent = (uint16_t *)(sb + o_gent), *cent = (uint16_t *)(sb + o_cent);
        uint64_t *res = (uint64_t *)(sb + o_res);
        const uint64_t wend = s0 + window;
        TFG_HIP(hipMemsetAsync(res, 0, 32, ctx->stream));
        hipLaunchKernelGGL(str_map_kernel, dim3(nch), dim3(LENT), 0, ctx->stream, pkt, s0, wend, pend, ex, cn);
        hipLaunchKernelGGL(str_group_kernel, dim3(ngr), dim3(LENT), 0, ctx->stream, ex, cn, nch, gex, gcn);
        hipLaunchKernelGGL(str_resolve_groups_kernel, dim3(1), dim3(1), 0, ctx->stream, gex, gcn, ngr, (uint64_t)rows, gent,
                           gbase, res);
        hipLaunchKernelGGL(str_resolve_chunks_kernel, dim3((ngr + 63) / 64), dim3(64), 0, ctx->stream, ex, cn, nch, gent,
                           gbase, ngr, cent, cbase);
        hipLaunchKernelGGL(str_emit_kernel, dim3(nch), dim3(64), 0, ctx->stream, pkt, s0, wend, pend, cent, cbase,
                           (uint64_t)rows, seg.starts, res + 2);
        TFG_LAUNCH_CHECK();
        uint64_t h[4];
        if (int rc = read_u64_host(ctx, res, h, 4)) return rc;
        if (h[1]) { // a long record crossed a chunk boundary: sequential walk (exact, slower)
            hipLaunchKernelGGL(str_seq_kernel, dim3(1), dim3(1), 0, ctx->stream, pkt, s0, pend, (uint64_t)rows, seg.starts,
                               res);
            TFG_LAUNCH_CHECK();
            if (int rc = read_u64_host(ctx, res, h, 2)) return rc;
            TFG_CHECK(h[0] == (uint64_t)rows, TFG_ERR_INVALID_ARG, "String column truncated: %llu of %lld rows",
                      (unsigned long long)h[0], (long long)rows);
            end = h[1];
            return TFG_OK;
        }
        if (h[0] >= (uint64_t)rows) {
            end = h[2];
            return TFG_OK;
        }
        TFG_CHECK(wend < pend, TFG_ERR_INVALID_ARG, "String column truncated: %llu of %lld rows", (unsigned long long)h[0],
                  (long long)rows);
        window = std::min<uint64_t>(pend - s0, window * 2);
    }
}

// Plans one column of one part: records its offsets and advances the reader past its data.
static int plan_segment(Ctx *ctx, PacketReader &rd, const CType &t, int64_t rows, Seg &seg) {
    seg.rows = rows;
    if (t.nullable) {
        seg.null_off = rd.pos;
        if (int rc = rd.skip((uint64_t)rows)) return rc;
    }
    seg.data_off = rd.pos;
    if (!t.string) return rd.skip((uint64_t)rows * t.width);
    if (t.v2) {
        if (int rc = rd.skip((uint64_t)rows * 8)) return rc;
        // chars bytes = sum of the sizes (device reduction through the scan)
        Carver cv;
        const size_t o_sz = cv.take<uint64_t>(rows), o_ex = cv.take<uint64_t>(rows + 1), o_scan = cv.take<uint8_t>(scan_tmp_bytes(rows));
        void *sp;
        if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
        char *sb = (char *)sp;
        TFG_HIP(hipMemcpyAsync(sb + o_sz, rd.pkt + seg.data_off, (size_t)rows * 8, hipMemcpyDeviceToDevice, ctx->stream));
        if (int rc = exclusive_scan_u64(ctx, (const uint64_t *)(sb + o_sz), (uint64_t *)(sb + o_ex), rows, sb + o_scan)) return rc;
        uint64_t tot;
        if (int rc = read_u64_host(ctx, (const uint64_t *)(sb + o_ex) + rows, &tot, 1)) return rc;
        seg.chars_off = rd.pos;
        seg.chars_bytes = tot;
        return rd.skip(tot);
    }
    uint64_t end = 0;
    if (int rc = parse_legacy_strings(ctx, rd.pkt, rd.bytes, rd.pos, rows, seg, end)) return rc;
    // chars bytes with terminators = record bytes - varuint bytes + rows; computed at read time
    Carver cv;
    const size_t o_sz = cv.take<uint64_t>(rows), o_ex = cv.take<uint64_t>(rows + 1), o_scan = cv.take<uint8_t>(scan_tmp_bytes(rows));
    void *sp;
    if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
    char *sb = (char *)sp;
    hipLaunchKernelGGL(str_legacy_sizes_kernel, dim3(stream_grid(rows, 256)), dim3(256), 0, ctx->stream, rd.pkt, rd.bytes,
                       seg.starts, rows, (uint64_t *)(sb + o_sz));
    TFG_LAUNCH_CHECK();
    if (int rc = exclusive_scan_u64(ctx, (const uint64_t *)(sb + o_sz), (uint64_t *)(sb + o_ex), rows, sb + o_scan)) return rc;
    if (int rc = read_u64_host(ctx, (const uint64_t *)(sb + o_ex) + rows, &seg.chars_bytes, 1)) return rc;
    TFG_CHECK(end >= rd.pos, TFG_ERR_LOGICAL, "String parse went backwards");
    return rd.skip(end - rd.pos);
}

} // namespace tfg

using namespace tfg;

extern "C" {

int tfg_codec_encode(tfg_ctx *ctx, int version, int ncols, const tfg_codec_column *cols, int64_t n, uint8_t *out,
                     size_t capacity, size_t *out_bytes) {
    TFG_CHECK(ctx && out_bytes && ncols >= 0 && n >= 0 && (ncols == 0 || cols), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(version == TFG_CODEC_CHBLOCK || version == TFG_CODEC_V1, TFG_ERR_INVALID_ARG, "codec version %d", version);
    if (int rc = set_device(ctx)) return rc;
    *out_bytes = 0;
    if (version == TFG_CODEC_V1 && n == 0) return TFG_OK; // V1 encodes nothing without rows (:379-386)
    std::vector<CType> ts(ncols);
    for (int c = 0; c < ncols; ++c) {
        TFG_CHECK(cols[c].name && cols[c].type_name, TFG_ERR_INVALID_ARG, "column %d: null name", c);
        TFG_CHECK(parse_type_name(cols[c].type_name, ts[c]), TFG_ERR_ILLEGAL_TYPE, "column %d: type %s not supported", c,
                  cols[c].type_name);
        TFG_CHECK(n == 0 || (cols[c].data && (!ts[c].string || cols[c].offsets) && (!ts[c].nullable || cols[c].nullmap)),
                  TFG_ERR_INVALID_ARG, "column %d: null data", c);
    }
    // header
    std::string hdr;
    if (version == TFG_CODEC_V1) hdr.push_back((char)COMP_NONE);
    put_varuint(hdr, (uint64_t)ncols);
    put_varuint(hdr, (uint64_t)n);
    // per column: the host header piece before its data, and the data size
    std::vector<std::string> pre(ncols);
    std::vector<uint64_t> dbytes(ncols, 0), chars(ncols, 0);
    std::vector<size_t> o_pos(ncols, 0);
    Carver cv;
    for (int c = 0; c < ncols; ++c)
        if (ts[c].string && n > 0) o_pos[c] = cv.take<uint64_t>((size_t)n + 1);
    const size_t o_rec = cv.take<uint64_t>((size_t)n), o_scan = cv.take<uint8_t>(scan_tmp_bytes(n));
    char *sb = nullptr;
    if (n > 0) {
        void *sp;
        if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
        sb = (char *)sp;
    }
    for (int c = 0; c < ncols; ++c) {
        std::string &p = version == TFG_CODEC_V1 ? hdr : pre[c];
        put_string(p, cols[c].name);
        put_string(p, ts[c].name);
        if (n == 0) continue;
        uint64_t b = ts[c].nullable ? (uint64_t)n : 0;
        if (!ts[c].string) {
            b += (uint64_t)n * ts[c].width;
        } else if (ts[c].v2) {
            if (int rc = read_u64_host(ctx, cols[c].offsets + (n - 1), &chars[c], 1)) return rc;
            b += (uint64_t)n * 8 + chars[c];
        } else {
            hipLaunchKernelGGL(str_legacy_len_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, ctx->stream, cols[c].offsets,
                               n, (uint64_t *)(sb + o_rec));
            TFG_LAUNCH_CHECK();
            if (int rc = exclusive_scan_u64(ctx, (const uint64_t *)(sb + o_rec), (uint64_t *)(sb + o_pos[c]), n, sb + o_scan))
                return rc;
            uint64_t tot;
            if (int rc = read_u64_host(ctx, (const uint64_t *)(sb + o_pos[c]) + n, &tot, 1)) return rc;
            b += tot;
        }
        dbytes[c] = b;
    }
    std::string part; // V1: the part's row count
    if (version == TFG_CODEC_V1) put_varuint(part, (uint64_t)n);
    uint64_t total = hdr.size() + part.size();
    for (int c = 0; c < ncols; ++c) total += pre[c].size() + dbytes[c];
    *out_bytes = total;
    if (!out) return TFG_OK; // size query
    TFG_CHECK(capacity >= total, TFG_ERR_CAPACITY, "packet needs %llu bytes, capacity %zu", (unsigned long long)total, capacity);
    std::string host = hdr + part; // host pieces are copied synchronously (pageable memory)
    uint64_t at = 0;
    auto put_host = [&](const std::string &s) -> int {
        if (!s.empty()) TFG_HIP(hipMemcpyAsync(out + at, s.data(), s.size(), hipMemcpyHostToDevice, ctx->stream));
        at += s.size();
        return TFG_OK;
    };
    if (int rc = put_host(host)) return rc;
    for (int c = 0; c < ncols; ++c) {
        if (int rc = put_host(pre[c])) return rc;
        if (n == 0) continue;
        if (ts[c].nullable) {
            TFG_HIP(hipMemcpyAsync(out + at, cols[c].nullmap, (size_t)n, hipMemcpyDeviceToDevice, ctx->stream));
            at += (uint64_t)n;
        }
        if (!ts[c].string) {
            TFG_HIP(hipMemcpyAsync(out + at, cols[c].data, (size_t)n * ts[c].width, hipMemcpyDeviceToDevice, ctx->stream));
            at += (uint64_t)n * ts[c].width;
        } else if (ts[c].v2) {
            uint64_t *sizes = (uint64_t *)(sb + o_rec);
            hipLaunchKernelGGL(str_v2_sizes_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, ctx->stream, cols[c].offsets, n,
                               sizes);
            TFG_LAUNCH_CHECK();
            TFG_HIP(hipMemcpyAsync(out + at, sizes, (size_t)n * 8, hipMemcpyDeviceToDevice, ctx->stream));
            at += (uint64_t)n * 8;
            if (chars[c]) TFG_HIP(hipMemcpyAsync(out + at, cols[c].data, chars[c], hipMemcpyDeviceToDevice, ctx->stream));
            at += chars[c];
        } else {
            hipLaunchKernelGGL(str_legacy_write_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, ctx->stream,
                               (const uint8_t *)cols[c].data, cols[c].offsets, (const uint64_t *)(sb + o_pos[c]), n, out + at);
            TFG_LAUNCH_CHECK();
            at += dbytes[c] - (ts[c].nullable ? (uint64_t)n : 0);
        }
    }
    TFG_CHECK(at == total, TFG_ERR_LOGICAL, "encoded %llu of %llu bytes", (unsigned long long)at, (unsigned long long)total);
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    return TFG_OK;
}

int tfg_codec_decode(tfg_ctx *ctx, int version, const uint8_t *packet, size_t bytes, tfg_codec_packet **out) {
    TFG_CHECK(ctx && out && (bytes == 0 || packet), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(version == TFG_CODEC_CHBLOCK || version == TFG_CODEC_V1, TFG_ERR_INVALID_ARG, "codec version %d", version);
    if (int rc = set_device(ctx)) return rc;
    *out = nullptr;
    auto *p = new tfg_codec_packet();
    p->ctx = ctx;
    p->pkt = packet;
    p->bytes = bytes;
    auto done = [&](int rc) {
        if (rc) delete p;
        else *out = p;
        return rc;
    };
    if (bytes == 0) return done(TFG_OK); // the empty Block (decodeImpl: eof -> Block{})
    PacketReader rd{ctx, packet, bytes};
    if (version == TFG_CODEC_V1) {
        uint8_t m;
        if (int rc = rd.byte(m)) return done(rc);
        if (m == COMP_LZ4 || m == COMP_ZSTD) { // CompressedCHBlockChunkReadBuffer: decompress, then read as NONE
            size_t raw = 0;
            if (int rc = tfg_codec_decompress(ctx, packet, bytes, nullptr, 0, &raw)) return done(rc);
            if (hipMalloc(&p->owned, raw) != hipSuccess) return done(fail(TFG_ERR_OOM, "decompressed packet of %zu bytes", raw));
            if (int rc = tfg_codec_decompress(ctx, packet, bytes, p->owned, raw, &raw)) return done(rc);
            p->pkt = p->owned;
            p->bytes = raw;
            rd = PacketReader{ctx, p->owned, raw};
            if (int rc = rd.byte(m)) return done(rc);
        } else if (m != COMP_NONE) {
            return done(fail(TFG_ERR_NOT_IMPLEMENTED, "compressed packet (method byte 0x%02x): NONE, LZ4 and ZSTD only", m));
        }
    }
    uint64_t ncols, rows;
    if (int rc = rd.varuint(ncols)) return done(rc);
    if (int rc = rd.varuint(rows)) return done(rc);
    if (ncols > 4096) return done(fail(TFG_ERR_INVALID_ARG, "column count %llu", (unsigned long long)ncols));
    p->rows = (int64_t)rows;
    p->names.resize(ncols);
    p->types.resize(ncols);
    p->segs.resize(ncols);
    auto read_meta = [&](uint64_t c) -> int {
        std::string tn;
        if (int rc = rd.str(p->names[c])) return rc;
        if (int rc = rd.str(tn)) return rc;
        TFG_CHECK(parse_type_name(tn, p->types[c]), TFG_ERR_ILLEGAL_TYPE, "column %llu: type %s not supported",
                  (unsigned long long)c, tn.c_str());
        return TFG_OK;
    };
    if (version == TFG_CODEC_V1) {
        for (uint64_t c = 0; c < ncols; ++c)
            if (int rc = read_meta(c)) return done(rc);
        uint64_t got = 0;
        while (got < rows) { // parts (decodeColumnsByBlock)
            uint64_t sz;
            if (int rc = rd.varuint(sz)) return done(rc);
            if (sz == 0 || sz > rows - got) return done(fail(TFG_ERR_INVALID_ARG, "part of %llu rows", (unsigned long long)sz));
            for (uint64_t c = 0; c < ncols; ++c) {
                p->segs[c].emplace_back();
                if (int rc = plan_segment(ctx, rd, p->types[c], (int64_t)sz, p->segs[c].back())) return done(rc);
            }
            got += sz;
        }
    } else {
        for (uint64_t c = 0; c < ncols; ++c) {
            if (int rc = read_meta(c)) return done(rc);
            if (rows) {
                p->segs[c].emplace_back();
                if (int rc = plan_segment(ctx, rd, p->types[c], (int64_t)rows, p->segs[c].back())) return done(rc);
            }
        }
    }
    return done(TFG_OK);
}

int tfg_codec_packet_info(tfg_codec_packet *p, int *out_cols, int64_t *out_rows) {
    TFG_CHECK(p && out_cols && out_rows, TFG_ERR_INVALID_ARG, "null argument");
    *out_cols = (int)p->types.size();
    *out_rows = p->rows;
    return TFG_OK;
}

int tfg_codec_column_info(tfg_codec_packet *p, int i, char *name, size_t name_len, char *type_name, size_t type_len,
                          int *out_type, int *out_nullable, uint64_t *out_chars_bytes) {
    TFG_CHECK(p && i >= 0 && i < (int)p->types.size(), TFG_ERR_INVALID_ARG, "column %d out of range", i);
    const CType &t = p->types[i];
    if (name && name_len) snprintf(name, name_len, "%s", p->names[i].c_str());
    if (type_name && type_len) snprintf(type_name, type_len, "%s", t.name.c_str());
    if (out_type) *out_type = t.type;
    if (out_nullable) *out_nullable = t.nullable ? 1 : 0;
    if (out_chars_bytes) {
        uint64_t b = 0;
        for (const Seg &s : p->segs[i]) b += s.chars_bytes;
        *out_chars_bytes = b;
    }
    return TFG_OK;
}

int tfg_codec_column_read(tfg_codec_packet *p, int i, void *out_data, uint64_t *out_offsets, uint8_t *out_nullmap) {
    TFG_CHECK(p && i >= 0 && i < (int)p->types.size(), TFG_ERR_INVALID_ARG, "column %d out of range", i);
    Ctx *ctx = p->ctx;
    if (int rc = set_device(ctx)) return rc;
    const CType &t = p->types[i];
    TFG_CHECK(p->rows == 0 || (out_data && (!t.string || out_offsets) && (!t.nullable || out_nullmap)), TFG_ERR_INVALID_ARG,
              "null output");
    int64_t row0 = 0;
    uint64_t chars0 = 0;
    for (const Seg &s : p->segs[i]) {
        const int64_t n = s.rows;
        if (t.nullable)
            TFG_HIP(hipMemcpyAsync(out_nullmap + row0, p->pkt + s.null_off, (size_t)n, hipMemcpyDeviceToDevice, ctx->stream));
        if (!t.string) {
            TFG_HIP(hipMemcpyAsync((uint8_t *)out_data + (size_t)row0 * t.width, p->pkt + s.data_off, (size_t)n * t.width,
                                   hipMemcpyDeviceToDevice, ctx->stream));
        } else {
            Carver cv;
            const size_t o_sz = cv.take<uint64_t>(n), o_ex = cv.take<uint64_t>(n + 1), o_scan = cv.take<uint8_t>(scan_tmp_bytes(n));
            void *sp;
            if (int rc = scratch_get(ctx, cv.off, &sp)) return rc;
            char *sb = (char *)sp;
            uint64_t *sizes = (uint64_t *)(sb + o_sz), *ex = (uint64_t *)(sb + o_ex);
            if (t.v2) {
                TFG_HIP(hipMemcpyAsync(sizes, p->pkt + s.data_off, (size_t)n * 8, hipMemcpyDeviceToDevice, ctx->stream));
                if (int rc = exclusive_scan_u64(ctx, sizes, ex, n, sb + o_scan)) return rc;
                hipLaunchKernelGGL(str_v2_offsets_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, ctx->stream, ex, sizes, n,
                                   chars0, out_offsets + row0);
                TFG_LAUNCH_CHECK();
                if (s.chars_bytes)
                    TFG_HIP(hipMemcpyAsync((uint8_t *)out_data + chars0, p->pkt + s.chars_off, s.chars_bytes,
                                           hipMemcpyDeviceToDevice, ctx->stream));
            } else {
                hipLaunchKernelGGL(str_legacy_sizes_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, ctx->stream, p->pkt,
                                   p->bytes, s.starts, n, sizes);
                TFG_LAUNCH_CHECK();
                if (int rc = exclusive_scan_u64(ctx, sizes, ex, n, sb + o_scan)) return rc;
                hipLaunchKernelGGL(str_legacy_copy_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, ctx->stream, p->pkt,
                                   s.starts, ex, n, chars0, out_offsets + row0, (uint8_t *)out_data);
                TFG_LAUNCH_CHECK();
            }
            chars0 += s.chars_bytes;
        }
        row0 += n;
    }
    return TFG_OK;
}

int tfg_codec_packet_destroy(tfg_codec_packet *p) {
    if (p) {
        if (p->ctx) (void)hipStreamSynchronize(p->ctx->stream);
        delete p;
    }
    return TFG_OK;
}

} // extern "C"
