// codec_zstd.h — the device ZSTD codec of a packet's frames: the decode (zstd.hip), called by
// tfg_codec_decompress (lz4.hip) once the frame table is known, and the encode (zstd_enc.hip),
// called by tfg_codec_compress.
#pragma once
#include "common.h"

namespace tfg {
// Frames [0, nf) of `packet`: dfo / dro the device frame tables (frame f's 9-byte header at
// packet + fo[f], its raw bytes at dst + ro[f]), fo / ro their host copies.  Decodes every frame
// into dst; a malformed frame raises *err (device) or returns an error.  Syncs the stream.
int zstd_decode_frames(Ctx *ctx, const uint8_t *packet, uint64_t nf, const uint64_t *dfo, const uint64_t *dro,
                       const uint64_t *fo, const uint64_t *ro, uint8_t *dst, unsigned *err);

// The sender: body[0, n) in frames of ZE_FRAME raw bytes, frame f (its 9-byte packet header and
// one ZSTD frame) written to slots + f * ZE_SLOT, its size to sizes[f].  tmp: zstd_encode_tmp_bytes
// of device scratch.  Launches only (no sync).
constexpr uint32_t ZE_FRAME = 64 * 1024;
constexpr uint64_t ZE_SLOT = 9 + 9 + 3 + ZE_FRAME + 64; // headers + a raw block
size_t zstd_encode_tmp_bytes(uint64_t nframes);
int zstd_encode_frames(Ctx *ctx, const uint8_t *body, uint64_t n, uint64_t nframes, uint8_t *slots, uint32_t *sizes,
                       void *tmp);
} // namespace tfg
