// codec_zstd.h — the device ZSTD decode of a packet's frames (zstd.hip), called by
// tfg_codec_decompress (lz4.hip) once the frame table is known.
#pragma once
#include "common.h"

namespace tfg {
// Frames [0, nf) of `packet`: dfo / dro the device frame tables (frame f's 9-byte header at
// packet + fo[f], its raw bytes at dst + ro[f]), fo / ro their host copies.  Decodes every frame
// into dst; a malformed frame raises *err (device) or returns an error.  Syncs the stream.
int zstd_decode_frames(Ctx *ctx, const uint8_t *packet, uint64_t nf, const uint64_t *dfo, const uint64_t *dro,
                       const uint64_t *fo, const uint64_t *ro, uint8_t *dst, unsigned *err);
} // namespace tfg
