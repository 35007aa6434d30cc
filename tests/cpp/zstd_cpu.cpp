// Host build of tiflash_amd/csrc/zstd_dec.h for the CPU check of the ZSTD decoder against the
// system libzstd (tests/test_zstd.py).  Test infrastructure only: the product decoder runs on the
// device (lz4.hip: the same stage-1 source, one wave per frame, and a wave-parallel stage 2).
#include <cstdlib>

#include "../../tiflash_amd/csrc/zstd_dec.h"

extern "C" int64_t tfz_decode_frame_cpu(const uint8_t *src, int64_t n, uint8_t *dst, uint64_t cap) {
    tfz::ZWork *w = (tfz::ZWork *)calloc(1, sizeof(tfz::ZWork));
    w->stage = nullptr;
    const int64_t r = tfz::zstd_frame(src, n, dst, cap, w);
    free(w);
    return r;
}
