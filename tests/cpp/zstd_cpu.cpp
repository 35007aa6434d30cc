// Host build of tiflash_amd/csrc/zstd_dec.h for the CPU check of the ZSTD decoder against the
// system libzstd (tests/test_zstd.py).  Test infrastructure only: the product decoder runs on the
// device (lz4.hip, one thread per frame).
#include <cstdlib>

#include "../../tiflash_amd/csrc/zstd_dec.h"

extern "C" int64_t tfz_decode_frame_cpu(const uint8_t *src, int64_t n, uint8_t *dst, uint64_t cap) {
    tfz::ZWork *w = (tfz::ZWork *)calloc(1, sizeof(tfz::ZWork));
    w->lit = (uint8_t *)calloc(tfz::ZMAX_BLOCK + 32, 1);
    w->stage = nullptr;
    const int64_t r = tfz::zstd_frame(src, n, dst, cap, w);
    free(w->lit);
    free(w);
    return r;
}
