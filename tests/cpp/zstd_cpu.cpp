// Host build of tiflash_amd/csrc/zstd_dec.h for the CPU check of the ZSTD decoder against the
// system libzstd (tests/test_zstd.py).  Test infrastructure only: the product decoder runs on the
// device (zstd.hip: the same scan / block / resolve source as kernels, and a parallel execution).
#include "../../tiflash_amd/csrc/zstd_dec.h"

// decodes one frame body that must decode to exactly `cap` bytes; the size, or -1
extern "C" int64_t tfz_decode_frame_cpu(const uint8_t *src, int64_t n, uint8_t *dst, uint64_t cap) {
    return tfz::zstd_frame(src, n, dst, cap);
}

// scan statistics of one frame body (blocks, records; -1 on error): test / tuning aid
extern "C" int64_t tfz_entropy_stats_cpu(const uint8_t *src, int64_t n, uint64_t cap, uint64_t *nblocks, uint64_t *nrec) {
    tfz::ZScan s;
    if (!tfz::zstd_scan(src, n, cap, s)) return -1;
    *nblocks = s.c.blocks;
    *nrec = s.c.recs;
    return 0;
}
