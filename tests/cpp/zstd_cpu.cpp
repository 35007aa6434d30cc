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

// stage-1 statistics of one frame body (records, literal bytes; -1 on error): test / tuning aid
extern "C" int64_t tfz_entropy_stats_cpu(const uint8_t *src, int64_t n, uint64_t cap, uint64_t *nseq, uint64_t *nlit) {
    tfz::ZWork *w = (tfz::ZWork *)calloc(1, sizeof(tfz::ZWork));
    tfz::ZOut o{};
    o.seq_cap = tfz::zstd_seq_cap(cap, (uint64_t)n);
    o.lit_cap = cap;
    o.seq = new tfz::ZSeq[o.seq_cap];
    o.lit = new uint8_t[cap + 1];
    const int64_t r = tfz::zstd_frame_entropy(src, n, cap, w, o);
    *nseq = o.nseq;
    *nlit = o.nlit;
    delete[] o.seq;
    delete[] o.lit;
    free(w);
    return r;
}
