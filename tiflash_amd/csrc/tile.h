// tile.h — coalesced tile loaders shared by the filter / hash / partition kernels.
//
// A "chunk" is 16 bytes of one column (one dwordx4 per lane); lane-consecutive chunks are
// byte-consecutive, so a wave moves 1 KiB per load instruction (Guideline 13 of the CDNA
// programming guide).  Partial / misaligned chunks fall back to per-element accesses.
#pragma once
#include "common.h"

namespace tfg {

template <int W> struct ElemOf;
template <> struct ElemOf<1> { using T = uint8_t; };
template <> struct ElemOf<2> { using T = uint16_t; };
template <> struct ElemOf<4> { using T = uint32_t; };
template <> struct ElemOf<8> { using T = uint64_t; };
struct alignas(16) U128 {
    uint64_t lo, hi;
};
template <> struct ElemOf<16> { using T = U128; };

// Load the elements of chunk `c` (elements [c*16/W, c*16/W + 16/W)) of a column of width W.
// Elements at or beyond n are left as zero.
template <int W>
__device__ __forceinline__ void load_chunk(const void *col, int64_t c, int64_t n, bool aligned,
                                           typename ElemOf<W>::T (&v)[16 / W]) {
    using E = typename ElemOf<W>::T;
    constexpr int PER = 16 / W;
    const int64_t r0 = c * PER;
    if (aligned && r0 + PER <= n) {
        uint4 q = reinterpret_cast<const uint4 *>(col)[c];
        memcpy(&v[0], &q, 16);
    } else {
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            if (r0 + e < n) v[e] = reinterpret_cast<const E *>(col)[r0 + e];
            else memset(&v[e], 0, sizeof(E));
        }
    }
}

template <typename T> __device__ __forceinline__ T load_elem(const void *col, int64_t r) {
    return reinterpret_cast<const T *>(col)[r];
}

inline bool is_aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

} // namespace tfg
