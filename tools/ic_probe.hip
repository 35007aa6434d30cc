// Measurement instrument (not product code): the non-partitioned C3 probe against a build table
// meant to stay resident in the 256 MB Infinity Cache.  The
// build side (10M keys) goes into a bucketised open-addressing table: 2^b buckets of 128 B, each
// 16 slots of {tag32, row + 1}; a probe reads its one bucket line (eight lanes cooperatively, one
// 16-byte load each), checks the tags, verifies a tag match against the build key array and
// gathers the build payload.  Every probe row is read once (no probe-side partition).  Timed
// against the partitioned v1 probe in tools/ic_probe.py.  Build:
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/ic_probe.hip -o tools/_ic_probe.so
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

constexpr int SLOTS = 16; // 8-byte slots a 128-byte bucket
constexpr int LPR = 8;    // lanes a probe row (each loads 16 B = 2 slots)
constexpr int RPG = 4;    // rows in flight per lane group

__device__ __forceinline__ uint64_t mix(uint64_t x) { // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

__global__ void build_kernel(const int64_t *bk, int64_t n, int bits, unsigned long long *table, unsigned *overflow) {
    const uint64_t mask = (1ull << bits) - 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix((uint64_t)bk[i]);
        const unsigned long long v = ((h & 0xFFFFFFFFull) << 32) | (uint64_t)(i + 1);
        uint64_t b = h >> (64 - bits);
        bool done = false;
        for (int step = 0; step < 1024 && !done; ++step, b = (b + 1) & mask) { // linear probing
            unsigned long long *s = table + b * SLOTS;
            for (int k = 0; k < SLOTS && !done; ++k)
                if (s[k] == 0ull && atomicCAS(&s[k], 0ull, v) == 0ull) done = true;
        }
        if (!done) atomicAdd(overflow, 1u);
    }
}

// mode 0: count matches only; mode 1: materialise (probe key, probe payload, build payload) per
// match, the output rows of a workgroup claimed by one atomic per round.  A full bucket (every
// slot taken) continues into the next one (the build's linear probing): rounds repeat for the
// rows whose bucket was full, uniformly over the workgroup
template <int MODE>
__global__ void __launch_bounds__(256) probe_kernel(const int64_t *pk, const int64_t *ppay, int64_t n, int bits,
                                                   const unsigned long long *table, const int64_t *bk,
                                                   const int64_t *bpay, unsigned long long *count, int64_t *out0,
                                                   int64_t *out1, int64_t *out2, uint64_t cap) {
    __shared__ unsigned long long s_base;
    __shared__ unsigned s_wsum[4];
    const int lane = threadIdx.x & 63, sub = lane & (LPR - 1), gshift = lane & ~(LPR - 1);
    const int grp_global = (int)((blockIdx.x * blockDim.x + threadIdx.x) / LPR);
    const int groups = (int)(gridDim.x * blockDim.x / LPR);
    const uint64_t bmask = (1ull << bits) - 1;
    unsigned long long local = 0;
    const int64_t steps = (n + (int64_t)groups * RPG - 1) / ((int64_t)groups * RPG);
    for (int64_t st = 0; st < steps; ++st) {
        int64_t row[RPG], key[RPG];
        uint64_t bkt[RPG];
        uint32_t tag[RPG];
        bool act[RPG];
#pragma unroll
        for (int u = 0; u < RPG; ++u) {
            row[u] = (st * RPG + u) * (int64_t)groups + grp_global;
            act[u] = row[u] < n;
            key[u] = act[u] ? __builtin_nontemporal_load(pk + row[u]) : 0;
        }
#pragma unroll
        for (int u = 0; u < RPG; ++u) {
            const uint64_t h = mix((uint64_t)key[u]);
            tag[u] = (uint32_t)h;
            bkt[u] = h >> (64 - bits);
        }
        for (int round = 0;; ++round) {
            bool any_act = false;
#pragma unroll
            for (int u = 0; u < RPG; ++u) any_act |= act[u];
            if (!__syncthreads_or(any_act)) break;
            uint4 line[RPG];
#pragma unroll
            for (int u = 0; u < RPG; ++u)
                line[u] = act[u] ? reinterpret_cast<const uint4 *>(table + bkt[u] * SLOTS)[sub] : make_uint4(0, 0, 0, 0);
            unsigned mine = 0; // this lane's matches (slot k of row u: bit u * 2 + k)
#pragma unroll
            for (int u = 0; u < RPG; ++u) {
                const uint64_t s0 = ((uint64_t)line[u].y << 32) | line[u].x, s1 = ((uint64_t)line[u].w << 32) | line[u].z;
                if (act[u]) {
                    if (s0 && (uint32_t)(s0 >> 32) == tag[u] && bk[(s0 & 0xFFFFFFFFull) - 1] == key[u]) mine |= 1u << (2 * u);
                    if (s1 && (uint32_t)(s1 >> 32) == tag[u] && bk[(s1 & 0xFFFFFFFFull) - 1] == key[u]) mine |= 2u << (2 * u);
                }
                // the bucket was full (all 8 lanes' slots taken): the row goes on to the next one
                const uint64_t fb = __ballot(act[u] && s0 && s1);
                const bool full = ((fb >> gshift) & 0xFFull) == 0xFFull;
                act[u] = act[u] && full;
                bkt[u] = (bkt[u] + 1) & bmask;
            }
            const unsigned cnt = __popc(mine);
            if constexpr (MODE == 0) {
                local += cnt;
            } else {
                unsigned x = cnt;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const unsigned y = __shfl_up(x, d, 64);
                    if (lane >= d) x += y;
                }
                if (lane == 63) s_wsum[threadIdx.x >> 6] = x;
                __syncthreads();
                unsigned pre = 0, tot = 0;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    if (w < (int)(threadIdx.x >> 6)) pre += s_wsum[w];
                    tot += s_wsum[w];
                }
                if (threadIdx.x == 0) s_base = tot ? atomicAdd(count, (unsigned long long)tot) : 0ull;
                __syncthreads();
                uint64_t pos = s_base + pre + x - cnt;
                for (unsigned m = mine; m; m &= m - 1) {
                    const int bit = __ffs(m) - 1, u = bit >> 1, k = bit & 1;
                    const uint64_t s = k ? (((uint64_t)line[u].w << 32) | line[u].z) : (((uint64_t)line[u].y << 32) | line[u].x);
                    const int64_t br = (int64_t)(s & 0xFFFFFFFFull) - 1;
                    if (pos < cap) {
                        __builtin_nontemporal_store(key[u], out0 + pos);
                        __builtin_nontemporal_store(ppay[row[u]], out1 + pos);
                        __builtin_nontemporal_store(bpay[br], out2 + pos);
                    }
                    ++pos;
                }
                __syncthreads(); // s_wsum / s_base are rewritten by the next round
            }
        }
    }
    if constexpr (MODE == 0) {
        for (int d = 32; d > 0; d >>= 1) local += __shfl_down(local, d, 64);
        if (lane == 0 && local) atomicAdd(count, local);
    }
}

} // namespace

extern "C" int icp_build(const int64_t *bk, int64_t n, int bits, unsigned long long *table, unsigned *overflow,
                         float *ms) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    if (hipMemsetAsync(table, 0, (size_t)SLOTS * 8 << bits, 0) != hipSuccess) return 1;
    if (hipMemsetAsync(overflow, 0, 4, 0) != hipSuccess) return 1;
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(build_kernel, dim3(4096), dim3(256), 0, 0, bk, n, bits, table, overflow);
    hipEventRecord(b, 0);
    if (hipEventSynchronize(b) != hipSuccess) return 2;
    hipEventElapsedTime(ms, a, b);
    return 0;
}

extern "C" int icp_probe(int mode, const int64_t *pk, const int64_t *ppay, int64_t n, int bits,
                         const unsigned long long *table, const int64_t *bk, const int64_t *bpay,
                         unsigned long long *count, int64_t *o0, int64_t *o1, int64_t *o2, uint64_t cap, int grid,
                         int reps, float *ms) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float total = 0;
    for (int i = 0; i <= reps; ++i) { // launch 0 warms up
        if (hipMemsetAsync(count, 0, 8, 0) != hipSuccess) return 1;
        hipEventRecord(a, 0);
        if (mode == 0)
            hipLaunchKernelGGL(probe_kernel<0>, dim3(grid), dim3(256), 0, 0, pk, ppay, n, bits, table, bk, bpay, count, o0,
                               o1, o2, cap);
        else
            hipLaunchKernelGGL(probe_kernel<1>, dim3(grid), dim3(256), 0, 0, pk, ppay, n, bits, table, bk, bpay, count, o0,
                               o1, o2, cap);
        hipEventRecord(b, 0);
        if (hipEventSynchronize(b) != hipSuccess) return 2;
        float t = 0;
        hipEventElapsedTime(&t, a, b);
        if (i > 0) total += t;
    }
    *ms = total / reps;
    return 0;
}
