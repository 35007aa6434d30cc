// fused_trace.hip — timing tool (not part of the product): builds agg_fused.hip with its
// TFG_FUSED_TRACE hooks, runs the fused C2 kernel on 100M synthetic rows and prints, per phase
// of the round loop, the average time per iteration over all workgroups (wall clock, 100 MHz).
// Build + run on the GPU box: bash tools/fused_trace.sh
#define TFG_FUSED_TRACE 1
#include "../tiflash_amd/csrc/agg_fused.hip"

#include <cstdio>
#include <vector>

using namespace tfg;

__global__ void init_kernel(int64_t *f, int64_t *k, double *v, int64_t n, int64_t groups) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull + 12345;
        h ^= h >> 31;
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 29;
        f[i] = (int64_t)(h % 100);
        k[i] = (int64_t)((h >> 8) % (uint64_t)groups);
        v[i] = (double)((h >> 20) & 0xFFFFF) / 256.0;
    }
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main() {
    const int64_t n = 100000000, groups = 1000000;
    int64_t *f, *k;
    double *v;
    CK(hipMalloc(&f, n * 8));
    CK(hipMalloc(&k, n * 8));
    CK(hipMalloc(&v, n * 8));
    hipLaunchKernelGGL(init_kernel, dim3(4096), dim3(256), 0, 0, f, k, v, n, groups);
    const int rounds = (int)((n + (int64_t)NB * TR - 1) / ((int64_t)NB * TR));
    FArgs A{};
    A.key = (const uint64_t *)k;
    A.val = (const uint64_t *)v;
    A.n = n;
    A.rounds = rounds;
    char *zero;
    CK(hipMalloc(&A.ring_rec, RING_REC_BYTES));
    CK(hipMalloc(&zero, RING_RUN_BYTES + CONS_BYTES + CTL_BYTES));
    A.ring_run = (uint32_t *)zero;
    A.cons_done = (uint32_t *)(zero + RING_RUN_BYTES);
    A.err = (uint32_t *)(zero + RING_RUN_BYTES + CONS_BYTES);
    A.cursor = (unsigned long long *)(zero + RING_RUN_BYTES + CONS_BYTES + 16);
    const size_t tg = (size_t)NB * (CAP + 1);
    CK(hipMalloc(&A.io.tmp_key, tg * 8));
    CK(hipMalloc(&A.io.tmp_key_null, tg));
    CK(hipMalloc(&A.io.tmp_sum, tg * 8));
    CK(hipMalloc(&A.io.tmp_cnt, tg * 8));
    CK(hipMalloc(&A.io.out_cnt, NB * 8));
    CK(hipMalloc(&A.io.tmp_base, NB * 8));
    CK(hipMalloc(&A.io.spill_key, n * 8));
    CK(hipMalloc(&A.io.spill_val, n * 8));
    const size_t tn = (size_t)NB * rounds * 8;
    CK(hipMalloc(&A.trace, tn * 8));
    PredT<2, int64_t, false> pred{f, nullptr, Num{0, 96, 96, 96.0}, TFG_LT};
    auto kern = agg_fused_kernel<PredT<2, int64_t, false>, 3, true>;
    void *args[] = {(void *)&pred, (void *)&A};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms = 0;
    for (int rep = 0; rep < 4; ++rep) {
        CK(hipMemsetAsync(zero, 0, RING_RUN_BYTES + CONS_BYTES + CTL_BYTES, 0));
        CK(hipMemsetAsync(A.trace, 0, tn * 8, 0));
        CK(hipEventRecord(e0, 0));
        CK(hipLaunchCooperativeKernel((const void *)kern, dim3(NB), dim3(FT), args, LDS_BYTES, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        uint64_t w[4];
        CK(hipMemcpy(w, A.err, 32, hipMemcpyDeviceToHost));
        printf("run %d: %.3f ms  err %llu  spilled %llu  groups %llu\n", rep, ms, (unsigned long long)w[0],
               (unsigned long long)w[2], (unsigned long long)w[3]);
    }
    std::vector<unsigned long long> tr(tn);
    CK(hipMemcpy(tr.data(), A.trace, tn * 8, hipMemcpyDeviceToHost));
    // producer iteration i: 0 start, 1 after rank + scan + place of round i, 2 after the drain
    // of round i - 1's stores + its publish + round i's slot wait, 3 after prefetch + store issue
    // consumer iteration q: 4 start, 5 after poll + scan + record-load issue of round q;
    // 6 (indexed by round q) after round q's fold + release, in iteration q + 1
    const char *names[] = {"P sort (rank, scan, place)", "P drain prev + publish + slot wait",
                           "P prefetch + store issue", "P -> next iteration", "C poll + scan + load issue",
                           "C fold prev round + release", "C -> next iteration"};
    double acc[7] = {}, cnt[7] = {};
    double pr = 0, prn = 0, cr = 0, crn = 0;
    for (int b = 0; b < NB; ++b)
        for (int i = 4; i < rounds - 2; ++i) {
            const unsigned long long *t = &tr[((size_t)b * rounds + i) * 8];
            const unsigned long long *u = &tr[((size_t)b * rounds + i + 1) * 8];
            const unsigned long long from[7] = {t[0], t[1], t[2], t[3], t[4], u[5], t[6]};
            const unsigned long long to[7] = {t[1], t[2], t[3], u[0], t[5], t[6], tr[((size_t)b * rounds + i + 2) * 8 + 4]};
            for (int p = 0; p < 7; ++p)
                if (from[p] && to[p] && to[p] >= from[p]) {
                    acc[p] += (double)(to[p] - from[p]);
                    cnt[p] += 1;
                }
            if (t[0] && u[0]) { pr += (double)(u[0] - t[0]); prn += 1; }
            if (t[4] && u[4]) { cr += (double)(u[4] - t[4]); crn += 1; }
        }
    printf("rounds %d, LDS %d B\n", rounds, LDS_BYTES);
    for (int p = 0; p < 7; ++p) printf("  %-40s %8.3f us\n", names[p], cnt[p] ? acc[p] / cnt[p] / 100.0 : 0.0);
    printf("  %-40s %8.3f us\n", "producer round", prn ? pr / prn / 100.0 : 0.0);
    printf("  %-40s %8.3f us\n", "consumer round", crn ? cr / crn / 100.0 : 0.0);
    const int mid = rounds / 2;
    unsigned long long lo = ~0ull, hi = 0, clo = ~0ull, chi = 0;
    for (int b = 0; b < NB; ++b) {
        lo = std::min(lo, tr[((size_t)b * rounds + mid) * 8]);
        hi = std::max(hi, tr[((size_t)b * rounds + mid) * 8]);
        clo = std::min(clo, tr[((size_t)b * rounds + mid) * 8 + 4]);
        chi = std::max(chi, tr[((size_t)b * rounds + mid) * 8 + 4]);
    }
    printf("  producer start skew at round %d: %.3f us; consumer %.3f us; consumer lag %.3f us\n", mid,
           (hi - lo) / 100.0, (chi - clo) / 100.0, ((double)clo - (double)lo) / 100.0);
    return 0;
}
