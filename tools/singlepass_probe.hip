// Measurement instrument (not product code): the single-pass C2 design — every kept row's sum and
// count added straight into a global 1M-group table with device-scope atomics, no staging — timed
// against the staged path ("the ceiling of the staged design").  Build:
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/singlepass_probe.hip -o tools/_singlepass.so
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

// dense keys 0 .. G-1 index the table directly (the best case for a single pass: no probing)
__global__ void __launch_bounds__(256) singlepass_kernel(const double *f, const int64_t *k, const double *v,
                                                         int64_t n, double t, double *sum,
                                                         unsigned long long *cnt) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        if (!(f[r] < t)) continue;
        const int64_t key = k[r];
        atomicAdd(&sum[key], v[r]);
        atomicAdd(&cnt[key], 1ull);
    }
}

} // namespace

extern "C" int sp_run(const double *f, const int64_t *k, const double *v, int64_t n, double t, double *sum,
                      unsigned long long *cnt, int64_t groups, int reps, float *ms_out) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 1;
    const unsigned grid = 256 * 16;
    float total = 0;
    for (int i = 0; i < reps; ++i) {
        if (hipMemsetAsync(sum, 0, groups * 8, 0) != hipSuccess) return 2;
        if (hipMemsetAsync(cnt, 0, groups * 8, 0) != hipSuccess) return 2;
        hipEventRecord(a, 0);
        hipLaunchKernelGGL(singlepass_kernel, dim3(grid), dim3(256), 0, 0, f, k, v, n, t, sum, cnt);
        hipEventRecord(b, 0);
        if (hipEventSynchronize(b) != hipSuccess) return 3;
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (i > 0) total += ms; // the first launch warms up
    }
    *ms_out = reps > 1 ? total / (reps - 1) : 0.f;
    hipEventDestroy(a);
    hipEventDestroy(b);
    return hipGetLastError() == hipSuccess ? 0 : 4;
}
