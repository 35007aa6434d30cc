// agg_bucket_fast_tiled.hip — the tiled bucket kernel (agg_bucket_tiled_kernel) of the FastOps row
// policies: the second kernel of the C2 filter -> GROUP BY step.
#include <cstdlib>

#include "agg_dev.h"

namespace tfg {

// TFG_AGG_BT768=1 (experiment): the one-workgroup-per-CU tables with 768 threads (12 waves: three
// per SIMD, so up to 168 VGPRs a lane) instead of 1024 (four per SIMD: 128 VGPRs, 19 spilled)
constexpr int BT_MID = 768;
bool launch_bucket_fast_tiled(int fast, int B, const AggSpec &S, hipStream_t st, const TiledIn &tin, int mode,
                              const GroupsIO &old, const uint64_t *ooff, const GroupsIO &tmp, uint64_t *new_cnt,
                              uint64_t *tmp_base) {
    static const bool mid = [] {
        const char *v = getenv("TFG_AGG_BT768");
        return v && *v == '1';
    }();
    return with_fast_ops(fast, [&](auto ops) {
        using Ops = typename decltype(ops)::type;
        if (mid && S.bt == BT_BIG) {
            hipLaunchKernelGGL((agg_bucket_tiled_kernel<Ops, BT_MID>), dim3(B), dim3(BT_MID), S.lds_bytes, st, S, tin,
                               mode, old, ooff, tmp, new_cnt, tmp_base);
            return;
        }
        launch_bucket_one_tiled<Ops>(B, S, st, tin, mode, old, ooff, tmp, new_cnt, tmp_base);
    });
}

} // namespace tfg
