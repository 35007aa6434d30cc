// agg_bucket_fast_tiled.hip — the tiled bucket kernel (agg_bucket_tiled_kernel) of the FastOps row
// policies: the second kernel of the C2 filter -> GROUP BY step.
#include "agg_dev.h"

namespace tfg {

bool launch_bucket_fast_tiled(int fast, int B, const AggSpec &S, hipStream_t st, const TiledIn &tin, int mode,
                              const GroupsIO &old, const uint64_t *ooff, const GroupsIO &tmp, uint64_t *new_cnt,
                              uint64_t *tmp_base) {
    return with_fast_ops(fast, [&](auto ops) {
        launch_bucket_one_tiled<typename decltype(ops)::type>(B, S, st, tin, mode, old, ooff, tmp, new_cnt, tmp_base);
    });
}

} // namespace tfg
