// agg_bucket_fast.hip — bucket kernel instantiations of the FastOps row policies (one 8-byte key
// without NULLs, count / sum Int64 / sum Float64 / sum Decimal64 -> Int128): the C2 hot path.
#include "agg_dev.h"

namespace tfg {

bool launch_bucket_fast(int fast, int B, const AggSpec &S, hipStream_t st, const RowsIO &rows, const RowsIO &rows1,
                        int mode, const uint64_t *stage_off, const GroupsIO &old, const uint64_t *ooff,
                        const GroupsIO &tmp, uint64_t *new_cnt) {
    return with_fast_ops(fast, [&](auto ops) {
        launch_bucket_one<typename decltype(ops)::type>(B, S, st, rows, rows1, mode, stage_off, old, ooff, tmp, new_cnt);
    });
}

} // namespace tfg
