// agg_bucket_generic.hip — bucket kernel instantiations of GenericOps (any key width, nullable
// keys and arguments, partial states, Decimal256), and the dispatch to the wide-key family.
#include "agg_dev.h"

namespace tfg {

void launch_bucket_wide_generic(bool w256, int B, const AggSpec &S, hipStream_t st, const RowsIO &rows,
                                const RowsIO &rows1, int mode, const uint64_t *stage_off, const GroupsIO &old,
                                const uint64_t *ooff, const GroupsIO &tmp, uint64_t *new_cnt);

void launch_bucket_generic(bool wide, bool w256, int B, const AggSpec &S, hipStream_t st, const RowsIO &rows,
                           const RowsIO &rows1, int mode, const uint64_t *stage_off, const GroupsIO &old,
                           const uint64_t *ooff, const GroupsIO &tmp, uint64_t *new_cnt) {
    if (wide) {
        launch_bucket_wide_generic(w256, B, S, st, rows, rows1, mode, stage_off, old, ooff, tmp, new_cnt);
        return;
    }
#define TFG_GB(...) launch_bucket_one<__VA_ARGS__>(B, S, st, rows, rows1, mode, stage_off, old, ooff, tmp, new_cnt)
    if (w256) switch (S.n_aggs) {
        case 1: TFG_GB(GenericOps<1, true>); break;
        case 2: TFG_GB(GenericOps<2, true>); break;
        case 3: TFG_GB(GenericOps<3, true>); break;
        default: TFG_GB(GenericOps<4, true>); break;
        }
    else switch (S.n_aggs) {
        case 1: TFG_GB(GenericOps<1>); break;
        case 2: TFG_GB(GenericOps<2>); break;
        case 3: TFG_GB(GenericOps<3>); break;
        default: TFG_GB(GenericOps<4>); break;
        }
#undef TFG_GB
}

} // namespace tfg
