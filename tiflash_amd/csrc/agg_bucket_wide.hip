// agg_bucket_wide.hip — bucket kernel instantiations of the wide-key row policies (16-byte packed
// keys128 / key_string keys): WideFastOps on the tiled path (C5), WideOps on the general path.
#include "agg_dev.h"

namespace tfg {

bool launch_bucket_wide_tiled(int code, int B, const AggSpec &S, hipStream_t st, const TiledIn &tin, int mode,
                              const GroupsIO &old, const uint64_t *ooff, const GroupsIO &tmp, uint64_t *new_cnt,
                              uint64_t *tmp_base) {
    auto go = [&](auto tag) {
        using Ops = typename decltype(tag)::type;
        if (S.bt == BT_QUAD) // four 256-thread workgroups per CU (TFG_WIDE_QUAD)
            hipLaunchKernelGGL((agg_bucket_tiled_kernel<Ops, BT_QUAD>), dim3(B), dim3(BT_QUAD), S.lds_bytes, st, S, tin,
                               mode, old, ooff, tmp, new_cnt, tmp_base);
        else
            launch_bucket_one_tiled<Ops>(B, S, st, tin, mode, old, ooff, tmp, new_cnt, tmp_base);
        return true;
    };
    switch (code) {
    case 410: return go(OpsTag<WideFastOps<4, 1, 0>>{});
    case 310: return go(OpsTag<WideFastOps<3, 1, 0>>{});
    case 210: return go(OpsTag<WideFastOps<2, 1, 0>>{});
    case 140: return go(OpsTag<WideFastOps<1, 4, 0>>{});
    case 130: return go(OpsTag<WideFastOps<1, 3, 0>>{});
    case 120: return go(OpsTag<WideFastOps<1, 2, 0>>{});
    case 400: return go(OpsTag<WideFastOps<4, 0, 0>>{});
    case 300: return go(OpsTag<WideFastOps<3, 0, 0>>{});
    case 200: return go(OpsTag<WideFastOps<2, 0, 0>>{});
    case 100: return go(OpsTag<WideFastOps<1, 0, 0>>{});
    default: return false;
    }
}

void launch_bucket_wide_generic(bool w256, int B, const AggSpec &S, hipStream_t st, const RowsIO &rows,
                                const RowsIO &rows1, int mode, const uint64_t *stage_off, const GroupsIO &old,
                                const uint64_t *ooff, const GroupsIO &tmp, uint64_t *new_cnt) {
#define TFG_WB(...) launch_bucket_one<__VA_ARGS__>(B, S, st, rows, rows1, mode, stage_off, old, ooff, tmp, new_cnt)
    if (w256) switch (S.n_aggs) {
        case 1: TFG_WB(WideOps<1, true>); break;
        case 2: TFG_WB(WideOps<2, true>); break;
        case 3: TFG_WB(WideOps<3, true>); break;
        default: TFG_WB(WideOps<4, true>); break;
        }
    else switch (S.n_aggs) {
        case 1: TFG_WB(WideOps<1>); break;
        case 2: TFG_WB(WideOps<2>); break;
        case 3: TFG_WB(WideOps<3>); break;
        default: TFG_WB(WideOps<4>); break;
        }
#undef TFG_WB
}

} // namespace tfg
