"""Filters that keep (almost) nothing: after a consume that kept fewer rows than it had tiles, the
next tiled consume checks all-false tiles with vector loads of the predicate column (partition.h
VSKIP).  Both forms must give the oracle's groups exactly: an all-false batch, then batches that
keep a few scattered rows, one whole tile and the last rows, with aligned and misaligned
predicate columns of Int64 / Int32 / Float64.  Reference: FilterTransformAction.cpp:134-138
(all-false blocks skipped), Aggregator.cpp:852-1024."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _expect(f, k, v, thr):
    m = f < thr
    ks, vs = k[m], v[m]
    out = {}
    for kk, vv in zip(ks.tolist(), vs.tolist()):
        s, c = out.get(kk, (0.0, 0))
        out[kk] = (s + vv, c + 1)
    return out


def _got(res):
    keys = res["keys"].cpu().numpy()
    s = res["states"][0].cpu().numpy()
    c = res["states"][1].view(torch.int64).cpu().numpy()
    return {int(a): (float(b), int(cc)) for a, b, cc in zip(keys, s, c)}


@pytest.mark.parametrize("ptype", ["int64", "int32", "float64"])
@pytest.mark.parametrize("misalign", [0, 1])
def test_sparse_filter_after_all_false(tfa, ctx, dev, ptype, misalign):
    rng = np.random.default_rng(17 + misalign)
    n = 3_000_000
    k = rng.integers(0, 50_000, n).astype(np.int64)
    v = (rng.integers(0, 1 << 20, n) / 64.0).astype(np.float64)
    npt = {"int64": np.int64, "int32": np.int32, "float64": np.float64}[ptype]
    tp = {"int64": tfa.INT64, "int32": tfa.INT32, "float64": tfa.FLOAT64}[ptype]
    base = np.full(n + misalign, 100, dtype=npt)
    agg = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)])
    kd, vd = torch.from_numpy(k).to(dev), torch.from_numpy(v).to(dev)

    def run(fh):
        full = np.concatenate([np.full(misalign, 100, dtype=npt), fh]) if misalign else fh
        fd = torch.from_numpy(full).to(dev)[misalign:]
        agg.reset()
        agg.consume_filtered(fd, tfa.LT, 50, kd, [vd, None], pred_type=tp)
        return _got(agg.result())

    f0 = base[:n].copy()
    assert run(f0) == {}  # all false: nothing kept
    assert run(f0) == {}  # again, now on the sparse (vector-check) form
    f1 = f0.copy()
    f1[rng.integers(0, n, 40)] = 7          # scattered rows
    f1[16384:16384 + 8192] = 3              # a whole tile's worth
    f1[-5:] = 1                             # the last rows (partial tile)
    assert run(f1) == _expect(f1, k, v, 50)  # sparse form (the previous batch kept nothing)
    assert run(f1) == _expect(f1, k, v, 50)
    f2 = (rng.integers(0, 100, n)).astype(npt)
    assert run(f2) == _expect(f2, k, v, 50)  # dense again
    agg.close()
