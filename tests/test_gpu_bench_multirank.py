"""Rehearsal of bench.py's N > 1 legs on the one GPU of a test box, so the driver's 8-GPU run
never meets an untested path: `bench.py --gpus 2 --dist-backend gloo` starts two ranks through
torch.distributed.run (the same launcher the driver uses), both on cuda:0, at reduced sizes, with
every N > 1 leg on — C2 two-phase (partial -> hash repartition -> exchange -> final), the C4
repartitioned join (both sides repartitioned, one fused exchange) and C5 two-phase String GROUP BY
(packed keys through the exchange) — and checks every leg's global invariant (`check.ok`: each kept
row counted once over all ranks, every probe row probed once, C5 counts = rows).  The reference
runs every MPP test at 1..N servers the same way (TestUtils/MPPTaskTestUtils.h:150-160).  gloo moves
host memory only, so the exchange stages the device columns through the host here; the production
backend (RCCL) exchanges device buffers with the same calls above it."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_gloo_all_legs():
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--steps", "2", "--warmup", "1", "--rows", "4000000", "--groups", "50000",
           "--join-build", "400000", "--join-probe", "4000000", "--c4", "1",
           "--c5-rows", "4000000", "--c5-groups", "400000", "--codec-rows", "0", "--no-cpu", "--no-variants"]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240)
    assert p.returncode == 0, f"bench --gpus 2 failed:\n{p.stderr[-4000:]}"
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, f"expected one JSON line from rank 0, got:\n{p.stdout[-2000:]}"
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["dist_backend"] == "gloo"
    assert d["check"]["ok"], d["check"]
    assert d["check"]["kept_total"] > 0
    for leg in ("repartitioned_join", "string_agg"):
        assert leg in d, f"leg {leg} missing from the N>1 line: {sorted(d)}"
        assert d[leg]["check"]["ok"], (leg, d[leg]["check"])
