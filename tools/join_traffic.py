"""C3 probe traffic attribution: the bench's join (10M build x 100M probe, Int64 keys) probed once
per variant, so a rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE pass over join_probe_kernel can split
the kernel's HBM reads by what it touches.

  full     probe payload [key, ppay] + 1 build payload word (the bench's probe)
  nobuild  probe payload [key, ppay], a build side without payload (key-only build records)
  miss     the full probe over probe keys that never match (no output at all)

usage: python3 tools/join_traffic.py <variant> [--build N --probe N]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variant", choices=["full", "nobuild", "miss"])
    ap.add_argument("--build", type=int, default=10_000_000)
    ap.add_argument("--probe", type=int, default=100_000_000)
    a = ap.parse_args()
    import torch
    import tiflash_amd as tfa
    dev = torch.device("cuda:0")
    ctx = tfa.Context(0)
    nb, npr = a.build, a.probe
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    bk = torch.randperm(nb, device=dev, generator=g).to(torch.int64) * 4 + 1
    bpay = torch.randint(0, 1 << 40, (nb,), device=dev, generator=g, dtype=torch.int64)
    hit = torch.rand(npr, device=dev, generator=g) < (0.0 if a.variant == "miss" else 0.5)
    pk = torch.where(hit, bk[torch.randint(0, nb, (npr,), device=dev, generator=g)],
                     torch.randint(0, 1 << 40, (npr,), device=dev, generator=g) * 4 + 3)
    ppay = torch.randint(0, 1 << 40, (npr,), device=dev, generator=g, dtype=torch.int64)
    del hit
    j = tfa.Join(ctx, tfa.INT64, expected_build_rows=nb)
    j.build(bk, payload=[] if a.variant == "nobuild" else [bpay])
    j.finalize()
    cap = npr
    bw = 0 if a.variant == "nobuild" else 1
    outs = ([torch.empty(cap, dtype=torch.int64, device=dev) for _ in range(2)],
            [torch.empty(cap, dtype=torch.int64, device=dev) for _ in range(bw)],
            torch.empty(cap, dtype=torch.uint8, device=dev))
    for _ in range(2):
        op, ob, _ = j.probe_rows(pk, [pk, ppay], bw, capacity=cap, outs=outs)
    torch.cuda.synchronize()
    print(f"variant {a.variant}: matches {op[0].shape[0]}", flush=True)
    j.close()


if __name__ == "__main__":
    main()
