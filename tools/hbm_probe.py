"""Streaming-bandwidth probe (torch copy / reduction) to calibrate what 'HBM-bound' means here."""
import torch, time
x = torch.empty(400_000_000, dtype=torch.int64, device="cuda").random_()
y = torch.empty_like(x)
for name, fn, b in [("copy", lambda: y.copy_(x), 2 * x.numel() * 8), ("sum", lambda: x.sum(), x.numel() * 8),
                    ("fill", lambda: y.fill_(3), x.numel() * 8)]:
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): fn()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{name}: {ms:.3f} ms  {b / ms / 1e6:.0f} GB/s")
