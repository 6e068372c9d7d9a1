"""Achievable HBM rates on this box for context: a 1 GiB device-to-device copy (torch), a
0.9 GiB copy (the front-end writer's shape) and a 1 GiB read (int64 sum), timed with HIP
events."""
import torch

def timed(fn, k=20):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(k):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / k

n = 1 << 30
x = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
y = torch.empty_like(x)
for name, m in (("copy 1 GiB", n), ("copy 0.9 GiB", int(0.9 * n))):
    ms = timed(lambda: y[:m].copy_(x[:m]))
    print(f"{name}: {ms:.4f} ms  {2 * m / ms / 1e6:.0f} GB/s (read + write)")
xs = x.view(torch.int64)
ms = timed(lambda: xs.sum())
print(f"read 1 GiB (int64 sum): {ms:.4f} ms  {n / ms / 1e6:.0f} GB/s")
