"""Probe (diagnostic only): HBM write-only, read-only and copy bandwidth on one GPU."""
import torch

def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3

n = 8 << 30  # bytes
x = torch.empty(n // 8, dtype=torch.int64, device="cuda")
y = torch.empty(n // 8, dtype=torch.int64, device="cuda")
x.fill_(3)
w = t(lambda: y.fill_(7))
r = t(lambda: x.sum())
c = t(lambda: y.copy_(x))
print(f"write {n / w / 1e12:.2f} TB/s  read {n / r / 1e12:.2f} TB/s  copy {2 * n / c / 1e12:.2f} TB/s")
