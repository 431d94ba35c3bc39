"""Achievable HBM rate on this box for the access mixes of the memory-bound passes: a bf16 copy
(1 read : 1 write) and a 1 read : 3 write fan-out, 200-400 MB footprints, timed with HIP events."""
import torch
x = torch.randn(16 * 224 * 224 * 64, device="cuda").to(torch.bfloat16)
ys = [torch.empty_like(x) for _ in range(3)]
def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3
b = x.numel() * 2
us = t(lambda: ys[0].copy_(x))
print(f"copy {b*2/1e6:.0f} MB: {us:.1f} us {b*2/us/1e3:.0f} GB/s")
def fan():
    for y in ys:
        y.copy_(x)
us = t(fan)
print(f"3 copies {b*6/1e6:.0f} MB: {us:.1f} us {b*6/us/1e3:.0f} GB/s")
