"""HBM bandwidth probe: torch copy (read+write) vs the flat AdamW kernel (28 B/param) at GPT-2 size."""
import torch

from distributed_training_amd.ops import native

dev = torch.device("cuda", 0)


def t_us(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


n = 124_475_904
a = torch.empty(n * 4, dtype=torch.uint8, device=dev)
b = torch.empty_like(a)
us = t_us(lambda: b.copy_(a))
print(f"copy {n * 4 / 1e6:.0f} MB: {us:.1f} us -> {2 * n * 4 / us / 1e6:.2f} TB/s (read+write)")
p = torch.randn(n, device=dev)
g = torch.randn(n, device=dev).bfloat16()
m = torch.zeros(n, device=dev)
v = torch.zeros(n, device=dev)
pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
step = torch.zeros(1, device=dev)
C = native()
us = t_us(lambda: C.flat_adam(p, g, m, v, None, pb, step, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1.0, True, False, False, True, -1))
print(f"flat_adam {n} params: {us:.1f} us -> {28 * n / us / 1e6:.2f} TB/s")
