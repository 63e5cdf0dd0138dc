#!/usr/bin/env python3
"""Flat AdamW (csrc/optim.hip) on N fp32 master parameters with bf16 gradients and a bf16 copy-out:
28 B of HBM traffic per parameter.  Prints the median time and the achieved bandwidth.

    python scripts/bench_adam.py [n=1e9]
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
C = native()
p, m, v = (torch.zeros(n, device="cuda") for _ in range(3))
g = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
pb = torch.empty(n, device="cuda", dtype=torch.bfloat16)
step = torch.zeros(1, device="cuda")


def run():
    C.flat_adam(p, g, m, v, None, pb, step, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1.0, True, False, False, True, -1, 0)


for _ in range(3):
    run()
torch.cuda.synchronize()
ts = []
for _ in range(10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    run()
    b.record()
    b.synchronize()
    ts.append(a.elapsed_time(b))
ts.sort()
ms = ts[len(ts) // 2]
print(json.dumps({"n": n, "ms": round(ms, 3), "TB_s": round(28 * n / ms / 1e9, 2)}), flush=True)
