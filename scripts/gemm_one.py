#!/usr/bin/env python3
"""Run one GEMM shape repeatedly (dta tile N and torch) -- a target for rocprofv3 --pmc."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
tile = int(sys.argv[4]) if len(sys.argv) > 4 else 0
x = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
for _ in range(5):
    native().gemm(x, w, tile=tile)
    F.linear(x, w)
torch.cuda.synchronize()
