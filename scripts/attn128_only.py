#!/usr/bin/env python3
"""Llama-3-8B-shape flash attention (B 1, S 8192, H 32 / Hkv 8, D 128, causal) forward and backward only,
10 calls each: a short target for rocprofv3 --pmc passes (scripts/gpu.sh pmc)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

B, S, H, HKV, D = 1, 8192, 32, 8, 128
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
k = torch.randn(B, S, HKV, D, device=dev, dtype=torch.bfloat16, generator=g)
v = torch.randn(B, S, HKV, D, device=dev, dtype=torch.bfloat16, generator=g)
do = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
C = native()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    o, lse = C.attn_fwd(q, k, v, True, D ** -0.5, -1)
    C.attn_bwd(do, q, k, v, o, lse, True, D ** -0.5, -1)
torch.cuda.synchronize()
