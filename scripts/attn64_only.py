#!/usr/bin/env python3
"""GPT-2-shape flash attention (B 8, S 1024, H 12, D 64, causal) forward and backward
only, 20 calls each: a short target for rocprofv3 --pmc passes."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

B, S, H, D = 8, 1024, 12, 64
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
q, k, v, do = (torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g) for _ in range(4))
C = native()
for _ in range(20):
    o, lse = C.attn_fwd(q, k, v, True, D ** -0.5, -1)
    C.attn_bwd(do, q, k, v, o, lse, True, D ** -0.5, -1)
torch.cuda.synchronize()
