#!/usr/bin/env python3
"""The GPT-2 MLP's fused GEMM epilogues at 8192 x 3072 x 768: the up-projection with the GELU dual store
(h and gelu(h)) and the input gradient through the GELU (x gelu'(h)) -- each csrc/gemm_k64.hip tile with
the LDS-staged epilogue and with the per-fragment one (tile | 128), vs hipBLASLt + the separate
elementwise kernel, and the plain GEMM for reference.  Median of interleaved rounds (us).

    python scripts/bench_fused_epi.py
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402
from distributed_training_amd.ops.lm import _time_us  # noqa: E402

C = native()
T, F, D = 8192, 3072, 768
x = torch.randn(T, D, device="cuda").bfloat16()
w1 = (torch.randn(F, D, device="cuda") * 0.05).bfloat16()
b1 = torch.randn(F, device="cuda").bfloat16()
h = torch.randn(T, F, device="cuda").bfloat16()
dy = torch.randn(T, D, device="cuda").bfloat16()
w2 = (torch.randn(D, F, device="cuda") * 0.05).bfloat16()  # fc2 weight [D, F]: dh = dy W2 (NN, b N-major)
oh, oa = torch.empty(T, F, device="cuda").bfloat16(), torch.empty(T, F, device="cuda").bfloat16()

fwd = {"torch+gelu": lambda: C.gelu_fwd(torch.addmm(b1, x, w1.t()), -1)}
bwd = {"torch*dgelu": lambda: C.gelu_bwd(dy @ w2, h, -1)}
for t in (3, 7, 5, 6, 8):
    for bits in (0, 128):
        fwd[f"k64_t{t | bits}"] = (lambda t=t | bits: C.gemm64(x, w1, False, False, oh, oa, False, 1.0, b1, 2, None, t))
        bwd[f"k64_t{t | bits}"] = (lambda t=t | bits: C.gemm64(dy, w2, False, True, oh, None, False, 1.0, None, 16, h, t))
    fwd[f"plain_t{t}"] = (lambda t=t: C.gemm64(x, w1, tile=t))
    bwd[f"plain_t{t}"] = (lambda t=t: C.gemm64(dy, w2, False, True, tile=t))
for name, fns in (("fc_fwd_gelu_dual", fwd), ("fc2_dgrad_dgelu", bwd)):
    print(json.dumps({"gemm": name, "M": T, "N": F, "K": D,
                      "us": {k: round(v, 1) for k, v in _time_us(fns, rounds=7, reps=8).items()}}), flush=True)
