#!/usr/bin/env python3
"""Run one GEMM shape repeatedly -- a target for rocprofv3 --pmc / --kernel-trace.

    python scripts/gemm_one.py M N K [layout] [impls]
layout: nt (forward x W^T), nn (dgrad dy W), tn (wgrad dy^T x); impls: comma list of
torch, k64 (csrc/gemm_k64.hip auto tile) or k64tN (tiles 9 / 10: csrc/gemm_w4.hip)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
layout = sys.argv[4] if len(sys.argv) > 4 else "nt"
impls = (sys.argv[5] if len(sys.argv) > 5 else "torch,k64").split(",")
a_t, b_t = {"nt": (False, False), "nn": (False, True), "tn": (True, True)}[layout]
a = (torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")).bfloat16()
b = ((torch.randn(K, N, device="cuda") if b_t else torch.randn(N, K, device="cuda")) * 0.02).bfloat16()
C = native()


def run(impl):
    if impl == "torch":
        return (a.t() if a_t else a) @ (b if b_t else b.t())
    tile = int(impl[4:]) if impl.startswith("k64t") else 0
    return C.gemm64(a, b, a_t, b_t, tile=tile)[0]


for _ in range(10):
    for impl in impls:
        run(impl)
torch.cuda.synchronize()
