#!/usr/bin/env python3
"""Forward (x W^T, both K-major) GEMM shapes: the 4-wave W4 kernel (csrc/gemm_k64.hip tiles 9 / 10 = 4 / 5
LDS buffers) vs the 8-wave k64 tiles vs torch (hipBLASLt), interleaved rounds in one process, random
N(0,1) bf16 (rule 24/25).  One JSON line per shape, with the max relative error vs torch.

    python scripts/bench_w4.py [rounds]
"""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from bench_gemm64 import bench, relerr  # noqa: E402

from distributed_training_amd.ops import native  # noqa: E402

SHAPES = [  # (name, M, N, K)
    ("llama_o", 8192, 4096, 4096), ("llama_qkv", 8192, 6144, 4096), ("llama_gate_up", 8192, 28672, 4096),
    ("llama_down", 8192, 4096, 14336), ("sq8192", 8192, 8192, 8192), ("gpt2_fc", 8192, 3072, 768),
    ("gpt2_qkv", 8192, 2304, 768), ("gpt2_fc2", 8192, 768, 3072), ("gpt2_head_M", 8192, 50176, 768),
]


def main() -> None:
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    C = native()
    for name, M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        ref = F.linear(x, w)
        fns = {"torch": lambda: F.linear(x, w)}
        errs = {}
        for t in (5, 6, 3, 9, 10):
            if C.gemm64_tile(M, N, K, t):
                fns[f"t{t}"] = (lambda t=t: C.gemm64(x, w, tile=t)[0])
                errs[f"t{t}"] = float(f"{relerr(fns[f't{t}'](), ref):.2e}")
        times = bench(fns, rounds)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "us": {k: round(v, 1) for k, v in times.items()},
                          "TF": {k: round(fl / v / 1e6) for k, v in times.items()}, "relerr": errs}), flush=True)
        del x, w, ref
    # epilogues on W4: bias, GELU dual store, residual
    M, N, K = 8192, 3072, 768
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    b = (torch.randn(N, device="cuda") * 0.1).bfloat16()
    res = torch.randn(M, N, device="cuda").bfloat16()
    h = torch.addmm(b, x, w.t())
    out = {}
    for t in (9, 10):
        hh, aa = C.gemm64(x, w, bias=b, epi=2, out=torch.empty_like(h), out2=torch.empty_like(h), tile=t)
        rr = C.gemm64(x, w, epi=32, res=res, tile=t)[0]
        out[f"t{t}"] = {"bias": relerr(hh, h), "gelu": relerr(aa, F.gelu(hh.float(), approximate="tanh")),
                        "res": relerr(rr, (x @ w.t()) + res)}
    print(json.dumps({"epilogues": out}), flush=True)


if __name__ == "__main__":
    main()
