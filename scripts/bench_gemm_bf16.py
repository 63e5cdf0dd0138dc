#!/usr/bin/env python3
"""dta general bf16 GEMM (csrc/gemm_bf16.hip) vs torch (hipBLASLt) on the GPT-2
small and Llama-3 8B projection shapes: forward (x W^T), input gradient (dy W),
weight gradient (dy^T x).  Random N(0,1) bf16 operands (never zeros: DVFS
inflates zero-filled runs).  One JSON line per (shape, kind, tile)."""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

T = 8192
MODELS = {
    "gpt2": [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072), ("head", 50304, 768)],
    "llama": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
              ("head", 128256, 4096)],
}


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    models = sys.argv[1].split(",") if len(sys.argv) > 1 else ["gpt2", "llama"]
    C = native()
    for model in models:
        for name, nout, nin in MODELS[model]:
            x = torch.randn(T, nin, device="cuda").bfloat16()
            w = (torch.randn(nout, nin, device="cuda") * 0.02).bfloat16()
            dy = torch.randn(T, nout, device="cuda").bfloat16()
            fl = 2.0 * T * nout * nin
            cases = {
                "fwd": (lambda: F.linear(x, w), (T, nout, nin), lambda tile: C.gemm(x, w, tile=tile)),
                "dgrad": (lambda: torch.mm(dy, w), (T, nin, nout), lambda tile: C.gemm(dy, w, False, True, tile=tile)),
                "wgrad": (lambda: torch.mm(dy.t(), x), (nout, nin, T),
                          lambda tile: C.gemm(dy, x, True, True, tile=tile)),
            }
            for kind, (tfn, (M, N, K), dfn) in cases.items():
                ref = tfn()
                row = {"model": model, "gemm": name, "kind": kind, "M": M, "N": N, "K": K,
                       "torch_us": round(timeit(tfn), 1)}
                row["torch_TF"] = round(fl / row["torch_us"] / 1e6, 1)
                auto = C.gemm_tile(M, N, K, 0)
                row["auto_tile"] = auto
                for tile in (1, 2, 3):
                    if not C.gemm_tile(M, N, K, tile):
                        continue
                    got = dfn(tile)
                    err = (got.float() - ref.float()).abs().max().item() / max(ref.float().abs().max().item(), 1e-6)
                    us = timeit(lambda: dfn(tile))
                    row[f"t{tile}_us"] = round(us, 1)
                    row[f"t{tile}_TF"] = round(fl / us / 1e6, 1)
                    row[f"t{tile}_relerr"] = float(f"{err:.2e}")
                print(json.dumps(row), flush=True)
                del ref


if __name__ == "__main__":
    main()
