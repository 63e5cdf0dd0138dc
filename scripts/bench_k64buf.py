#!/usr/bin/env python3
"""csrc/gemm_k64.hip LDS-DMA through flat global_load_lds (tile t | 32) vs buffer descriptors (tile t, the
default: 32-bit lane offsets, scalar K-step), same tiles, interleaved rounds in one process on random bf16
(cdna_hip_programming.md rules 24 / 25); one JSON line per (shape, layout, tile).

    python scripts/bench_k64buf.py [rounds]
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from bench_gemm64 import bench, relerr  # noqa: E402

from distributed_training_amd.ops import native  # noqa: E402

SHAPES = [("llama_o", 8192, 4096, 4096), ("llama_gate_up", 8192, 28672, 4096), ("llama_down", 8192, 4096, 14336),
          ("gpt2_fc", 8192, 3072, 768), ("gpt2_qkv", 8192, 2304, 768), ("gpt2_fc_w", 3072, 768, 8192)]
LAYOUTS = {"nt": (False, False), "nn": (False, True), "tn": (True, True)}


def main() -> None:
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    C = native()
    for name, M, N, K in SHAPES:
        for lay, (a_t, b_t) in LAYOUTS.items():
            a = (torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")).bfloat16()
            b = ((torch.randn(K, N, device="cuda") if b_t else torch.randn(N, K, device="cuda")) * 0.02).bfloat16()
            ref = (a.float().t() if a_t else a.float()) @ (b.float() if b_t else b.float().t())
            for t in (5, 6, 7, 8):
                if not C.gemm64_tile(M, N, K, t):
                    continue
                fns = {"flat": (lambda t=t: C.gemm64(a, b, a_t, b_t, tile=t | 32)[0]),
                       "buf": (lambda t=t: C.gemm64(a, b, a_t, b_t, tile=t)[0])}
                err = {k: float(f"{relerr(f(), ref):.2e}") for k, f in fns.items()}
                us = bench(fns, rounds)
                fl = 2.0 * M * N * K
                print(json.dumps({"shape": name, "layout": lay, "tile": t, "us": {k: round(v, 1) for k, v in us.items()},
                                  "TF": {k: round(fl / v / 1e6) for k, v in us.items()},
                                  "buf_speedup": round(us["flat"] / us["buf"], 3), "relerr": err}), flush=True)
            del a, b, ref


if __name__ == "__main__":
    main()
