#!/usr/bin/env python3
"""Weight-gradient GEMM (C = A^T B, K = tokens): native split-K MFMA kernel vs
torch.mm (hipBLASLt) on the GPT-2 small / Llama-3 8B shapes."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

SHAPES = [  # (K tokens, M = out features, N = in features)
    (8192, 2304, 768), (8192, 768, 768), (8192, 3072, 768), (8192, 768, 3072),
    (8192, 6144, 4096), (8192, 4096, 4096), (8192, 28672, 4096), (8192, 4096, 14336),
]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def linear_shapes():
    """Forward (y = x W^T) and input-gradient (dx = dy W) GEMMs of GPT-2 small on hipBLASLt."""
    for T, out_f, in_f in [(8192, 2304, 768), (8192, 768, 768), (8192, 3072, 768), (8192, 768, 3072),
                           (8192, 50304, 768)]:
        x = torch.randn(T, in_f, device="cuda").bfloat16()
        w = torch.randn(out_f, in_f, device="cuda").bfloat16()
        dy = torch.randn(T, out_f, device="cuda").bfloat16()
        fl = 2.0 * T * out_f * in_f
        tf = timeit(lambda: torch.mm(x, w.t()))
        tb = timeit(lambda: torch.mm(dy, w))
        print(json.dumps({"T": T, "out": out_f, "in": in_f, "fwd_us": round(tf, 1), "fwd_TF": round(fl / tf / 1e6, 1),
                          "dgrad_us": round(tb, 1), "dgrad_TF": round(fl / tb / 1e6, 1)}), flush=True)


def main():
    if "--no-linear" not in sys.argv:
        linear_shapes()
    C = native()
    for K, M, N in SHAPES:
        a = torch.randn(K, M, device="cuda").bfloat16()
        b = torch.randn(K, N, device="cuda").bfloat16()
        fl = 2.0 * K * M * N
        t_ref = timeit(lambda: torch.mm(a.t(), b))
        row = {"K": K, "M": M, "N": N, "torch_us": round(t_ref, 1), "torch_TF": round(fl / t_ref / 1e6, 1)}
        for sp in (1, 2, 4, 8):  # register-staged split-K kernel
            if (K // 64) % sp:
                continue
            t = timeit(lambda: C.gemm_tn(a, b, False, -sp))
            row[f"reg_s{sp}_us"] = round(t, 1)
        tiles = (M // 128) * (N // 128)
        for sp in sorted({1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 32}):  # LDS-DMA kernel
            if sp > 1 and tiles * sp > 4096:
                continue
            t = timeit(lambda: C.gemm_tn(a, b, False, sp))
            row[f"gd_s{sp}_us"] = round(t, 1)
        row["gd_auto_split"] = C.gemm_tn_split(M, N, K)
        t = timeit(lambda: C.gemm_tn(a, b, False, 0))
        row["gd_auto_us"] = round(t, 1)
        t = timeit(lambda: C.gemm_tn_colsum(a, b, False, 0))
        row["gd_auto_colsum_us"] = round(t, 1)
        best = min(v for k, v in row.items() if k.endswith("_us") and not k.startswith("torch") and "colsum" not in k)
        row["native_best_TF"] = round(fl / best / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
