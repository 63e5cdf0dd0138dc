#!/usr/bin/env python3
"""Weight + bias gradient (dW = dy^T x, db = sum_t dy) on the GPT-2 small / Llama-3 8B
shapes: the 128x128 split-K kernel (csrc/gemm.hip, tile 0) against the general GEMM's
256x256 / 256x128 tiles with split-K and the bias gradient on the MFMA pipe
(csrc/gemm_bf16.hip dta_gemm_wgrad, tiles 1 / 2), over a range of splits; every
variant checked against fp32 torch first.  One JSON line per shape."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

SHAPES = [(8192, 2304, 768), (8192, 768, 768), (8192, 3072, 768), (8192, 768, 3072),
          (8192, 6144, 4096), (8192, 4096, 4096)]


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
    return s.elapsed_time(e) / reps * 1e3


def main():
    C = native()
    torch.manual_seed(0)
    for K, M, N in SHAPES:
        a = torch.randn(K, M, device="cuda").bfloat16()
        b = torch.randn(K, N, device="cuda").bfloat16()
        ref = a.float().t() @ b.float()
        refb = a.float().sum(0)
        fl = 2.0 * K * M * N
        row = {"K": K, "M": M, "N": N}
        row["torch_us"] = round(timeit(lambda: (torch.mm(a.t(), b), a.sum(0))), 1)
        cands = [(0, 0)]
        for tile in (1, 2):
            sp0 = C.gemm_wgrad_split(M, N, K, tile)
            if not sp0:
                continue
            for sp in sorted({1, 2, 3, 4, 6, 8, 12, 16, sp0}):
                if sp <= 4 * sp0 and K // 32 // sp >= 8:
                    cands.append((tile, sp))
        for tile, sp in cands:
            dw, db = C.gemm_tn_colsum(a, b, False, sp, -1, None, None, tile)
            err = ((dw.float() - ref).abs().max() / ref.abs().max()).item()
            errb = ((db.float() - refb).abs().max() / refb.abs().max()).item()
            if err > 1e-2 or errb > 1e-2:
                row[f"t{tile}s{sp}_BAD"] = [round(err, 5), round(errb, 5)]
                continue
            t = timeit(lambda: C.gemm_tn_colsum(a, b, False, sp, -1, None, None, tile))
            row[f"t{tile}s{sp}"] = round(t, 1)
        best = min((v, k) for k, v in row.items() if k.startswith("t") and not k.endswith("BAD")
                   and isinstance(v, float) and k != "torch_us")
        row["best"] = best[1]
        row["best_TF"] = round(fl / best[0] / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
