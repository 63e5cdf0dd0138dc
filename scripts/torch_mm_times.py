"""hipBLASLt (torch.mm, bf16, random operands) times for the GEMM shapes of scripts/k64_epi_diag.hip:
y[M, N] = x[M, K] W[N, K]^T, median of 7 rounds -- the library reference for the diagnostic builds."""
import json

import torch

SHAPES = [(8192, 4096, 4096), (8192, 6144, 4096), (8192, 28672, 4096), (8192, 4096, 14336), (8192, 3072, 768),
          (8192, 128256, 4096), (16384, 4096, 4096)]
for M, N, K in SHAPES:
    a = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
    w = (torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1) * 0.02
    reps = max(2, int(2e5 / (2 * M * N * K / 1.3e15 * 1e6)))
    for _ in range(3):
        torch.mm(a, w.t())
    ts = []
    for _ in range(7):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            torch.mm(a, w.t())
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / reps)
    t = sorted(ts)[3]
    print(json.dumps({"lib": "hipblaslt", "M": M, "N": N, "K": K, "us": round(t, 1), "tf": round(2 * M * N * K / t * 1e-6)}),
          flush=True)
