#!/usr/bin/env python3
"""Why the k64 256 x 256 tile (id 5) loses to hipBLASLt on the forward (NT: both operands K-major) layout
while it wins the NN / TN layouts of the same M N K: time one Llama-sized product in every layout, and the
NT layout again with padded row pitches (K + pad elements: a different HBM channel / L2 set walk for the
8-rows-of-128-B DMA pieces), against torch (hipBLASLt).  hipEvent medians, interleaved rounds.

    python scripts/gemm_layout_probe.py [M N K] [rounds]
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (8192, 28672, 4096)
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
C = native()
dev = torch.device("cuda", 0)


def padded(rows, cols, pad, scale=1.0):
    base = (torch.randn(rows, cols + pad, device=dev) * scale).bfloat16()
    return base[:, :cols]


def case(layout, pad):
    a_t, b_t = {"nt": (False, False), "nn": (False, True), "tn": (True, True)}[layout]
    a = padded(K, M, pad) if a_t else padded(M, K, pad)
    b = padded(K, N, pad, 0.02) if b_t else padded(N, K, pad, 0.02)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    k64 = lambda: C.gemm64(a, b, a_t, b_t, out=out, tile=5)  # noqa: E731
    lib = lambda: torch.matmul(a.t() if a_t else a, b if b_t else b.t(), out=out)  # noqa: E731
    return {"k64/t5": k64, "torch": lib}


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


cases = [("nt", 0), ("nn", 0), ("tn", 0), ("nt", 64), ("nt", 128), ("nt", 8)]
res = {}
for r in range(rounds):
    for layout, pad in cases:
        for impl, fn in case(layout, pad).items():
            us = timeit(fn)
            res.setdefault((layout, pad, impl), []).append(us)
            torch.cuda.empty_cache()
flop = 2.0 * M * N * K
for (layout, pad, impl), v in res.items():
    us = sorted(v)[len(v) // 2]
    print(json.dumps({"M": M, "N": N, "K": K, "layout": layout, "pad": pad, "impl": impl, "us": round(us, 1),
                      "tflops": round(flop / us / 1e6, 1), "rounds": [round(x, 1) for x in v]}))
