#!/usr/bin/env python3
"""GPT-2 LM-head forward (8192 x 50304 x 768, N not a multiple of 256) on the 256 x 256 k64 tile:
the 196 whole 256-column panels in one launch plus the 128-column edge strip on a 256 x 128 tile,
both writing into one [T, V] output -- vs hipBLASLt (torch) and the best single k64 tile.

    python scripts/bench_head_split.py   -> one JSON line per variant (median of 20 timed calls)
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

C = native()
T, V, D = 8192, 50304, 768
x = torch.randn(T, D, device="cuda").bfloat16()
w = (torch.randn(V, D, device="cuda") * 0.02).bfloat16()
out = torch.empty(T, V, device="cuda", dtype=torch.bfloat16)
VB = (V // 256) * 256


def split(t_main: int, t_edge: int) -> torch.Tensor:
    C.gemm64(x, w[:VB], out=out[:, :VB], tile=t_main)
    C.gemm64(x, w[VB:], out=out[:, VB:], tile=t_edge)
    return out


variants = {
    "torch": lambda: x @ w.t(),
    "k64_t7": lambda: C.gemm64(x, w, out=out, tile=7)[0],
}
for tm in (5, 1):
    for te in (6, 2, 7):
        variants[f"split_t{tm}_t{te}"] = (lambda tm=tm, te=te: split(tm, te))
ref = (x.float() @ w.float().t())
for name, fn in variants.items():
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    y = fn()
    torch.cuda.synchronize()
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    us = ts[len(ts) // 2]
    print(json.dumps({"variant": name, "us": round(us, 1), "tf": round(2 * T * V * D / us / 1e6, 1),
                      "max_rel_err": round(err, 5)}), flush=True)
