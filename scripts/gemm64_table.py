#!/usr/bin/env python3
"""Text table of scripts/bench_gemm64.py JSON lines (optionally side by side with an earlier run)."""
import json
import sys


def load(p):
    return [json.loads(l) for l in open(p) if l.startswith("{")]


rows = load(sys.argv[1])
old = {(r["model"], r["gemm"], r["kind"]): r for r in load(sys.argv[2])} if len(sys.argv) > 2 else {}
for r in rows:
    us = r["us"]
    best = r.get("k64_best")
    prev = old.get((r["model"], r["gemm"], r["kind"]))
    extra = ""
    if prev and prev.get("k64_best"):
        extra = f"  (before: {prev['us'][prev['k64_best']]} us)"
    if best:
        print(f'{r["model"]:6s} {r["gemm"]:8s} {r["kind"]:6s} M{r["M"]:7d} N{r["N"]:7d} K{r["K"]:7d}  torch {us["torch"]:8.1f} us '
              f'({r["TF"]["torch"]:5d} TF)  k64 {best[4:]} {us[best]:8.1f} us ({r["TF"][best]:5d} TF)  '
              f'torch/k64 {r["torch_over_k64"]:.3f}{extra}')
    else:
        print(f'{r["model"]:6s} {r["gemm"]:16s} {r["kind"]:12s} ' + "  ".join(f"{k} {v}" for k, v in us.items()))
