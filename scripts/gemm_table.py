#!/usr/bin/env python3
"""Summarise scripts/bench_gemm_bf16.py output: best dta tile vs torch per shape."""
import json
import sys

for l in open(sys.argv[1]):
    if not l.startswith('{"model'):
        continue
    d = json.loads(l)
    tiles = [(d[k], k[:2]) for k in d if k.startswith("t") and k.endswith("_us") and k != "torch_us"]
    us, t = min(tiles)
    fl = 2 * d["M"] * d["N"] * d["K"]
    print(f"{d['model']:6}{d['gemm']:8}{d['kind']:6} M{d['M']:>6} N{d['N']:>6} K{d['K']:>6}  torch {d['torch_us']:8.1f} us "
          f"({d['torch_TF']:5.0f} TF)  dta {t} {us:8.1f} us ({fl / us / 1e6:5.0f} TF)  torch/dta {d['torch_us'] / us:.2f}")
