#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: top kernels, per-step ms."""
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total GPU kernel time {tot / 1e6:.2f} ms over {steps} step(s) = {tot / 1e6 / steps:.3f} ms/step")
print(f"{'ms/step':>8} {'calls':>6} {'avg_us':>9} {'%':>5}  kernel")
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} "
          f"{float(r['Percentage']):5.1f}  {r['Name'][:100]}")
