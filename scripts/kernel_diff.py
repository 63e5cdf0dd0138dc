#!/usr/bin/env python3
"""Per-kernel time per step in two rocprofv3 kernel traces (e.g. an A/B of GEMM picks), over the last N steps
cut at a marker kernel (default: the fused AdamW, once per step).

    python scripts/kernel_diff.py A/run_kernel_trace.csv B/run_kernel_trace.csv [marker] [last_n]
"""
import csv
import sys
from collections import defaultdict


def per_step(path: str, marker: str, last_n: int):
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
    ends = [e for s, e, n in ks if marker in n]
    a, b = ends[-(last_n + 1)], ends[-1]
    t = defaultdict(float)
    c = defaultdict(int)
    for s, e, n in ks:
        if s >= a and e <= b:
            t[n] += (e - s) / 1e3
            c[n] += 1
    return {k: v / last_n for k, v in t.items()}, {k: v / last_n for k, v in c.items()}, (b - a) / 1e6 / last_n


def main() -> None:
    pa, pb = sys.argv[1], sys.argv[2]
    marker = sys.argv[3] if len(sys.argv) > 3 else "flat_adam_kernel"
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    ta, ca, wa = per_step(pa, marker, n)
    tb, cb, wb = per_step(pb, marker, n)
    print(f"wall per step: A {wa:.3f} ms, B {wb:.3f} ms, B - A {wb - wa:+.3f} ms")
    rows = []
    for k in set(ta) | set(tb):
        rows.append((tb.get(k, 0.0) - ta.get(k, 0.0), ta.get(k, 0.0), tb.get(k, 0.0), ca.get(k, 0), cb.get(k, 0), k))
    rows.sort(key=lambda r: -abs(r[0]))
    print(f"{'B-A us':>9} {'A us':>9} {'B us':>9} {'nA':>5} {'nB':>5}  kernel")
    for d, x, y, na, nb, k in rows[:25]:
        print(f"{d:9.1f} {x:9.1f} {y:9.1f} {na:5.1f} {nb:5.1f}  {k[:100]}")


if __name__ == "__main__":
    main()
