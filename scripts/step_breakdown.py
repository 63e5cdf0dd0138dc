#!/usr/bin/env python3
"""Per-step kernel breakdown of a training run from a rocprofv3 kernel trace, over the LAST
steps only (the per-shape GEMM timing and graph warm-ups of the first steps excluded): step
boundaries are the launches of the optimizer kernel (one per step).

    python scripts/step_breakdown.py gpurun_out/prof_g2/run_kernel_trace.csv [steps=5] [marker=flat_adam]
"""
import csv
import sys
from collections import defaultdict


def main() -> None:
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    marker = sys.argv[3] if len(sys.argv) > 3 else "flat_adam"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    steps = min(steps, len(ends) - 1)
    if steps < 1:
        raise SystemExit(f"need >= 2 '{marker}' launches, found {len(ends)}")
    a, b = ends[-1 - steps], ends[-1]
    tot, cnt = defaultdict(float), defaultdict(int)
    for r in rows[a + 1:b + 1]:
        k = r["Kernel_Name"][:110]
        tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[k] += 1
    wall = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e6 / steps
    busy = sum(tot.values()) / 1e3 / steps
    lib = sum(v for k, v in tot.items() if "Cijk" in k) / 1e3 / steps
    print(f"# {steps} step(s): wall {wall:.3f} ms/step, kernels {busy:.3f} ms/step "
          f"({100 * busy / wall:.1f} % busy), hipBLASLt (Cijk_*) {lib:.3f} ms/step ({100 * lib / wall:.1f} %)")
    print(f"{'ms/step':>9} {'calls':>6} {'avg_us':>9} {'%':>6}  kernel")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        ms = v / 1e3 / steps
        if ms < 0.005:
            continue
        print(f"{ms:9.3f} {cnt[k] // steps:6d} {v / cnt[k]:9.1f} {100 * ms / wall:6.1f}  {k}")


if __name__ == "__main__":
    main()
