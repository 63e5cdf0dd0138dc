#!/usr/bin/env python3
"""Per-step wall vs kernel-busy time from a rocprofv3 kernel trace (``--kernel-trace --output-format csv``).

    python scripts/step_gaps.py run_kernel_trace.csv [marker] [last_n]

Steps are cut at the end of each kernel whose name contains ``marker`` (default: the fused AdamW kernel,
one per training step).  For the last ``last_n`` steps it prints the wall span, the time at least one kernel
was running (the union of kernel intervals) and the idle rest -- a host-bound step shows idle time, a
GPU-bound one none -- plus the kernel count and the busiest kernels of the window."""
import csv
import sys
from collections import defaultdict


def main() -> None:
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "flat_adam_kernel"
    last_n = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    ends = [e for s, e, n in ks if marker in n]
    if len(ends) < 2:
        print(f"fewer than two '{marker}' kernels in the trace")
        return
    cuts = ends[-(last_n + 1):]
    tot_wall = tot_busy = 0
    names = defaultdict(float)
    for a, b in zip(cuts, cuts[1:]):
        win = [(max(s, a), min(e, b), n) for s, e, n in ks if e > a and s < b]
        busy, cur_s, cur_e = 0, None, None
        for s, e, n in sorted(win):
            names[n] += (e - s) / 1e3
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        tot_wall += b - a
        tot_busy += busy
        print(f"step: wall {(b - a) / 1e6:8.3f} ms  busy {busy / 1e6:8.3f} ms  idle {(b - a - busy) / 1e6:7.3f} ms  "
              f"kernels {len(win)}")
    n = len(cuts) - 1
    print(f"mean over {n}: wall {tot_wall / n / 1e6:.3f} ms/step, busy {tot_busy / n / 1e6:.3f}, "
          f"idle {(tot_wall - tot_busy) / n / 1e6:.3f}")
    for k, v in sorted(names.items(), key=lambda kv: -kv[1])[:12]:
        print(f"  {v / n / 1e3:8.3f} ms/step  {k[:110]}")


if __name__ == "__main__":
    main()
