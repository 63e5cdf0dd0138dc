#!/usr/bin/env python3
"""Per-kernel PMC summary of a rocprofv3 --pmc counter_collection.csv: mean kernel
time, effective clock (GRBM_GUI_ACTIVE / 8 XCDs / time), MFMA busy share."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
disp = defaultdict(dict)
meta = {}
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if pat and pat not in name:
        continue
    d = int(r["Dispatch_Id"])
    disp[d][r["Counter_Name"]] = float(r["Counter_Value"])
    meta[d] = (name, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(int)
for d, c in disp.items():
    name, ns = meta[d]
    k = name[:70]
    cnt[k] += 1
    agg[k]["ns"] += ns
    for n, v in c.items():
        agg[k][n] += v
print(f"{'calls':>5} {'avg_us':>9} {'clk_GHz':>7} {'mfma%':>6}  kernel")
for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
    n = cnt[k]
    us = a["ns"] / n / 1e3
    clk = a.get("GRBM_GUI_ACTIVE", 0) / 8 / a["ns"] if a["ns"] else 0
    busy = a.get("SQ_BUSY_CYCLES", 0)
    mfma = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    # MFMA busy cycles are per SIMD: share of (GRBM cycles x 1024 SIMDs)
    share = mfma / (a.get("GRBM_GUI_ACTIVE", 1) / 8 * 1024) * 100 if a.get("GRBM_GUI_ACTIVE") else 0
    print(f"{n:5d} {us:9.1f} {clk:7.2f} {share:6.1f}  {k}")
