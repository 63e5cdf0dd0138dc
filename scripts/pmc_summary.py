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
print(f"{'calls':>5} {'avg_us':>9} {'clk_GHz':>7} {'mfma%':>6} {'wait%':>6} {'winst%':>6} {'act%':>6} {'ldsbc%':>6}  kernel")
for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
    n = cnt[k]
    us = a["ns"] / n / 1e3
    clk = a.get("GRBM_GUI_ACTIVE", 0) / 8 / a["ns"] if a["ns"] else 0
    busy = a.get("SQ_BUSY_CYCLES", 0)
    mfma = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    # MFMA busy cycles are per SIMD: share of (GRBM cycles x 1024 SIMDs)
    share = mfma / (a.get("GRBM_GUI_ACTIVE", 1) / 8 * 1024) * 100 if a.get("GRBM_GUI_ACTIVE") else 0
    wc = a.get("SQ_WAVE_CYCLES", 0) or 1
    # SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY as shares of wave-cycles; LDS bank
    # conflict cycles per MFMA busy cycle (when both are collected)
    w = a.get("SQ_WAIT_ANY", 0) / wc * 100
    wi = a.get("SQ_WAIT_INST_ANY", 0) / wc * 100
    act = a.get("SQ_ACTIVE_INST_ANY", 0) / wc * 100
    bc = a.get("SQ_LDS_BANK_CONFLICT", 0) / mfma * 100 if mfma else 0
    print(f"{n:5d} {us:9.1f} {clk:7.2f} {share:6.1f} {w:6.1f} {wi:6.1f} {act:6.1f} {bc:6.1f}  {k}")
