#!/usr/bin/env python3
"""Comm / compute overlap from a rocprofv3 ``--kernel-trace --marker-trace`` CSV run
(scripts/trace_overlap.sh).

Collective kernels (the IPC direct-push collectives, RCCL) run on the
communicator's stream; everything else of the step on the compute stream.
Reports, over the traced steps: device time of the collectives, how much of it
ran while a compute kernel was also running (overlap), the kernel census per
stream, and the host-side roctx ranges (bucket launches, unit gathers /
reduce-scatters, phases).

    python scripts/overlap_report.py gpurun_out/trace_ddp
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

COMM_KEYS = ("ipc_coll_kernel", "p2p_allreduce", "nccl", "rccl")


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def _col(row, *names):
    low = {k.lower(): k for k in row}
    for n in names:
        if n.lower() in low:
            return row[low[n.lower()]]
    raise KeyError(f"none of {names} in {list(row)[:12]}")


def _union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _measure(iv):
    return sum(e - s for s, e in iv)


def _intersect(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(d):
    d = Path(d)
    kfiles = sorted(d.rglob("*kernel_trace.csv"))
    if not kfiles:
        print(f"no kernel trace under {d}")
        return 1
    ks = _rows(kfiles[0])
    mfiles = sorted(d.rglob("*marker_api_trace.csv"))
    ms = _rows(mfiles[0]) if mfiles else []
    # the timed window: the last 4 "step" ranges (bench_lm pushes one per step)
    steps = []
    for r in ms:
        name = ""
        for k in ("Function", "Message", "Name", "Operation"):
            try:
                name = _col(r, k)
                break
            except KeyError:
                continue
        if name == "step":
            steps.append((int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))))
    t0 = steps[-4][0] if len(steps) >= 4 else None
    comm, comp = [], []
    census = defaultdict(lambda: [0, 0.0])
    for r in ks:
        s, e = int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))
        if t0 is not None and s < t0:
            continue
        name = _col(r, "Kernel_Name")
        stream = _col(r, "Stream_Id", "Queue_Id")
        is_comm = any(k in name.lower() for k in COMM_KEYS)
        (comm if is_comm else comp).append((s, e))
        key = ("comm" if is_comm else "compute", stream, name.split("(")[0][:70])
        census[key][0] += 1
        census[key][1] += (e - s) / 1e3
    cu, pu = _union(comm), _union(comp)
    ov = _intersect(cu, pu)
    span = (max(e for _, e in comm + comp) - min(s for s, _ in comm + comp)) if comm + comp else 0
    print(f"# rocprofv3 kernel + marker trace, rank 0 of 2 sharing one MI355X ({kfiles[0].name})")
    print(f"# window: {'last 4 timed steps' if t0 is not None else 'whole run'}; span {span / 1e6:.2f} ms")
    print(f"collective kernels: {len(comm)}, device time {_measure(cu) / 1e6:.3f} ms (union)")
    print(f"compute kernels:    {len(comp)}, device time {_measure(pu) / 1e6:.3f} ms (union)")
    share = ov / _measure(cu) if cu else 0.0
    print(f"collective time overlapped by compute kernels: {ov / 1e6:.3f} ms = {100 * share:.1f} %")
    print("\n# kernel census (window): class, stream, count, total us, kernel")
    for (cls, stream, name), (n, us) in sorted(census.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{cls:8s} {stream:>4s} {n:5d} {us:10.1f}  {name}")
    if ms:
        rng = defaultdict(lambda: [0, 0.0])
        for r in ms:
            try:
                name = _col(r, "Function", "Message", "Name")
                s, e = int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))
            except (KeyError, ValueError):
                continue
            if t0 is not None and s < t0:
                continue
            rng[name][0] += 1
            rng[name][1] += (e - s) / 1e3
        print("\n# roctx ranges (host, window): count, total us, name")
        for name, (n, us) in sorted(rng.items(), key=lambda kv: -kv[1][1])[:30]:
            print(f"{n:5d} {us:10.1f}  {name}")
        _per_collective(ms, ks, t0, pu)
    return 0


def _per_collective(ms, ks, t0, pu):
    """Collective kernels attributed to the host range that enqueued them (bucket all-reduce,
    FSDP unit all-gather / reduce-scatter): every comm kernel starting after a collective range
    began and before the next one began belongs to it.  Per range name: kernels, device time,
    and the share of it overlapped by compute kernels."""
    marks = []
    for r in ms:
        try:
            name = _col(r, "Function", "Message", "Name")
            s = int(_col(r, "Start_Timestamp"))
        except (KeyError, ValueError):
            continue
        if (t0 is None or s >= t0) and any(k in name for k in ("allgather", "reduce_scatter", "allreduce")):
            marks.append((s, name))
    if not marks:
        return
    marks.sort()
    comm = sorted((int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp")))
                  for r in ks if any(k in _col(r, "Kernel_Name").lower() for k in COMM_KEYS)
                  and (t0 is None or int(_col(r, "Start_Timestamp")) >= t0))
    per = defaultdict(list)
    j = 0
    for i, (s, name) in enumerate(marks):
        nxt = marks[i + 1][0] if i + 1 < len(marks) else float("inf")
        while j < len(comm) and comm[j][0] < s:
            j += 1
        k = j
        while k < len(comm) and comm[k][0] < nxt:
            per[name].append(comm[k])
            k += 1
    print("\n# collectives by enqueueing range (window): kernels, device us, overlapped by compute %, range")
    for name, iv in sorted(per.items()):
        u = _union(iv)
        tot = _measure(u)
        ovl = _intersect(u, pu)
        print(f"{len(iv):5d} {tot / 1e3:10.1f} {100 * ovl / tot if tot else 0.0:6.1f}  {name}")


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/trace_ddp"))
