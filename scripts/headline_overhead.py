#!/usr/bin/env python3
"""Fixed cost of one persistent-loop call (bench.py's timed region) decomposed:
host time inside run_steps, GPU time between events around it, and the host
round trip of an empty kernel + sync; wall time of n-step calls for n = 1, 20,
80 (slope = per-step time, intercept = fixed cost).  Median of 15 reps."""
import json
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    from distributed_training_amd.data.datasets import DeviceDataLoader, MyTrainDataset
    from distributed_training_amd.engine.fused_mlp import FusedMLPProgram
    from distributed_training_amd.models.mlp import MLP
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.comm import make_comm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.sampler import DistributedSampler

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = make_comm(dev)
    torch.manual_seed(0)
    ds = MyTrainDataset(2048, 20, 1, seed=0)
    model = MLP(20, 512, 1, activation="relu").to(dev)
    ddp = DistributedDataParallel(model, comm=comm, device=dev)
    opt = FusedSGD(ddp.parameters(), lr=1e-3)
    loader = DeviceDataLoader(ds, 32, sampler=DistributedSampler(ds, num_replicas=1, rank=0), device=dev)
    p = FusedMLPProgram(model, opt, loader, comm, loss="mse")
    p.run_steps(64)
    torch.cuda.synchronize()
    x = torch.zeros(1, device=dev)
    res = {}

    def rec(k, v):
        res.setdefault(k, []).append(v)

    for _ in range(15):
        for n in (1, 20, 80):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            p.run_steps(n)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rec(f"wall_{n}", (t2 - t0) * 1e6)
            rec(f"host_call_{n}", (t1 - t0) * 1e6)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        p.run_steps(20)
        e1.record()
        torch.cuda.synchronize()
        rec("gpu_events_20", e0.elapsed_time(e1) * 1e3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        rec("empty_kernel_roundtrip", (time.perf_counter() - t0) * 1e6)
    # bench.py's own sequence on fresh programs: 5-step warm-up call, sync, timed 20-step call
    for _ in range(7):
        torch.manual_seed(0)
        model = MLP(20, 512, 1, activation="relu").to(dev)
        ddp = DistributedDataParallel(model, comm=comm, device=dev)
        opt = FusedSGD(ddp.parameters(), lr=1e-3)
        q = FusedMLPProgram(model, opt, loader, comm, loss="mse")
        q.run_steps(5)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        q.run_steps(20)
        e1.record()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rec("fresh_wall_20", (t2 - t0) * 1e6)
        rec("fresh_host_call_20", (t1 - t0) * 1e6)
        rec("fresh_gpu_events_20", e0.elapsed_time(e1) * 1e3)
        t0 = time.perf_counter()
        q.run_steps(20)
        torch.cuda.synchronize()
        rec("fresh_second_wall_20", (time.perf_counter() - t0) * 1e6)
    # the same timed call with _run_persistent's pieces timed separately
    for _ in range(7):
        torch.manual_seed(0)
        model = MLP(20, 512, 1, activation="relu").to(dev)
        ddp = DistributedDataParallel(model, comm=comm, device=dev)
        opt = FusedSGD(ddp.parameters(), lr=1e-3)
        q = FusedMLPProgram(model, opt, loader, comm, loss="mse")
        q.run_steps(5)
        torch.cuda.synchronize()
        ts = [time.perf_counter()]
        hp = q.hyper()
        ts.append(time.perf_counter())
        q._ensure(q.launched + 20)
        ts.append(time.perf_counter())
        if q._up_done is not None:
            if not q._up_done.query():
                torch.cuda.current_stream(dev).wait_event(q._up_done)
            q._up_done = None
        ts.append(time.perf_counter())
        key = (id(q._xinfo), tuple(sorted(hp.items())))
        same = q._plaunch is not None and q._plaunch[0] == key
        ts.append(time.perf_counter())
        q._plaunch[1].launch(20)
        ts.append(time.perf_counter())
        q._last_start = q.launched
        for j in range(20):
            q._batch_of.pop(q.launched + j, None)
        q.launched += 20
        ts.append(time.perf_counter())
        q._prefetch()
        ts.append(time.perf_counter())
        torch.cuda.synchronize()
        ts.append(time.perf_counter())
        for name, a, b in (("hyper", 0, 1), ("ensure", 1, 2), ("up_done", 2, 3), ("key", 3, 4), ("launch", 4, 5),
                           ("bookkeeping", 5, 6), ("prefetch", 6, 7), ("sync", 7, 8)):
            rec("brk_" + name, (ts[b] - ts[a]) * 1e6)
        rec("brk_cached_launch", float(same))
    med = {k: round(statistics.median(v), 2) for k, v in res.items()}
    med["per_step_us"] = round((med["wall_80"] - med["wall_20"]) / 60, 3)
    med["fixed_us"] = round(med["wall_20"] - 20 * med["per_step_us"], 2)
    print(json.dumps(med))


if __name__ == "__main__":
    main()
