#!/usr/bin/env python3
"""Decompose the fixed cost of a short timed region of the headline bench.

Prints, for K-step calls of the persistent MLP program after a warm-up:
  wall_us      -- sync; t0; run_steps(K); sync; t1   (what bench.py times)
  host_us      -- time until run_steps(K) returned (host enqueue work)
  kernel_us    -- device time of the launch between two events
and the same for an empty device op (sync round trip floor).
"""
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
    torch.manual_seed(0)
    ds = MyTrainDataset(2048, 20, 1, seed=0)
    model = MLP(20, 512, 1, activation="relu").to(dev)
    comm = make_comm(dev)
    ddp = DistributedDataParallel(model, comm=comm, device=dev)
    opt = FusedSGD(ddp.parameters(), lr=1e-3)
    loader = DeviceDataLoader(ds, 32, sampler=DistributedSampler(ds, num_replicas=1, rank=0), device=dev)
    out = {}
    # bench.py's exact sequence on fresh programs: 5 warm-up steps, then one timed 20-step call
    first = []
    for _ in range(3):
        p = FusedMLPProgram(model, opt, loader, comm, loss="mse")
        p.run_steps(5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p.run_steps(20)
        torch.cuda.synchronize()
        first.append((time.perf_counter() - t0) * 1e6)
    out["bench_like_first_call_K20_us"] = first

    class Spy:  # host time from t0 to the kernel launch call
        def __init__(self, real):
            self.real, self.t = real, None

        def launch(self, *a):
            self.t = time.perf_counter()
            return self.real.launch(*a)

    pre, bare = [], []
    for _ in range(5):
        key, real = p._plaunch
        spy = Spy(real)
        p._plaunch = (key, spy)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p.run_steps(20)
        torch.cuda.synchronize()
        pre.append((spy.t - t0) * 1e6)
        p._plaunch = (key, real)
        p._ensure(p.launched + 20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        real.launch(20)  # bare launch of the same loop (indices are in place)
        torch.cuda.synchronize()
        bare.append((time.perf_counter() - t0) * 1e6)
        p.launched += 20
    out["host_before_launch_us"] = pre
    out["bare_launch_sync_K20_us"] = bare
    prog = FusedMLPProgram(model, opt, loader, comm, loss="mse")
    prog.run_steps(5)
    torch.cuda.synchronize()
    for K in (1, 20, 100, 1000):
        walls, hosts, kerns = [], [], []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            prog.run_steps(K)
            e1.record()
            th = time.perf_counter()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            walls.append((t1 - t0) * 1e6)
            hosts.append((th - t0) * 1e6)
            kerns.append(e0.elapsed_time(e1) * 1e3)
        out[f"K{K}"] = {"wall_us": statistics.median(walls), "host_us": statistics.median(hosts),
                        "kernel_us": statistics.median(kerns),
                        "us_per_step_wall": statistics.median(walls) / K}
    # in-kernel launch timeline (s_memrealtime, 100 MHz): entry, params loaded, first batch, loop end, exit
    from distributed_training_amd.ops import mlp_fused as mf
    for K in (1, 20):
        dbg = torch.zeros(72, dtype=torch.int64, device=dev)
        prog._ensure(prog.launched + K)
        torch.cuda.synchronize()
        mf.persistent_steps(prog.Xp, prog.Y, prog.ring, prog.cursor, prog.loss_ring, prog.loss_cursor,
                            prog.mom_started_dev, prog.P[0], prog.M[0], prog.layout, 32, K, "relu", "mse", 1.0,
                            prog.hyper(), dbg=dbg, dbg_step=-1)
        torch.cuda.synchronize()
        prog.launched += K
        st = dbg[64:69].cpu().tolist()
        out[f"timeline_K{K}_us"] = [(v - st[0]) / 100.0 for v in st]
    floor = []
    x = torch.zeros(1, device=dev)
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        floor.append((time.perf_counter() - t0) * 1e6)
    out["empty_op_sync_us"] = statistics.median(floor)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
