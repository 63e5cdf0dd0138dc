#!/usr/bin/env python3
"""Core clock of the persistent MLP loop: s_memtime (shader clock) vs
s_memrealtime (100 MHz) stamps at launch entry / params loaded / first batch /
loop end / exit, for a 20-step and a 1000-step launch, cold and after a
GPU-wide busy kernel."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    from distributed_training_amd.data.datasets import DeviceDataLoader, MyTrainDataset
    from distributed_training_amd.engine.fused_mlp import FusedMLPProgram
    from distributed_training_amd.models.mlp import MLP
    from distributed_training_amd.ops import mlp_fused as mf
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
    prog = FusedMLPProgram(model, opt, loader, comm, loss="mse")
    prog.run_steps(5)
    torch.cuda.synchronize()
    big = torch.randn(8192, 8192, device=dev)
    out = {}
    for name, K, busy in (("k20_cold", 20, False), ("k20_busy", 20, True), ("k1000", 1000, False),
                          ("k20_cold2", 20, False)):
        dbg = torch.zeros(80, dtype=torch.int64, device=dev)
        prog._ensure(prog.launched + K)
        torch.cuda.synchronize()
        if busy:
            (big @ big).sum()
        mf.persistent_steps(prog.Xp, prog.Y, prog.ring, prog.cursor, prog.loss_ring, prog.loss_cursor,
                            prog.mom_started_dev, prog.P[0], prog.M[0], prog.layout, 32, K, "relu", "mse", 1.0,
                            prog.hyper(), dbg=dbg, dbg_step=-2)
        torch.cuda.synchronize()
        prog.launched += K
        rt = dbg[64:69].cpu().tolist()
        ct = dbg[72:77].cpu().tolist()
        seg = []
        for i in range(4):
            us = (rt[i + 1] - rt[i]) / 100.0
            cyc = ct[i + 1] - ct[i]
            seg.append({"us": us, "cycles": cyc, "GHz": round(cyc / us / 1e3, 3) if us > 0 else None})
        out[name] = {"segments(entry->params, ->first batch, ->loop end, ->exit)": seg,
                     "loop_us_per_step": round((rt[3] - rt[2]) / 100.0 / K, 3),
                     "loop_cycles_per_step": round((ct[3] - ct[2]) / K, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def phases():
    """Per-wave phase stamps (s_memtime) of one step inside a 64-step launch (needs an
    extension built with -DDTA_MP_PHASES: the stamps are compiled out by default):
    0 step start, 1 forward done, 2 after barrier 1, 3 loss phase done, 4 after
    barrier 2, 6 first tile's act-grad GEMM done, 7 first tile's SGD done, 5 step end."""
    from distributed_training_amd.data.datasets import DeviceDataLoader, MyTrainDataset
    from distributed_training_amd.engine.fused_mlp import FusedMLPProgram
    from distributed_training_amd.models.mlp import MLP
    from distributed_training_amd.ops import mlp_fused as mf
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.comm import make_comm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.sampler import DistributedSampler

    dev = torch.device("cuda", 0)
    comm = make_comm(dev)
    torch.manual_seed(0)
    ds = MyTrainDataset(2048, 20, 1, seed=0)
    model = MLP(20, 512, 1, activation="relu").to(dev)
    ddp = DistributedDataParallel(model, comm=comm, device=dev)
    opt = FusedSGD(ddp.parameters(), lr=1e-3)
    loader = DeviceDataLoader(ds, 32, sampler=DistributedSampler(ds, num_replicas=1, rank=0), device=dev)
    prog = FusedMLPProgram(model, opt, loader, comm, loss="mse")
    prog.run_steps(5)
    res = {}
    for step in (10, 40):
        dbg = torch.zeros(72, dtype=torch.int64, device=dev)
        prog._ensure(prog.launched + 64)
        torch.cuda.synchronize()
        mf.persistent_steps(prog.Xp, prog.Y, prog.ring, prog.cursor, prog.loss_ring, prog.loss_cursor,
                            prog.mom_started_dev, prog.P[0], prog.M[0], prog.layout, 32, 64, "relu", "mse", 1.0,
                            prog.hyper(), dbg=dbg, dbg_step=step)
        torch.cuda.synchronize()
        prog.launched += 64
        d = dbg[:64].view(8, 8).cpu()
        t0 = int(d[:, 0].min())
        res[f"step{step}"] = {f"wave{w}": [int(d[w, k]) - t0 for k in (0, 1, 2, 3, 4, 6, 7, 5)] for w in range(8)}
    print(json.dumps(res))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "phases":
    phases()
