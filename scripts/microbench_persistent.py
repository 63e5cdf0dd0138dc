#!/usr/bin/env python3
"""Persistent MLP loop: us/step from events over N-step launches + per-phase
s_memtime stamps of one step (8 waves)."""
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
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.sampler import DistributedSampler

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ds = MyTrainDataset(2048, 20, 1, seed=0)
    model = MLP(20, 512, 1).to(dev)
    opt = FusedSGD(model.parameters(), lr=1e-3)
    loader = DeviceDataLoader(ds, 32, sampler=DistributedSampler(ds, num_replicas=1, rank=0), device=dev)
    prog = FusedMLPProgram(model, opt, loader, RcclComm(0, 1, dev), loss="mse")
    assert prog.persistent
    prog.run_steps(64)
    torch.cuda.synchronize()
    out = {}
    for n in (64, 256, 1024):
        prog._ensure(prog.launched + n)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        mf.persistent_steps(prog.Xp, prog.Y, prog.ring, prog.cursor, prog.loss_ring, prog.loss_cursor,
                            prog.mom_started_dev, prog.P[0], prog.M[0], prog.layout, 32, n, "relu", "mse",
                            1.0, prog.hyper())
        e.record()
        torch.cuda.synchronize()
        out[f"us_per_step_n{n}"] = s.elapsed_time(e) * 1e3 / n
        prog.launched += n
    dbg = torch.zeros(64, dtype=torch.int64, device=dev)
    prog._ensure(prog.launched + 64)
    mf.persistent_steps(prog.Xp, prog.Y, prog.ring, prog.cursor, prog.loss_ring, prog.loss_cursor,
                        prog.mom_started_dev, prog.P[0], prog.M[0], prog.layout, 32, 64, "relu", "mse", 1.0,
                        prog.hyper(), dbg=dbg, dbg_step=40)
    torch.cuda.synchronize()
    d = dbg.view(8, 8).cpu()
    base = int(d[:, 0].min())
    out["stamps_cycles_rel"] = [[int(x) - base for x in row] for row in d.tolist()]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
