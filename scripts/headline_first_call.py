#!/usr/bin/env python3
"""Why is the FIRST timed 20-step call after bench.py's 5-step warm-up slower
than later calls?  Fresh program each rep, then variants before the timed call:
  plain      -- bench.py's sequence
  second     -- one more untimed 20-step call first (a second launch)
  idle1ms    -- 1 ms host sleep after the sync (GPU idle)
  busy       -- a ~0.5 ms dummy GPU kernel right before the timed call (clock ramp)
  touch      -- read every byte the loop reads (dataset, ring, params) on all XCDs
Median of 5 reps each, interleaved."""
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
    big = torch.randn(4096, 4096, device=dev)
    res = {k: [] for k in ("plain", "second", "touch", "touch_nosync", "split", "split_touch")}
    for rep in range(5):
        for variant in res:
            torch.manual_seed(0)
            ds = MyTrainDataset(2048, 20, 1, seed=0)
            model = MLP(20, 512, 1, activation="relu").to(dev)
            ddp = DistributedDataParallel(model, comm=comm, device=dev)
            opt = FusedSGD(ddp.parameters(), lr=1e-3)
            loader = DeviceDataLoader(ds, 32, sampler=DistributedSampler(ds, num_replicas=1, rank=0), device=dev)
            p = FusedMLPProgram(model, opt, loader, comm, loss="mse")
            if variant.startswith("split"):
                p.run_steps(1)
                p.run_steps(4)
            else:
                p.run_steps(5)
            if variant in ("touch_nosync", "split_touch"):
                keep = p.Xp.float().sum() + p.Y.sum() + p.ring.float().sum() + p.P[0].sum()
            torch.cuda.synchronize()
            if variant == "second":
                p.run_steps(20)
                torch.cuda.synchronize()
            elif variant == "idle1ms":
                time.sleep(0.001)
            elif variant == "touch":
                (p.Xp.float().sum() + p.Y.sum() + p.ring.float().sum() + p.P[0].sum()).item()
            elif variant == "busy":
                (big @ big).sum()
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            p.run_steps(20)
            torch.cuda.synchronize()
            res[variant].append((time.perf_counter() - t0) * 1e6)
    print(json.dumps({k: {"median_us": round(statistics.median(v), 1), "all": [round(x, 1) for x in v]}
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
