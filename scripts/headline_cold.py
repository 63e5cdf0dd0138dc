#!/usr/bin/env python3
"""Is the short timed region of the headline bench slower on its FIRST call
because the dataset rows are cache-cold?  bench.py's sequence (5 warm-up
steps, sync, one timed 20-step call) on fresh programs, with and without a
read of the whole device-resident dataset between warm-up and the timed call,
plus a long warm-up for comparison."""
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
    out = {}
    for variant in ("plain", "touch", "warm64", "plain", "touch"):
        walls = []
        for rep in range(4):
            torch.manual_seed(0)
            ds = MyTrainDataset(2048, 20, 1, seed=0)
            model = MLP(20, 512, 1, activation="relu").to(dev)
            comm = make_comm(dev)
            ddp = DistributedDataParallel(model, comm=comm, device=dev)
            opt = FusedSGD(ddp.parameters(), lr=1e-3)
            loader = DeviceDataLoader(ds, 32, sampler=DistributedSampler(ds, num_replicas=1, rank=0), device=dev)
            p = FusedMLPProgram(model, opt, loader, comm, loss="mse")
            p.run_steps(64 if variant == "warm64" else 5)
            if variant == "touch":
                s = p.Xp.float().sum() + p.Y.sum() + p.ring.float().sum()  # all XCDs read the dataset
                s.item()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            p.run_steps(20)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
        out.setdefault(variant, []).append([round(w, 1) for w in walls])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
