#!/usr/bin/env python3
"""us/step of the persistent MLP loop with the in-kernel DDP exchange, W
processes sharing ONE GPU (protocol cost without xGMI latency)."""
import argparse
import json
import os
import socket
import sys
import time
import types
from pathlib import Path

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def worker(rank, ws, port, steps, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(ws),
                       "LOCAL_WORLD_SIZE": str(ws)})
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from distributed_training_amd.data.datasets import DeviceDataLoader, MyTrainDataset
    from distributed_training_amd.engine.fused_mlp import FusedMLPProgram
    from distributed_training_amd.models.mlp import MLP
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.sampler import DistributedSampler

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ds = MyTrainDataset(2048, 20, 1, seed=0)
    model = MLP(20, 512, 1).to(dev)
    opt = FusedSGD(model.parameters(), lr=1e-3)
    loader = DeviceDataLoader(ds, 32, sampler=DistributedSampler(ds, num_replicas=ws, rank=rank), device=dev)
    prog = FusedMLPProgram(model, opt, loader, types.SimpleNamespace(world_size=ws, rank=rank), loss="mse")
    prog.run_steps(256)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    prog.run_steps(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dist.barrier()
    prog.store_to_module()
    if rank == 0:
        q.put({"procs": ws, "persistent": prog.persistent, "us_per_step": dt / steps * 1e6})
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--steps", type=int, default=4096)
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    ps = [ctx.Process(target=worker, args=(r, a.procs, port, a.steps, q)) for r in range(a.procs)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    print(json.dumps(q.get() if not q.empty() else {"error": "no result"}))


if __name__ == "__main__":
    main()
