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


def worker(rank, ws, port, steps, with_comm, q):
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
    comm = types.SimpleNamespace(world_size=ws, rank=rank)
    if with_comm:
        # the per-step program's all-reduce: the one-shot p2p kernel the RCCL
        # communicator routes small fp32 buckets to (RCCL itself refuses two
        # ranks on one GPU)
        from distributed_training_amd.parallel.p2p import P2PAllReduce

        p2p = P2PAllReduce(rank, ws, dev, dist.distributed_c10d._get_default_store(), tag="bench_comm")
        comm.all_reduce_inline = lambda t, op="sum", stream=None: p2p.all_reduce(t, 1.0, stream=stream)
        comm.check_errors = p2p.check
    prog = FusedMLPProgram(model, opt, loader, comm, loss="mse")
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
        q.put({"procs": ws, "persistent": prog.persistent, "xmode": prog.xmode, "us_per_step": dt / steps * 1e6,
               "calibration_ms": getattr(prog, "exchange_times_ms", None)})
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--steps", type=int, default=4096)
    ap.add_argument("--comm", action="store_true", help="give the program an all-reduce (enables the per-step form)")
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    ps = [ctx.Process(target=worker, args=(r, a.procs, port, a.steps, a.comm, q)) for r in range(a.procs)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    print(json.dumps(q.get() if not q.empty() else {"error": "no result"}))


if __name__ == "__main__":
    main()
