#!/usr/bin/env python3
"""Latency of the one-shot p2p all-reduce kernel with W processes sharing ONE
GPU (the flag/IPC protocol cost without xGMI link latency; an upper bound on
what the kernel itself adds per step).  Graph-captured, like the fused step.

    python scripts/p2p_latency.py --procs 2 --elems 11280
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def worker(rank, ws, port, elems, reps, q, protocol):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from distributed_training_amd.parallel.p2p import P2PAllReduce

    torch.cuda.set_device(0)
    p2p = P2PAllReduce(rank, ws, torch.device("cuda", 0), dist.distributed_c10d._get_default_store(), tag="lat", protocol=protocol)
    x = torch.ones(elems, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(64):
                p2p.all_reduce(x, 1.0 / ws, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dist.barrier()
    p2p.check()
    if rank == 0:
        q.put(dt / (reps * 64) * 1e6)
    p2p.destroy()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--elems", type=int, default=11280)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--protocol", default="ll")
    a = ap.parse_args()
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    ps = [ctx.Process(target=worker, args=(r, a.procs, port, a.elems, a.reps, q, a.protocol)) for r in range(a.procs)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    us = q.get() if not q.empty() else None
    print(json.dumps({"procs": a.procs, "elems": a.elems, "protocol": a.protocol, "us_per_allreduce": us}))


if __name__ == "__main__":
    main()
