"""Helpers for multi-process CPU (gloo) tests."""
import os
import socket
import traceback

import torch.distributed as dist
import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _entry(rank, ws, port, fn, args, errq):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(ws), "LOCAL_RANK": str(rank)})
    try:
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        fn(rank, ws, *args)
    except BaseException:  # noqa: BLE001
        errq.put((rank, traceback.format_exc()))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_gloo(fn, ws: int = 2, *args):
    """Run ``fn(rank, ws, *args)`` in ``ws`` gloo processes; re-raise failures."""
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, ws, port, fn, args, errq)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    if errs:
        raise AssertionError("\n".join(f"rank {r}:\n{tb}" for r, tb in errs))
    bad = [p.exitcode for p in procs if p.exitcode != 0]
    assert not bad, f"worker exit codes {bad}"
