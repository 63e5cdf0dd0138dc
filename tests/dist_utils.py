"""Helpers for multi-process CPU (gloo) tests."""
import os
import socket
import time
import traceback

import torch.distributed as dist
import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def setup_env_on_free_port(env, attempts: int = 5):
    """``env.setup()`` (one-rank rendezvous on 127.0.0.1) on a fresh free port, retried on a fresh port
    when another process took the probed one before the store bound it (EADDRINUSE on a shared box)."""
    for i in range(attempts):
        os.environ["MASTER_PORT"] = str(free_port())
        try:
            env.setup()
            return env
        except dist.DistNetworkError as e:
            if "EADDRINUSE" not in str(e) or i == attempts - 1:
                raise
    return env


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


def run_gloo(fn, ws: int = 2, *args, timeout: float = 300.0, attempts: int = 3):
    """Run ``fn(rank, ws, *args)`` in ``ws`` gloo processes; re-raise failures.

    The first failing rank ends the run at once (its peers would otherwise wait in a
    collective until the timeout).  A rendezvous port taken between :func:`free_port`
    and rank 0's bind (EADDRINUSE on a busy host) is retried on a fresh port."""
    ctx = mp.get_context("spawn")
    for attempt in range(attempts):
        errq = ctx.SimpleQueue()
        port = free_port()
        procs = [ctx.Process(target=_entry, args=(r, ws, port, fn, args, errq)) for r in range(ws)]
        for p in procs:
            p.start()
        deadline = time.monotonic() + timeout
        errs = []
        while time.monotonic() < deadline:
            while not errq.empty():
                errs.append(errq.get())
            if errs or not any(p.is_alive() for p in procs) \
                    or any(p.exitcode not in (None, 0) for p in procs):
                break
            time.sleep(0.05)
        if errs:  # (give the failing rank's peers no time to write more)
            time.sleep(0.5)
        for p in procs:
            if p.is_alive():
                p.kill()
        for p in procs:
            p.join(10)
        while not errq.empty():
            errs.append(errq.get())
        if errs and attempt + 1 < attempts and any("EADDRINUSE" in tb or "address already in use" in tb
                                                   for _, tb in errs):
            continue
        if errs:
            raise AssertionError("\n".join(f"rank {r}:\n{tb}" for r, tb in errs))
        bad = [p.exitcode for p in procs if p.exitcode != 0]
        assert not bad, f"worker exit codes {bad} (timeout {timeout:.0f} s)"
        return
