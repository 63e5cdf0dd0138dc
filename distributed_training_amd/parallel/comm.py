"""Collective communication layer.

Two implementations behind one small interface:

* :class:`RcclComm` -- the GPU hot path.  A native RCCL communicator
  (``csrc/rccl_comm.cpp``) bootstrapped through torchrun's TCPStore, with its
  own high-priority HIP stream.  Collectives are enqueued on that stream after
  an event wait on the producing (compute) stream, so they overlap with the
  rest of backward; :class:`CommWork.wait` makes the consumer stream wait on
  the comm stream (no host synchronisation) and the whole thing can be
  captured into a hipGraph.
* :class:`TorchComm` -- ``torch.distributed`` (gloo on CPU, or any backend);
  used for the CPU plumbing path and as the control plane.

Reference parity: replaces the implicit c10d NCCL/Gloo process group of
``src/distributed_trainer.py:61-62`` and the explicit ``dist.broadcast`` /
``dist.all_reduce`` of ``src/playground/ddp_script.py:120-121,149-153``
(SURVEY.md §2.4, §2.7).
"""
from __future__ import annotations

import collections
import contextlib
import os
import sys
import threading
import time
from typing import Any, Callable, Deque, Iterator, List, Optional, Tuple

import torch
import torch.distributed as dist

_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
        "prod": dist.ReduceOp.PRODUCT}


@contextlib.contextmanager
def _stdout_to_stderr() -> Iterator[None]:
    """Redirect the C-level stdout (fd 1) to stderr for the duration."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


class CommWork:
    """Handle of an asynchronous collective."""

    def __init__(self, torch_work: Any = None, event: Any = None, post: Any = None) -> None:
        self._work = torch_work
        self._event = event
        self._post = post
        self._done = False

    def wait(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Order ``stream`` (default: the current stream) after the collective.  A torch work's
        ``wait()`` orders the CURRENT stream, so with an explicit ``stream`` it runs with that
        stream made current (and so does the post-processing, e.g. the avg division)."""
        if self._done:
            return
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            if self._work is not None:
                self._work.wait()
            if self._event is not None:
                (stream or torch.cuda.current_stream()).wait_event(self._event)
            if self._post is not None:
                self._post()
        self._done = True


class Communicator:
    rank: int = 0
    world_size: int = 1
    device: torch.device = torch.device("cpu")
    name = "base"

    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = False) -> Optional[CommWork]:
        raise NotImplementedError

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False) -> Optional[CommWork]:
        raise NotImplementedError

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum",
                            async_op: bool = False) -> Optional[CommWork]:
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, src: int = 0, async_op: bool = False) -> Optional[CommWork]:
        raise NotImplementedError

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError

    def supports_avg(self) -> bool:
        return False


class TorchComm(Communicator):
    """torch.distributed-backed communicator (gloo on CPU)."""

    name = "torch"

    def __init__(self, group: Any = None, device: Optional[torch.device] = None) -> None:
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world_size = dist.get_world_size(group) if dist.is_initialized() else 1
        self.device = device or torch.device("cpu")
        self.backend = dist.get_backend(group) if dist.is_initialized() else "none"

    def _w(self, work: Any, async_op: bool) -> Optional[CommWork]:
        if async_op:
            return CommWork(torch_work=work)
        return None

    def all_reduce(self, t: Any, op: str = "sum", async_op: bool = False) -> Optional[CommWork]:
        if self.world_size == 1:
            return CommWork() if async_op else None
        if op == "avg":
            t.div_(self.world_size)
            op = "sum"
        work = dist.all_reduce(t, op=_OPS[op], group=self.group, async_op=async_op)
        return self._w(work, async_op)

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False) -> Optional[CommWork]:
        if self.world_size == 1:
            if out.data_ptr() != inp.data_ptr():
                out.view(-1).copy_(inp.view(-1))
            return CommWork() if async_op else None
        work = dist.all_gather_into_tensor(out, inp, group=self.group, async_op=async_op)
        return self._w(work, async_op)

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum", async_op: bool = False) -> Optional[CommWork]:
        if self.world_size == 1:
            if out.data_ptr() != inp.data_ptr():
                out.view(-1).copy_(inp.view(-1))
            return CommWork() if async_op else None
        post = None
        if op == "avg":
            op = "sum"
            ws = self.world_size
            post = lambda: out.div_(ws)  # noqa: E731
        work = dist.reduce_scatter_tensor(out, inp, op=_OPS[op], group=self.group, async_op=async_op)
        if async_op:
            return CommWork(torch_work=work, post=post)
        if post:
            post()
        return None

    def broadcast(self, t: Any, src: int = 0, async_op: bool = False) -> Optional[CommWork]:
        if self.world_size == 1:
            return CommWork() if async_op else None
        if self.group is not None:  # ``src`` is a rank of this communicator's group, as for every backend here
            # (mapped to its global rank: ``group_src=`` exists only from torch 2.6)
            work = dist.broadcast(t, src=dist.get_global_rank(self.group, src), group=self.group, async_op=async_op)
        else:
            work = dist.broadcast(t, src=src, async_op=async_op)
        return self._w(work, async_op)

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        if self.world_size == 1:
            out.copy_(inp)
            return
        dist.all_to_all_single(out, inp, group=self.group)

    def barrier(self) -> None:
        if self.world_size > 1:
            dist.barrier(group=self.group)


def comm_timeout_s() -> float:
    """``DTA_COMM_TIMEOUT_S``: deadline of one device collective (default 600 s; <= 0: no watchdog)."""
    v = os.environ.get("DTA_COMM_TIMEOUT_S", "600").strip()
    return float(v) if v else 600.0


class CommWatchdog:
    """Host-side deadline on device collectives -- what c10d ProcessGroupNCCL's watchdog
    gives the reference's ``init_process_group`` (src/distributed_trainer.py:61-62).

    Every collective the communicator enqueues registers the event recorded behind it on
    the comm stream (:meth:`track`); a daemon thread queries the oldest pending event
    every ``poll_s``.  One that is still pending ``timeout_s`` after its enqueue means a
    peer never joined: the thread calls ``on_timeout`` (RcclComm: ``ncclCommAbort``, which
    also ends the kernels spinning on the dead peer), records the error, and the next
    :meth:`raise_if_error` on the training thread -- every ``CommWork.wait``, the DDP
    finalize / graph-replay poll, ``barrier`` -- raises ``RuntimeError``.  If the training
    thread does not get there within ``exit_grace_s`` (blocked in a host sync that the
    abort did not release), the process exits with status 3 (``DTA_COMM_TIMEOUT_EXIT=0``
    disables that), so a hung rank ends the job instead of holding the node.  No
    device synchronisation: tracking is a deque append per collective."""

    def __init__(self, name: str, timeout_s: float, on_timeout: Callable[[], None], poll_s: float = 0.0,
                 exit_grace_s: float = 60.0) -> None:
        self.name = name
        self.timeout_s = float(timeout_s)
        self.poll_s = float(poll_s) if poll_s > 0 else max(0.05, min(2.0, self.timeout_s / 20))
        self.exit_grace_s = float(exit_grace_s)
        self.on_timeout = on_timeout
        self.error: Optional[str] = None
        self._pending: Deque[Tuple[object, float, str]] = collections.deque()
        self._lock = threading.Lock()
        self._fire = threading.Lock()  # held by the one thread that runs the abort
        self._stop = threading.Event()
        self._reported = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def track(self, event: Any, desc: str) -> None:
        """``event``: anything with ``query() -> bool`` (a ``torch.cuda.Event`` recorded after the collective)."""
        if self.timeout_s <= 0:
            return
        with self._lock:
            self._pending.append((event, time.monotonic(), desc))
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name=f"dta-comm-watchdog-{self.name}", daemon=True)
            self._thread.start()

    def pending(self) -> int:
        with self._lock:
            return len(self._pending)

    def check(self) -> bool:
        """One watchdog pass; True if the deadline expired (now or before)."""
        if self.error is not None:
            return True
        now = time.monotonic()
        with self._lock:
            while self._pending and self._pending[0][0].query():
                self._pending.popleft()
            head = self._pending[0] if self._pending else None
        if head is None or now - head[1] <= self.timeout_s:
            return False
        if not self._fire.acquire(blocking=False):
            return True  # another thread is aborting; its error is published when the abort returned
        msg = (f"{self.name}: collective '{head[2]}' not complete {now - head[1]:.1f} s after its enqueue "
               f"(DTA_COMM_TIMEOUT_S={self.timeout_s:g}); communicator aborted")
        print(f"[dta watchdog] {msg}", file=sys.stderr, flush=True)
        try:
            self.on_timeout()
        except Exception as e:  # noqa: BLE001 - the error is reported either way
            print(f"[dta watchdog] abort failed: {e}", file=sys.stderr, flush=True)
        # published AFTER the abort: a training thread that raises has an aborted communicator (a test
        # saw the RuntimeError before the abort had run when the error was set first)
        self.error = msg
        return True

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            if self.check():
                break
        while self.error is None and not self._stop.wait(0.01):  # (the other thread's abort still running)
            pass
        if self.error is None or self._stop.is_set():
            return
        if os.environ.get("DTA_COMM_TIMEOUT_EXIT", "1") != "0" and not self._reported.wait(self.exit_grace_s):
            print(f"[dta watchdog] training thread did not observe the timeout within {self.exit_grace_s:g} s; "
                  "exiting", file=sys.stderr, flush=True)
            os._exit(3)

    def raise_if_error(self) -> None:
        if self.error is not None:
            self._reported.set()
            raise RuntimeError(self.error)

    def stop(self) -> None:
        self._stop.set()


class _StreamComm(Communicator):
    """Collectives enqueued on the communicator's own HIP stream: the stream
    first waits on the caller's (compute) stream, the returned work's event
    makes a consumer stream wait in turn -- no host synchronisation, and the
    caching allocator is told (``record_stream``) that the tensors are in use
    on the comm stream.  With a :class:`CommWatchdog` (``self.watchdog``) every
    eager collective is put under its deadline (captured ones are covered by the
    graph replay's own tracked event: :meth:`watch_stream`)."""

    stream: torch.cuda.Stream
    watchdog: Optional[CommWatchdog] = None

    def _enqueue(self, fn: Any, async_op: bool, tensors: List[torch.Tensor], desc: str = "collective"
                 ) -> Optional[CommWork]:
        self.raise_if_error()
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        try:
            fn(int(self.stream.cuda_stream))
        except RuntimeError:
            # the watchdog aborted the communicator while this enqueue raced it: report ITS error
            # (and tell it the training thread has seen the timeout) rather than the bare abort --
            # it is published once the abort call returns, so wait for that briefly
            wd = self.watchdog
            if wd is not None:
                deadline = time.monotonic() + 30.0
                while wd.error is None and wd._fire.locked() and time.monotonic() < deadline:
                    time.sleep(0.005)
            self.raise_if_error()
            raise
        for t in tensors:  # keep the caching allocator from recycling the memory early
            t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        if self.watchdog is not None and not torch.cuda.is_current_stream_capturing():
            self.watchdog.track(ev, desc)
        work = CommWork(event=ev, post=self.raise_if_error)
        if async_op:
            return work
        work.wait(cur)
        return None

    def watch_stream(self, stream: torch.cuda.Stream, desc: str) -> None:
        """Put the work enqueued so far on ``stream`` (e.g. a replayed step graph holding
        captured collectives) under the watchdog's deadline."""
        if self.watchdog is not None:
            ev = torch.cuda.Event()
            ev.record(stream)
            self.watchdog.track(ev, desc)

    def raise_if_error(self) -> None:
        if self.watchdog is not None:
            self.watchdog.raise_if_error()

    def poll_errors(self) -> None:
        """Raise if a bounded peer wait timed out (cheap: no device sync)."""
        self.raise_if_error()


class RcclComm(_StreamComm):
    """Native RCCL communicator on a dedicated HIP stream (GPU hot path)."""

    name = "rccl"

    def __init__(self, rank: int, world_size: int, device: torch.device, store: Any = None, tag: str = "default",
                 stream_priority: int = -1, timeout_s: Optional[float] = None) -> None:
        from ..ops import ensure_rccl

        C = ensure_rccl()
        self.rank, self.world_size, self.device = rank, world_size, device
        key = f"dta_rccl_uid/{tag}"
        if store is None and dist.is_initialized():
            store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            uid = C.rccl_unique_id()
            if store is not None:
                store.set(key, uid)
        else:
            if store is None:
                raise RuntimeError("RcclComm needs a store (torch.distributed initialised) for world_size > 1")
            uid = store.get(key)
        with _stdout_to_stderr():  # RCCL prints its version banner on stdout at init
            self._comm = C.RcclComm(uid, world_size, rank, device.index if device.index is not None else 0)
        # dedicated high-priority stream for collectives (lower number = higher priority)
        self.stream = torch.cuda.Stream(device=device, priority=stream_priority)
        # deadline per collective (c10d watchdog semantics); at one rank nothing waits for a peer, so only
        # an explicit timeout_s (tests) arms it there
        t = comm_timeout_s() if timeout_s is None else float(timeout_s)
        self.aborted = False
        if t > 0 and (world_size > 1 or timeout_s is not None):
            self.watchdog = CommWatchdog(f"rccl rank {rank}/{world_size}", t, self.abort)
        # one-shot xGMI all-reduce for small fp32 buckets (intra-node, self-tested)
        self._p2p = None
        if world_size > 1 and store is not None:
            from .p2p import maybe_create

            def _min(t: Any) -> None:
                self._comm.all_reduce(t, "min", int(torch.cuda.current_stream(device).cuda_stream))
                torch.cuda.current_stream(device).synchronize()

            self._p2p = maybe_create(rank, world_size, device, store, _min, tag=tag)

    def supports_avg(self) -> bool:
        return True

    def all_reduce(self, t: Any, op: str = "sum", async_op: bool = False) -> Optional[CommWork]:
        if self._p2p_ok(t, op):
            sc = 1.0 / self.world_size if op == "avg" else 1.0
            h, it = self._p2p._h, self._p2p.timeout_iters
            return self._enqueue(lambda s: h.all_reduce(t, sc, it, s), async_op, [t], "p2p all_reduce")
        return self._enqueue(lambda s: self._comm.all_reduce(t, op, s), async_op, [t],
                             f"all_reduce {t.numel()} x {t.dtype}")

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False) -> Optional[CommWork]:
        if self.world_size == 1:  # single rank: a device copy on the current stream
            if out.data_ptr() != inp.data_ptr():
                out.view(-1).copy_(inp.view(-1))
            return CommWork() if async_op else None
        return self._enqueue(lambda s: self._comm.all_gather(out, inp, s), async_op, [out, inp],
                             f"all_gather {inp.numel()} x {inp.dtype}")

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum", async_op: bool = False) -> Optional[CommWork]:
        return self._enqueue(lambda s: self._comm.reduce_scatter(out, inp, op, s), async_op, [out, inp],
                             f"reduce_scatter {out.numel()} x {out.dtype}")

    def broadcast(self, t: Any, src: int = 0, async_op: bool = False) -> Optional[CommWork]:
        return self._enqueue(lambda s: self._comm.broadcast(t, src, s), async_op, [t],
                             f"broadcast {t.numel()} x {t.dtype}")

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        self._enqueue(lambda s: self._comm.all_to_all(out, inp, s), False, [out, inp], "all_to_all")

    def abort(self) -> None:
        """``ncclCommAbort``: ends this rank's pending RCCL kernels; every later collective raises.
        Safe from the watchdog thread while the training thread enqueues: the native communicator
        flags itself first (new calls raise), then waits for in-flight enqueues before releasing the
        handle (csrc/rccl_comm.h)."""
        self.aborted = True
        self._comm.abort()

    def _p2p_ok(self, t: torch.Tensor, op: str) -> bool:
        return self._p2p is not None and op in ("sum", "avg") and self._p2p.supports(t)

    def all_reduce_inline(self, t: torch.Tensor, op: str = "sum", stream: Any = None) -> None:
        """Enqueue on ``stream`` (default: current) with no stream hop: used
        inside hipGraph-captured step programs."""
        s = stream or torch.cuda.current_stream(self.device)
        if self._p2p_ok(t, op):
            self._p2p.all_reduce(t, 1.0 / self.world_size if op == "avg" else 1.0, stream=s)
            return
        self._comm.all_reduce(t, op, int(s.cuda_stream))

    @property
    def p2p_enabled(self) -> bool:
        return self._p2p is not None

    def check_errors(self) -> None:
        if self._p2p is not None:
            self._p2p.check()

    def poll_errors(self) -> None:
        """Per-step check of the watchdog and of the p2p path's sticky timeout flag (no device
        sync): a peer that never delivered leaves a partial sum, so training must not go on silently."""
        self.raise_if_error()
        if self._p2p is not None:
            self._p2p.poll()

    def barrier(self) -> None:
        x = torch.zeros(1, device=self.device)
        self.all_reduce(x)
        torch.cuda.current_stream(self.device).synchronize()
        self.raise_if_error()

    def destroy(self) -> None:
        if self.watchdog is not None:
            self.watchdog.stop()
        self._comm.destroy()


def make_comm(device: torch.device, prefer: str = "auto", group: Any = None, bulk: bool = False) -> Communicator:
    """Pick the communicator for ``device``.

    GPU: native RCCL (``prefer`` auto|rccl, the default); the IPC direct-push
    collectives (:class:`~.ipc.IpcComm`) with ``prefer="ipc"`` / ``DTA_COMM=ipc``,
    and always when several ranks share one GPU (``DTA_SHARED_GPU=1``: RCCL
    refuses that).  ``bulk``: a communicator for large gradient / parameter traffic
    (the DDP / FSDP engines): on a multi-GPU node RCCL and the IPC push plane are
    BOTH built and each message is routed to the one that measured faster for its
    op, dtype and size (:class:`~.routed.RoutedComm`; ``DTA_IPC_COLL=0`` disables it;
    any failure falls back to RCCL on every rank).  CPU, or ``DTA_COMM=torch``:
    torch.distributed (gloo)."""
    from .ipc import IpcComm, shared_gpu
    from .p2p import intra_node

    rank = dist.get_rank() if dist.is_initialized() else 0
    ws = dist.get_world_size() if dist.is_initialized() else 1
    env = os.environ.get("DTA_COMM", "")
    if device.type == "cuda" and env != "torch":
        if ws > 1 and (shared_gpu() or prefer == "ipc" or env == "ipc"):
            return IpcComm(rank, ws, device)
        if prefer in ("auto", "rccl", "ipc"):
            rccl = RcclComm(rank, ws, device)
            if bulk and 1 < ws <= 8 and intra_node() and os.environ.get("DTA_IPC_COLL", "auto") != "0":
                try:
                    ipc = IpcComm(rank, ws, device, tag="routed")
                except Exception as e:  # noqa: BLE001 - raised on every rank alike (collective checks)
                    import logging

                    logging.getLogger(__name__).warning("IPC data plane unavailable (%s): RCCL only", e)
                    return rccl
                from .routed import RoutedComm

                return RoutedComm(rccl, ipc)
            return rccl
    return TorchComm(group=group, device=device)


def make_hybrid_comms(device: torch.device, shard_size: int) -> Tuple[Communicator, Communicator]:
    """The two communicators of HYBRID sharding (HSDP): ranks ``[g S, (g + 1) S)`` form shard group
    ``g`` (S = ``shard_size``: one node's GPUs under torchrun's rank order, so the FSDP gathers and
    reduce-scatters stay on xGMI) and the ranks with the same index in every shard group form a
    replica group (the inter-node gradient all-reduce).  GPU: RCCL communicators of their own
    (IPC ones when several ranks share one GPU); CPU: gloo subgroups (every rank creates every
    group, in one order, as torch.distributed.new_group requires)."""
    rank = dist.get_rank() if dist.is_initialized() else 0
    ws = dist.get_world_size() if dist.is_initialized() else 1
    if shard_size < 1 or ws % shard_size:
        raise ValueError(f"hybrid shard size {shard_size} must divide the world size {ws}")
    g, i, reps = rank // shard_size, rank % shard_size, ws // shard_size
    if device.type == "cuda" and os.environ.get("DTA_COMM", "") != "torch":
        from .ipc import IpcComm, shared_gpu

        if shared_gpu():
            return (IpcComm(i, shard_size, device, tag=f"hsdp_shard{g}"),
                    IpcComm(g, reps, device, tag=f"hsdp_rep{i}"))
        return (RcclComm(i, shard_size, device, tag=f"hsdp_shard{g}"),
                RcclComm(g, reps, device, tag=f"hsdp_rep{i}"))
    shard_groups = [dist.new_group(list(range(k * shard_size, (k + 1) * shard_size))) for k in range(reps)]
    rep_groups = [dist.new_group(list(range(j, ws, shard_size))) for j in range(shard_size)]
    return TorchComm(shard_groups[g], device), TorchComm(rep_groups[i], device)
