"""A whole training step captured in ONE hipGraph and replayed per batch.

The reference runs its step eagerly (src/distributed_trainer.py:160-165:
zero_grad -> forward -> loss -> backward -> optimizer.step), so every kernel of
it is a separate host launch.  A GPT-2 small step is ~450 kernels; at several
microseconds of host work per launch (autograd, Python, the HIP runtime) the host
can fall behind a 10 ms GPU step and leave the GPU idle between kernels, by an
amount that depends on the host CPU.  Here the step is recorded once on a capture
stream and replayed with one ``hipGraphLaunch``: no per-kernel host work at all.

What makes the native step capturable:
* no host synchronisation inside it (``bench_lm.py`` ``DTA_SYNC_DEBUG=1`` checks);
* the DDP engine's bucket hooks, the deferred weight-gradient queue and the fused
  optimizer are host logic that ENQUEUES kernels -- captured once, replayed as is;
* every gradient is written (not accumulated) into its flat-buffer slice after
  ``zero_grad(set_to_none=True)`` (done on the host at capture: the replay repeats
  the same overwrites), and the fused optimizers keep their step count on the device;
* the per-shape GEMM choice (``ops/lm.py`` ``_pick``, which times candidates with a
  synchronize) is made during the eager warm-up steps, before capture.
The collectives of the step are captured too.  Whether a step may be captured is ONE
policy, :func:`capture_policy`, shared by the Trainer (engine/trainer.py) and
``bench_lm.py``: the engine's host state must be capturable (DDP: always on the GPU;
FSDP: at one rank every unit aliases its shard, at several every unit gathers into a
fixed buffer -- parallel/fsdp.py ``_GatherRing``), and at world size > 1 every
collective of the step must route to the IPC push data plane, whose kernels keep their
epoch counters on the device (graph replays advance them) and whose captured multi-rank
DDP and FSDP replays are tested bit-identical to the eager steps (tests/test_ipc_gpu.py).
A collective routed to RCCL keeps the step eager unless ``DTA_GRAPH_RCCL=1`` opts in:
RCCL inside a replayed graph at world size > 1 has not been run on a multi-GPU node.

Host logic that the replay skips is redone around it:
* the communicator's error poll of the engine's end-of-backward finalize (a peer
  exchange that timed out must raise, not leave partial sums): :meth:`__call__`
  polls after every replay (a host-mapped flag, no device sync);
* a capture that fails (an op that cannot be recorded) leaves the engine mid-step:
  its hook state and the deferred weight-gradient queue are reset, and all ranks
  agree (MIN over the engine's communicator) before any of them falls back to the
  eager step -- one rank replaying while another runs eagerly would issue different
  collectives and hang.  ``ok`` is False then and the caller runs eagerly.

The static inputs are the tensors the step reads; :meth:`__call__` copies a new
batch into them (device-to-device) before the replay.
"""
from __future__ import annotations

import logging
import os
from typing import Any, Callable, Optional, Sequence, Tuple

import torch

logger = logging.getLogger(__name__)


def _plane(comm: Any, op: str, dtype: torch.dtype, nbytes: int) -> str:
    """The data plane a collective goes to: ``"ipc"`` (capturable push kernels), ``"rccl"``, or
    ``"host"`` (torch / gloo process-group calls: not capturable)."""
    from ..parallel.comm import RcclComm
    from ..parallel.ipc import IpcComm
    from ..parallel.routed import RoutedComm

    if isinstance(comm, RoutedComm):
        return _plane(comm.fast if comm.route_of(op, dtype, nbytes) == "fast" else comm.primary, op, dtype, nbytes)
    if isinstance(comm, IpcComm):
        return "ipc"
    if isinstance(comm, RcclComm):
        return "rccl"
    return "host"


def capture_policy(engine: Any) -> Tuple[bool, str]:
    """May ``engine``'s whole training step be captured as one hipGraph?  ``(ok, reason)``.

    * the engine's per-step host state must allow it (``graph_capturable()``: DDP on the GPU; FSDP
      aliasing its shards at one rank or gathering into fixed buffers at several);
    * at one rank no collective runs;
    * at several, every collective the step issues (``step_messages()``) must route to the IPC data
      plane -- or to RCCL with ``DTA_GRAPH_RCCL=1`` (RCCL replayed inside a graph at world size > 1 is
      not verified on a multi-GPU node, so it is an explicit opt-in); process-group (gloo / torch)
      calls never are.
    Reference: the eager step of src/distributed_trainer.py:160-165 under the DDP / FSDP wraps of
    src/dist_strategy/ddp_strategy.py:18-21 and fsdp_strategy.py:20-26."""
    cap = getattr(engine, "graph_capturable", None)
    if cap is None or not cap():
        return False, "engine state not capturable"
    ws = int(getattr(engine, "world_size", 1))
    if ws <= 1:
        return True, "one rank: no collective"
    msgs = getattr(engine, "step_messages", None)
    comm = getattr(engine, "comm", None)
    if msgs is None or comm is None:
        return False, "collectives unknown"
    planes = {_plane(comm, op, dt, n) for op, dt, n in msgs()}
    if getattr(engine, "rep", None) is not None:
        planes.add(_plane(engine.rep, "all_reduce", torch.float32, 1 << 30))
    if planes <= {"ipc"}:
        return True, "every collective on the IPC data plane"
    if "host" in planes:
        return False, "collectives on the process group (not capturable)"
    if os.environ.get("DTA_GRAPH_RCCL", "0") == "1":
        return True, "RCCL collectives captured (DTA_GRAPH_RCCL=1)"
    return False, "collectives routed to RCCL (set DTA_GRAPH_RCCL=1 to capture them)"


def _agree_all_ok(engine: Any, ok: bool, device: torch.device) -> bool:
    """MIN of ``ok`` over the engine's ranks (eager collective, outside any capture)."""
    comm = getattr(engine, "comm", None)
    if comm is None or getattr(comm, "world_size", 1) <= 1:
        return ok
    t = torch.tensor([1.0 if ok else 0.0], device=device if comm.device.type == "cuda" else "cpu")
    comm.all_reduce(t, op="min")
    return float(t.item()) >= 1.0


class GraphedStep:
    def __init__(self, step_fn: Callable[..., torch.Tensor], static_inputs: Sequence[torch.Tensor],
                 warmup: int = 3, engine: Optional[Any] = None) -> None:
        """``step_fn(*static_inputs)`` runs one full training step (zero_grad, forward,
        backward, optimizer step) and returns the loss tensor.  ``warmup`` eager steps
        run first on the capture stream (they are real training steps).  ``engine``:
        the DDP engine of the step (error polls, capture-failure reset, rank agreement)."""
        self.static = list(static_inputs)
        self.engine = engine
        dev = self.static[0].device
        self.device = dev
        self.stream = torch.cuda.Stream(dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        self.warmup_losses = []
        with torch.cuda.stream(self.stream):
            for _ in range(max(1, warmup)):
                # detached: a kept loss would keep its autograd graph -- and the parameters'
                # AccumulateGrad nodes, created on THIS stream -- alive, and a later eager step on
                # another stream would then accumulate through a node of the wrong stream
                self.warmup_losses.append(step_fn(*self.static).detach())
        torch.cuda.current_stream(dev).wait_stream(self.stream)
        torch.cuda.synchronize(dev)
        self.graph: Optional[torch.cuda.CUDAGraph] = torch.cuda.CUDAGraph()
        self.error: Optional[BaseException] = None
        self.loss: Optional[torch.Tensor] = None
        try:
            with torch.cuda.graph(self.graph, stream=self.stream):
                self.loss = step_fn(*self.static).detach()  # (as above: no graph kept alive)
        except Exception as e:  # noqa: BLE001 - reported through .ok / .error after the agreement
            # without its traceback: the frames hold the half-captured step's loss, whose autograd graph
            # (and AccumulateGrad nodes made on the capture stream) the eager steps would then accumulate through
            self.error = e.with_traceback(None)
            self._abandon()
        torch.cuda.synchronize(dev)
        if not _agree_all_ok(engine, self.error is None, dev):
            if self.error is None:
                self.error = RuntimeError("step capture failed on another rank")
            logger.warning("step graph disabled, eager step used: %s", self.error)
            self.graph = None
            self.loss = None
        self.replays = 0

    @property
    def ok(self) -> bool:
        return self.graph is not None

    def _abandon(self) -> None:
        """Undo the host state a half-captured step left behind."""
        from ..ops import lm

        lm.abandon_step()
        reset = getattr(self.engine, "reset_iteration", None)
        if reset is not None:
            reset()

    def poll(self) -> None:
        comm = getattr(self.engine, "comm", None)
        if comm is None or getattr(self.engine, "world_size", 1) <= 1:
            return
        watch = getattr(comm, "watch_stream", None)
        if watch is not None:  # the replay's captured collectives under the communicator's deadline
            watch(torch.cuda.current_stream(self.device), "step graph replay")
        poll = getattr(comm, "poll_errors", None)
        if poll is not None:
            poll()

    def __call__(self, *inputs: torch.Tensor) -> torch.Tensor:
        if self.graph is None:
            raise RuntimeError(f"step graph unavailable ({self.error}); run the eager step")
        for s, x in zip(self.static, inputs):
            if x is not s:
                s.copy_(x, non_blocking=True)
        self.graph.replay()
        self.replays += 1
        self.poll()  # the engine finalize's error check, which the replay does not run
        assert self.loss is not None
        return self.loss
