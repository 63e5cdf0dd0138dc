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
The bucket collectives of the DDP engine are captured too (RCCL and the IPC push
kernels are graph-capturable; tests/test_ipc_gpu.py replays a captured multi-rank
step against the eager one).  The FSDP engine at one rank too (every unit aliases its
shard: ``FullyShardedDataParallel.graph_capturable``); at several ranks it frees and
re-allocates unit storage between units, so it keeps the eager step.

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
from typing import Any, Callable, Optional, Sequence

import torch

logger = logging.getLogger(__name__)


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
