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
Collectives inside the step are captured too (RCCL and the IPC push kernels are
graph-capturable); the FSDP engine is not (it frees and re-allocates unit storage
between units), so it keeps the eager step.

The static inputs are the tensors the step reads; :meth:`__call__` copies a new
batch into them (device-to-device) before the replay.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch


class GraphedStep:
    def __init__(self, step_fn: Callable[..., torch.Tensor], static_inputs: Sequence[torch.Tensor],
                 warmup: int = 3):
        """``step_fn(*static_inputs)`` runs one full training step (zero_grad, forward,
        backward, optimizer step) and returns the loss tensor.  ``warmup`` eager steps
        run first on the capture stream (they are real training steps)."""
        self.static = list(static_inputs)
        dev = self.static[0].device
        self.stream = torch.cuda.Stream(dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        self.warmup_losses = []
        with torch.cuda.stream(self.stream):
            for _ in range(max(1, warmup)):
                self.warmup_losses.append(step_fn(*self.static))
        torch.cuda.current_stream(dev).wait_stream(self.stream)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            self.loss = step_fn(*self.static)
        self.replays = 0

    def __call__(self, *inputs: torch.Tensor) -> torch.Tensor:
        for s, x in zip(self.static, inputs):
            if x is not s:
                s.copy_(x, non_blocking=True)
        self.graph.replay()
        self.replays += 1
        return self.loss
