"""Native data-parallel engine (replacement of torch DDP's C++ Reducer).

Reference: ``DDPStrategy.prepare_model`` wraps the model in
``torch.nn.parallel.DistributedDataParallel`` with all defaults
(src/dist_strategy/ddp_strategy.py:15-21).

MI355X-first design:

* all trainable parameters are re-laid into one flat HBM buffer
  (:mod:`.flat`); gradients are views into one flat gradient buffer, so a DDP
  bucket is just a slice -- no flatten / unflatten kernels at all;
* buckets follow reverse registration order with a small first bucket so the
  first all-reduce starts early in backward; ``bucket_cap_mb="auto"`` sizes
  them from the xGMI model of :func:`.flat.xgmi_bucket_caps` (latency <= 10 %
  of a bucket's transfer, >= 6 buckets of overlap; GPT-2 small bf16 at 8
  ranks: 2.0 / 33 MiB), a number keeps torch's knob; every bucket ends on a
  multiple of world_size x 64 elements (padding in the flat layout), so a
  reduce-scatter / all-gather split of a bucket is 128-byte aligned per rank;
* ``zero_grad(set_to_none=True)`` drops the views so autograd hands each
  gradient over without an accumulate-add kernel; the native Linear backward
  writes weight / bias gradients straight into their slices (ops/lm.py
  ``_grad_dest``), and what else arrives as a fresh tensor is moved into the
  bucket slice by ONE multi-tensor copy kernel (with the 1/world_size pre-scale fused when the backend has no
  ``avg``) -- instead of one ``grad += new`` kernel per parameter;
* a post-accumulate-grad hook per parameter counts readiness; ready buckets
  are launched strictly in bucket order (identical collective order on every
  rank) on the communicator's own HIP stream (native RCCL, ``ncclAvg``), so
  they overlap with the remaining backward; the autograd-engine callback at
  the end of backward only makes the compute stream wait on the comm events
  (no host sync);
* init: parameter-shape verification across ranks + broadcast of the flat
  master buffer from rank 0 (torch's ``_verify_param_shape_across_processes``
  + ``_sync_module_states``, one collective instead of ``n_params``).

Checkpoint compatibility: ``state_dict()`` keys carry the ``module.`` prefix
exactly like torch DDP (reference checkpoint keys ``module.weight``,
``module.bias``).
"""
from __future__ import annotations

import contextlib
import hashlib
import logging
from typing import Any, Callable, Iterator, List, Optional, Tuple

import torch
import torch.nn as nn
from torch.autograd import Variable

from ..utils import profiling as prof
from .comm import Communicator, TorchComm
from .flat import FlatParamGroup, bucket_caps_for, build_flat_group, plan_buckets

logger = logging.getLogger(__name__)

MiB = 1 << 20


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, comm: Optional[Communicator] = None,
                 device: Optional[torch.device] = None, bucket_cap_mb: Any = "auto",
                 first_bucket_mb: Optional[float] = None, broadcast_buffers: bool = True,
                 param_dtype: torch.dtype = torch.float32, init_sync: bool = True) -> None:
        super().__init__()
        self.module = module
        self.comm = comm or TorchComm()
        self.device = device or next((p.device for p in module.parameters()), torch.device("cpu"))
        self.broadcast_buffers = broadcast_buffers
        self.world_size = self.comm.world_size
        named = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        if not named:
            raise ValueError("DistributedDataParallel: module has no trainable parameters")
        # bucket plan over the layout order (reverse registration), then the flat
        # layout with every bucket end padded to world_size x 64 elements
        layout = named[::-1]
        esize = torch.empty((), dtype=param_dtype).element_size()
        grad_bytes = sum(p.numel() for _, p in named) * esize
        if bucket_cap_mb in (None, "auto"):
            # measured: the α/β fit of the communicator's wrap-time all-reduce timings (RoutedComm),
            # else the assumed xGMI constants (parallel/flat.py bucket_caps_for)
            first_b, cap_b, self.bucket_caps_source = bucket_caps_for(self.comm, self.world_size, grad_bytes,
                                                                      param_dtype)
        else:
            cap_b = int(float(bucket_cap_mb) * MiB)
            first_b = MiB  # torch's dist._DEFAULT_FIRST_BUCKET_BYTES (also for first_bucket_mb="auto")
            self.bucket_caps_source = "configured"
        if first_bucket_mb not in (None, "auto"):
            first_b = int(float(first_bucket_mb) * MiB)
        self.bucket_bytes = (first_b, cap_b)
        plan = plan_buckets([p.numel() for _, p in layout], esize, cap_b, first_b)
        align = max(16, self.world_size * 64)
        self.flat: FlatParamGroup = build_flat_group(named, self.device, param_dtype=param_dtype, reverse=True,
                                                     pad_after={ids[-1]: align for ids in plan})
        self.flat.steal_ok = True
        self.buckets = self.flat.buckets_from_plan(plan)
        self._param_bucket = {}
        for b in self.buckets:
            for i in b.param_ids:
                self._param_bucket[i] = b.index
        if init_sync and self.world_size > 1:
            self._verify_shapes()
            self._sync_module_states()
        prepare = getattr(self.comm, "prepare", None)
        if prepare is not None and self.world_size > 1:
            # size-routed data planes (parallel/routed.py): every bucket's route calibrated now, not in a step
            esz = self.flat.grad.element_size()
            prepare([("all_reduce", self.flat.grad.dtype, (b.end - b.start) * esz) for b in self.buckets])
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i))
                       for i, p in enumerate(self.flat.params)]
        self.require_sync = True
        self._ov = None  # optimizer stepped bucket by bucket inside the backward (overlap_optimizer)
        self._ov_pending: list = []
        self._reset_iteration()
        logger.debug("DDP: %d params in %d bucket(s), %.2f MB flat", len(self.flat.params), len(self.buckets),
                     self.flat.total * self.flat.grad.element_size() / MiB)

    # ------------------------------------------------------------ init sync
    def _verify_shapes(self) -> None:
        sig = hashlib.sha256(repr([(n, s) for n, s in zip(self.flat.names, self.flat.shapes)]).encode()).digest()
        val = int.from_bytes(sig[:4], "little") & 0x3FFFFFFF
        dev = self.device
        t = torch.tensor([val, -val], dtype=torch.int64 if dev.type == "cpu" else torch.float64, device=dev)
        self.comm.all_reduce(t, op="max")
        if int(t[0].item()) != val or int(-t[1].item()) != val:
            raise RuntimeError("DDP: parameter names/shapes differ across ranks")

    @torch.no_grad()
    def _sync_module_states(self) -> None:
        self.comm.broadcast(self.flat.master, src=0)
        self.flat.sync_compute_from_master()
        self._broadcast_buffers()

    @torch.no_grad()
    def _broadcast_buffers(self) -> None:
        for b in self.module.buffers():
            if b.numel():
                self.comm.broadcast(b.data, src=0)

    # ------------------------------------------------------------ per step
    def reset_iteration(self) -> None:
        """Forget a step that stopped midway (e.g. a failed graph capture): hook counts,
        queued buckets and pending optimizer ranges.  A bucket all-reduce of the abandoned step
        that is still in flight writes its bucket slice on the comm stream: the current stream
        is ordered after it first, so it cannot land on top of the next step's gradients."""
        for w in self._works:
            if w is not None:
                w.wait()
        self._ov_pending = []
        self._reset_iteration()

    def _reset_iteration(self) -> None:
        self.flat.direct_claimed.clear()
        self._ready = [0] * len(self.buckets)
        self._next = 0
        self._works = []
        self._callback_queued = False
        self._pending = [[] for _ in self.buckets]

    def _make_hook(self, i: int) -> Callable[[torch.Tensor], None]:
        def hook(p: torch.Tensor) -> None:
            if not self.require_sync:
                return
            if not self._callback_queued:
                Variable._execution_engine.queue_callback(self._finalize)
                self._callback_queued = True
            b = self._param_bucket[i]
            if not self.flat.grad_is_view(i):
                self._pending[b].append(i)  # moved into the bucket by one batched copy at launch
            self._ready[b] += 1
            self._launch_ready()

        return hook

    def _launch_ready(self) -> None:
        while self._next < len(self.buckets) and self._ready[self._next] >= len(self.buckets[self._next].param_ids):
            self._launch(self._next)
            self._next += 1

    @torch.no_grad()
    def _gather_into_bucket(self, b: int, scale: float) -> bool:
        """Copy the bucket's freshly produced (non-view) gradients into its
        slice, scaled; rebind them as views.  Returns True if the whole slice
        was already pre-scaled (every gradient went through the copy)."""
        ids = self._pending[b]
        if not ids:
            return False
        fl = self.flat
        srcs = [fl.params[i].grad for i in ids]
        dsts = [fl.grad_view(i) for i in ids]
        if fl.grad.is_cuda and all(g.is_contiguous() and g.dtype == fl.grad.dtype for g in srcs):
            from ..ops import native

            native().mt_scale_copy([g.view(-1) for g in srcs], [d.view(-1) for d in dsts], scale, -1)
        else:
            for g, d in zip(srcs, dsts):
                d.copy_(g if scale == 1.0 else g * scale)
        for i, d in zip(ids, dsts):
            fl.params[i].grad = d
        self._pending[b] = []
        return len(ids) == len(self.buckets[b].param_ids)

    def _launch(self, b: int) -> None:
        with prof.range_(f"ddp.bucket{b}.allreduce"):  # host enqueue; the collective runs on the comm stream
            n = len(self._works)
            self._launch_bucket(b)
        if self._ov is not None:
            self._ov_pending.append((b, self._works[-1] if len(self._works) > n else None))
            self._ov_kick()

    def _launch_bucket(self, b: int) -> None:
        bk = self.buckets[b]
        sl = self.flat.grad[bk.start:bk.end]
        prescale = self.world_size > 1 and not self.comm.supports_avg()
        scaled = self._gather_into_bucket(b, 1.0 / self.world_size if prescale and self._whole(b) else 1.0)
        if self.world_size == 1:
            return
        if sl.is_cuda:
            from ..ops.lm import wgrad_join

            wgrad_join(sl.device)  # weight gradients still running on the side stream (ops/lm.py)
        if not prescale:
            self._works.append(self.comm.all_reduce(sl, op="avg", async_op=True))
        else:
            if not scaled:
                sl.div_(self.world_size)  # pre-divide like the torch Reducer (mul_out by 1/ws)
            self._works.append(self.comm.all_reduce(sl, op="sum", async_op=True))

    # ------------------------------------------------------------ optimizer in backward
    def overlap_optimizer(self, optimizer: Any) -> bool:
        """Run ``optimizer``'s update bucket by bucket INSIDE the backward, on a side HIP
        stream, as soon as a bucket's gradients are final (all-reduced across ranks; at one
        rank: written, including deferred weight gradients) -- the update of the late layers
        overlaps the backward of the early ones instead of following the whole backward.
        ``optimizer.step()`` then has nothing left to do for this engine's parameters.

        Valid because a bucket's parameters are read by nothing later in the same backward
        (a parameter's gradient is final only after every use of it has been
        differentiated), and the next forward is ordered after the side stream by the
        end-of-backward callback.  Not for loops that modify gradients between
        ``backward()`` and ``step()`` (clipping, unscaling): those keep the plain step.
        The update per element is the fused kernel's, so the result is bit-identical to
        ``step()``.  Returns False (nothing changed) when the optimizer or the engine do
        not qualify: a fused SGD / AdamW with one param group over exactly this engine's
        parameters, on GPU.
        Reference: the optimizer step of src/distributed_trainer.py:165 after the DDP
        backward of ddp_strategy.py:18 (torch's ``_apply_optimizer_in_backward`` idea)."""
        fl = self.flat
        if optimizer is None:
            self._ov = None  # (its flush listener stays registered but does nothing)
            return False
        if not (fl.grad.is_cuda and hasattr(optimizer, "step_range") and optimizer.range_capable(fl)):
            return False
        import weakref

        from ..ops import lm

        self._ov = optimizer
        self._ov_stream = torch.cuda.Stream(self.device)
        self._ov_first = True
        ref = weakref.ref(self)

        def on_flush() -> None:
            me = ref()
            if me is None:  # engine gone: drop this listener
                if on_flush in lm.FLUSH_LISTENERS:
                    lm.FLUSH_LISTENERS.remove(on_flush)
            elif me._ov is not None:
                me._ov_kick()

        lm.FLUSH_LISTENERS.append(on_flush)
        return True

    def _ov_range(self, b: int) -> Tuple[int, int]:
        bk = self.buckets[b]
        end = self.flat.master.numel() if b == len(self.buckets) - 1 else bk.end
        return bk.start, end

    def _ov_kick(self, force: bool = False) -> None:
        """Launch the update of every bucket whose gradients are final."""
        if not self._ov_pending:
            return
        from ..ops import lm

        if self.world_size == 1 and lm.wgrad_pending():
            if force:
                lm.wgrad_flush()  # (its listener comes back here with nothing pending)
            if lm.wgrad_pending():
                return
            if not self._ov_pending:
                return
        dev = self.flat.grad.device
        lm.wgrad_join(dev)  # deferred weight gradients launched on the current stream
        s = self._ov_stream
        s.wait_stream(torch.cuda.current_stream(dev))
        pend, self._ov_pending = self._ov_pending, []
        with torch.cuda.stream(s):
            for b, work in pend:
                if work is not None:
                    work.wait(s)
                lo, hi = self._ov_range(b)
                with prof.range_(f"ddp.bucket{b}.optimizer"):
                    self._ov.step_range(self.flat, lo, hi, self._ov_first)
                self._ov_first = False

    def _whole(self, b: int) -> bool:
        return len(self._pending[b]) == len(self.buckets[b].param_ids)

    def _finalize(self) -> None:
        with prof.range_("ddp.finalize"):
            self._finalize_impl()

    def _finalize_impl(self) -> None:
        # unused parameters: their (zeroed) grads still take part, in bucket order
        for b in range(self._next, len(self.buckets)):
            for i in self.buckets[b].param_ids:
                if i in self._pending[b]:
                    continue
                if not self.flat.grad_is_view(i):
                    self.flat.rebind_grad(i)  # unused parameter (None -> zeros) or a foreign grad
            self._launch(b)
        self._next = len(self.buckets)
        if self._ov is not None:
            self._ov_kick(force=True)
        for w in self._works:
            w.wait()
        if self._ov is not None:
            torch.cuda.current_stream(self.flat.grad.device).wait_stream(self._ov_stream)
            self._ov.end_ranges(self.flat)
            self._ov_first = True
            self.flat.stepped_in_backward = True
        self._reset_iteration()
        if self.flat.grad.is_cuda:
            from ..ops.lm import close_forward_generations

            close_forward_generations()
        if self.world_size > 1 and hasattr(self.comm, "poll_errors"):
            self.comm.poll_errors()  # a timed-out peer exchange raises here, not silently later

    def forward(self, *args: Any, **kwargs: Any) -> Any:
        if self._callback_queued:
            # the previous backward started (a hook fired) but never reached its finalize
            # callback -- it raised: forget its hook counts and queued buckets, or this step's
            # backward would never queue a finalize of its own
            self.reset_iteration()
        if self.broadcast_buffers and self.world_size > 1 and self.require_sync:
            self._broadcast_buffers()
        if self.flat.grad.is_cuda:
            from ..ops.lm import new_forward_generation

            new_forward_generation()  # native-Linear use counts (side-stream weight gradients)
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self) -> Iterator[None]:
        old = self.require_sync
        self.require_sync = False
        try:
            yield
        finally:
            self.require_sync = old

    def graph_capturable(self) -> bool:
        """The engine's per-step host logic only enqueues work on persistent buffers (bucket slices of
        the flat gradient, events), so the step can be captured as one hipGraph on the GPU -- whether
        its collectives may be is engine/step_graph.py ``capture_policy``'s call."""
        return bool(self.flat.grad.is_cuda)

    def step_messages(self) -> List[Tuple[str, torch.dtype, int]]:
        """The collectives one training step issues: ``(op, dtype, bytes)`` per bucket all-reduce."""
        esz = self.flat.grad.element_size()
        return [("all_reduce", self.flat.grad.dtype, (b.end - b.start) * esz) for b in self.buckets]

    def zero_grad(self, set_to_none: bool = True) -> None:
        self.flat.zero_grad(set_to_none)

    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Global-norm clip of the (all-reduced, replicated) flat gradient."""
        from .flat import clip_flat_grad_norm_

        return clip_flat_grad_norm_(self.flat, max_norm)

    # ------------------------------------------------------------ state
    def state_dict(self, *args: Any, **kwargs: Any) -> Any:
        sd = super().state_dict(*args, **kwargs)
        if self.flat.mixed:  # checkpoints carry the fp32 master, not the bf16 compute copy
            # matched by storage, so tied aliases (GPT-2 lm_head.weight = wte.weight) get it too
            master_of = {self.flat.param_view(i).data_ptr(): i for i in range(len(self.flat.params))}
            for key, v in sd.items():
                i = master_of.get(v.data_ptr()) if v.dtype == self.flat.param_dtype else None
                if i is not None and tuple(v.shape) == self.flat.shapes[i]:
                    sd[key] = self.flat.master_view(i).detach()
        return sd

    def load_state_dict(self, state_dict: Any, strict: bool = True) -> None:
        res = super().load_state_dict(state_dict, strict=strict)
        if self.flat.mixed:
            with torch.no_grad():
                for i, name in enumerate(self.flat.names):
                    key = f"module.{name}"
                    if key in state_dict:
                        self.flat.master_view(i).copy_(state_dict[key].to(self.flat.master.dtype))
                self.flat.sync_compute_from_master()
        return res

    def bucket_sizes(self) -> List[int]:
        return [b.end - b.start for b in self.buckets]
