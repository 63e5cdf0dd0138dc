"""Fused DDP step program for the 2-layer MLP (the headline benchmark model).

One training step on one rank = ONE hand-written gfx950 kernel
(``csrc/mlp_fused.hip``: pending SGD update + sampler gather + forward + loss +
backward, gradients pre-scaled by 1/world_size) followed by ONE RCCL
all-reduce of the flat gradient buffer (sum).  ``graph_steps`` consecutive
steps (kernel + all-reduce each) are captured into a single hipGraph and
replayed, so the host launches one graph per ``graph_steps`` steps.

Equivalence to the reference step (src/distributed_trainer.py:160-165,
zero_grad -> forward -> loss -> backward (DDP all-reduce) -> SGD step) is
exact up to bf16 MFMA operand rounding: the SGD update of step t is applied
at the start of step t+1 (or by :meth:`flush` before any read of the
weights), which is mathematically the same update order.

Batches follow ``DistributedSampler`` order exactly (per-epoch permutation,
padding and rank striding); each epoch's indices are uploaded once into a
device ring and a device-side cursor walks it.
"""
from __future__ import annotations

import contextlib
import logging
import os
import sys
import time
from typing import Any, Dict, List, Optional

import torch
import torch.nn as nn

from ..ops import mlp_fused as mf
from ..ops import native

logger = logging.getLogger(__name__)
_TRACE = bool(os.environ.get("DTA_BENCH_TRACE"))
# single-step launches at the start of the first (warm-up) call; DTA_MLP_WARM_SPLIT (A/B of the warm-up split)
_WARM_SPLIT = max(1, int(os.environ.get("DTA_MLP_WARM_SPLIT", "1")))


def fused_eligible(module: nn.Module, optimizer: Any, loader: Any, loss: str, device: torch.device) -> Optional[str]:
    """Return None when the fused program applies, else the reason it does not."""
    from ..data.datasets import DeviceDataLoader
    from ..models.mlp import MLP

    if device.type != "cuda":
        return "not a GPU run"
    if not isinstance(module, MLP) or module.num_layers != 2:
        return "model is not a 2-layer MLP"
    if module.activation not in mf.ACTIVATIONS:
        return f"activation {module.activation} not fused"
    if loss not in mf.LOSSES:
        return f"loss {loss} not fused"
    if not isinstance(loader, DeviceDataLoader) or not hasattr(loader.dataset, "X"):
        return "loader is not a device-resident feature loader"
    if len(optimizer.param_groups) != 1:
        return "optimizer has several param groups"
    g = optimizer.param_groups[0]
    if "momentum" not in g or "betas" in g:
        return "optimizer is not SGD"
    if g.get("momentum", 0) and g.get("dampening", 0):
        return "SGD dampening not fused"
    if not mf.supported(module.input_size, module.hidden[0], module.output_size, loader.batch_size,
                        momentum=bool(g.get("momentum", 0))):
        return "shape outside the fused kernel's limits"
    return None


class FusedMLPProgram:
    """Two execution modes:

    * persistent (full batches, shapes within the persistent kernel's limits):
      ``csrc/mlp_persistent.hip`` runs up to ~1000 complete steps per launch in
      one workgroup with the parameters resident in LDS; across ranks the
      gradients are exchanged inside the loop through IPC-mapped LL slots
      (one-shot, or reduce-scatter + all-gather);
    * per-step (otherwise): the multi-workgroup fused step kernel + gradient
      all-reduce, hipGraph-replayed.

    With several ranks the form is chosen by timing all of them on the node
    (``DTA_MLP_XMODE=auto``, the default; or force oneshot / rsag / step).
    """

    def __init__(self, module: Any, optimizer: Any, loader: Any, comm: Any, loss: str = "mse", graph_steps: int = 32,
                 own_tiles: Optional[int] = None, allreduce_world1: bool = True, loss_len: int = 4096,
                 persistent: Optional[bool] = None) -> None:
        self.module = module
        self.opt = optimizer
        self.loader = loader
        self.comm = comm
        self.loss = loss
        self.act = module.activation
        self.ws = comm.world_size
        self.device = loader.device
        self.B = loader.batch_size
        H = module.hidden[0]
        self.layout = mf.make_layout(module.input_size, H, module.output_size)
        nt = H // 32
        self.own_tiles = own_tiles or max(1, min(8, nt // 8 if nt >= 64 else (nt + 15) // 16 if nt > 8 else 1))
        if self.own_tiles > 8:
            self.own_tiles = 8
        self.graph_steps = max(2, graph_steps + (graph_steps % 2))  # even: ping-pong parity preserved
        self.allreduce_world1 = allreduce_world1
        dev = self.device
        T = self.layout.total
        self.P = [torch.zeros(T, device=dev) for _ in range(2)]
        self.G = [torch.zeros(T, device=dev) for _ in range(2)]
        hp = self.hyper()
        self.use_mom = bool(hp["momentum"])
        self.M = [torch.zeros(T, device=dev) for _ in range(2)] if self.use_mom else [None, None]
        self.X, self.Y = loader.tensors()
        self.X = self.X.float().contiguous()
        self.Y = self.Y.float().contiguous()
        self.steps_per_epoch = S = max(1, len(loader))
        full_batches = len(loader.sampler) % self.B == 0
        if persistent is None:
            persistent = os.environ.get("DTA_MLP_PERSISTENT", "1") != "0"
        self.persistent = bool(persistent and full_batches and mf.persistent_supported(
            module.input_size, H, module.output_size, self.B, momentum=bool(self.hyper()["momentum"]), world=self.ws))
        self._p2p = None
        self._xinfo = None
        self._xinfos = {}
        self.xepoch = torch.zeros(1, dtype=torch.int32, device=dev)
        # DDP across ranks: the persistent loop's in-kernel exchange ("oneshot" |
        # "rsag" | "helpers"), the per-step program ("step": multi-workgroup step kernel +
        # all-reduce), or "auto": all are timed on this node at construction and
        # every rank takes the fastest (xGMI latency and the store rate of the
        # loop's single CU decide it; neither is knowable off the target node)
        self.xmode = os.environ.get("DTA_MLP_XMODE", "auto")
        if self.xmode not in ("auto", "step", *mf.XMODES):
            raise ValueError(f"DTA_MLP_XMODE={self.xmode!r}")
        if self.xmode == "step" and self.ws > 1:
            self.persistent = False
        auto_x = self.xmode == "auto"
        if auto_x:
            self.xmode = "oneshot"
        if self.persistent and self.ws > 1:
            self.persistent = self._setup_exchange()
        self.chunk_steps = 1024
        # index ring: whole epochs, at least one graph (or one persistent launch)
        # beyond an epoch, so uploads for epoch e+1 can be enqueued while epoch
        # e's steps are still queued
        # persistent: room for two launches plus an epoch, so the next launch's
        # indices upload on a side stream while the current launch runs (slots
        # of the two launches never overlap; _run_persistent)
        ahead = 3 * self.chunk_steps if self.persistent else 2 * self.graph_steps
        k = max(2, -(-ahead // S) + 1)
        self.R = S * k
        self.ring = torch.zeros(self.R, self.B, dtype=torch.int32, device=dev)
        self.cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self.stage = mf.make_stage(dev)
        self.loss_ring = torch.zeros(loss_len, device=dev)
        self._staging: List = []   # (pinned tensor, event) kept alive until the copy ran
        # persistent mode: index uploads on their own stream, ordered after the
        # launch before the current one (whose ring slots they may reuse) and
        # before the launch that reads them
        self._up_stream = torch.cuda.Stream(dev) if self.persistent and dev.type == "cuda" else None
        self._up_fence_at = -1  # value of `launched` when the upload stream last waited on the compute stream
        self._up_done = None
        self._graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self._plaunch = None  # (key, packed persistent launch): re-packed when the form or hyper-parameters change
        self.loss_cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self.mom_started_dev = torch.zeros(1, dtype=torch.int32, device=dev)  # persistent mode
        self.Xp = mf.pad_features(self.X) if self.persistent else None
        self._reset_state()
        if auto_x and self.persistent and self.ws > 1:
            self._calibrate_exchange()

    def _reset_state(self) -> None:
        """Training state back to step 0 with the module's weights (the module
        itself is only written by :meth:`store_to_module`)."""
        if self._up_stream is not None:  # uploads in flight land before the ring is cleared ...
            torch.cuda.current_stream(self.device).wait_stream(self._up_stream)
            self._up_fence_at, self._up_done = -1, None
        for t in (*self.P, *self.G, *(m for m in self.M if m is not None)):
            t.zero_()
        self.ring.zero_()
        if self._up_stream is not None:  # ... and later ones after it
            self._up_stream.wait_stream(torch.cuda.current_stream(self.device))
        self.cursor.zero_()
        self.loss_ring.zero_()
        self.loss_cursor.zero_()
        self.mom_started_dev.zero_()
        self.staged = False        # staging slot `parity` holds the batch of step `launched`
        self.parity = 0
        self.pending = False
        self.mom_started = False
        self.launched = 0          # global steps enqueued (== device cursor when drained)
        self.host_step = 0         # global steps whose indices are uploaded
        self._last_start = 0       # first step of the last persistent launch
        self.next_epoch = 0        # next epoch to upload
        self._batch_of: Dict[int, int] = {}
        self.load_from_module()

    def _calibrate_exchange(self, steps: int = 256) -> None:
        """Time both exchange forms of the persistent loop on this node (xGMI
        topology, store issue rate of one CU) and keep the faster; every rank
        takes the same decision (MAX over ranks of each time).  The probe steps
        are discarded: the state is reset to step 0 afterwards."""
        import torch.distributed as dist

        times = {}
        can_step = hasattr(self.comm, "all_reduce_inline") or hasattr(self.comm, "all_reduce")
        for mode in (*self._xinfos, *(("step",) if can_step else ())):
            self.persistent = mode != "step"
            if self.persistent:
                self.xmode = mode
                self._xinfo = self._xinfos[mode]
            self._reset_state()
            self.run_steps(2 * self.graph_steps + 8)  # warm (first touch of the slots, graph capture)
            torch.cuda.synchronize(self.device)
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self.run_steps(steps)
            e1.record()
            torch.cuda.synchronize(self.device)
            ms = e0.elapsed_time(e1)
            # a form whose exchange timed out anywhere is ruled out (inf), not fatal:
            # the error flag is re-armed on every rank and the next form is probed
            if self._p2p._h.error() or (hasattr(self.comm, "_p2p") and self.comm._p2p is not None
                                        and self.comm._p2p._h.error()):
                logger.warning("MLP DDP step form %s timed out during calibration; excluded", mode)
                ms = float("inf")
            t = torch.tensor([ms], dtype=torch.float64,
                             device=self.device if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            times[mode] = float(t.item())
            if times[mode] == float("inf"):
                torch.cuda.synchronize(self.device)
                dist.barrier()
                self._p2p._h.clear_error()
                if hasattr(self.comm, "_p2p") and self.comm._p2p is not None:
                    self.comm._p2p._h.clear_error()
                torch.cuda.synchronize(self.device)
                dist.barrier()
        if all(v == float("inf") for v in times.values()):
            raise RuntimeError("no MLP DDP step form completed its calibration exchange")
        best = min(times, key=times.get)
        self.persistent = best != "step"
        self.xmode = best
        if self.persistent:
            self._xinfo = self._xinfos[best]
        self.exchange_times_ms = times
        logger.info("MLP DDP step form: %s (%s)", self.xmode,
                    ", ".join(f"{m} {v / steps * 1e3:.2f} us/step" for m, v in times.items()))
        torch.cuda.synchronize(self.device)
        self._reset_state()

    def _setup_exchange(self) -> bool:
        """DDP across ranks inside the persistent loop: a dedicated p2p buffer set
        whose LL slots the kernel writes directly (collective; every rank agrees)."""
        import torch.distributed as dist

        from ..parallel.p2p import P2PAllReduce, intra_node

        ok = 1
        if not (dist.is_initialized() and intra_node() and self.ws <= 8):
            ok = 0
        p2p = None
        if ok:
            try:
                # [2][world][slot] one-shot / reduce-scatter slots + [2][slot] all-gather slots;
                # the slot covers the parameters and the helper form's fragment-order array
                L = self.layout
                XE = mf.helper_elems(L.hidden, L.out_dim)
                T = max(L.total, XE)
                p2p = P2PAllReduce(self.comm.rank, self.ws, self.device, dist.distributed_c10d._get_default_store(),
                                   tag="fused_mlp", max_elems=T + -(-T // self.ws) + 64)
                # the kernel pushes through the same peer mappings: prove them with
                # one exchange of known values before any training step relies on them
                n = self.layout.total
                x = torch.arange(n, device=self.device, dtype=torch.float32) * (self.comm.rank + 1)
                p2p.all_reduce(x, 1.0)
                want = torch.arange(n, device=self.device, dtype=torch.float32) * (self.ws * (self.ws + 1) / 2)
                torch.cuda.synchronize(self.device)
                p2p.check()
                if not torch.equal(x, want):
                    raise RuntimeError("p2p self-test mismatch")
                # the self-test left {value, tag 1} in the slots: the loop's first
                # exchange epoch must be past it (epochs are xepoch + 1, + 2, ...)
                self.xepoch.fill_(1)
                hb = mf.helper_buffers(p2p, L.hidden, L.out_dim)
                self._xinfos = {m: mf.exchange_info(p2p, self.xepoch, T, m, helper=hb)
                                for m in mf.XMODES if m != "helpers" or hb is not None}
                if self.xmode not in self._xinfos:
                    raise RuntimeError(f"exchange form {self.xmode} unavailable")
                self._xinfo = self._xinfos[self.xmode]
            except Exception as e:  # noqa: BLE001 - fall back to the per-step program
                logger.warning("persistent DDP exchange unavailable (%s); per-step program used", e)
                ok = 0
        flag = torch.tensor([ok], dtype=torch.int32,
                            device=self.device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) != 1:
            if p2p is not None:
                p2p.destroy()
            self._xinfo = None
            return False
        self._p2p = p2p
        return True

    # ------------------------------------------------------------ state sync
    def hyper(self) -> Dict[str, float]:
        g = self.opt.param_groups[0]
        return {"lr": g["lr"], "momentum": g.get("momentum", 0.0), "dampening": g.get("dampening", 0.0),
                "weight_decay": g.get("weight_decay", 0.0), "nesterov": g.get("nesterov", False),
                "maximize": g.get("maximize", False)}

    @torch.no_grad()
    def load_from_module(self) -> None:
        """Copy the module's weights in (fp32 master copy when the DDP engine
        keeps one, so bf16 compute copies never round the master)."""
        v = self.layout.views(self.P[self.parity])
        for name, p in self.module.named_parameters():
            tag = getattr(p, "_dta_flat", None)
            src = tag[0].master_view(tag[1]) if tag is not None else p.detach()
            v[name].copy_(src.float())

    @torch.no_grad()
    def flush(self) -> None:
        """Apply the pending SGD update (so P[parity] holds the current weights)."""
        if self.persistent or not self.pending:
            return
        hp = self.hyper()
        c = self.parity
        native().flat_sgd(self.P[c], self.P[c], self.G[1 - c], self.M[c], None, hp["lr"], hp["momentum"],
                          hp["dampening"], hp["weight_decay"], 1.0, hp["nesterov"], hp["maximize"],
                          not self.mom_started, -1)
        self.mom_started = True
        self.pending = False

    @torch.no_grad()
    def store_to_module(self) -> None:
        self.flush()
        if hasattr(self.comm, "check_errors"):
            self.comm.check_errors()  # a p2p all-reduce that timed out on a dead peer raises here
        if self._p2p is not None:
            self._p2p.check()
        v = self.layout.views(self.P[self.parity])
        for name, p in self.module.named_parameters():
            tag = getattr(p, "_dta_flat", None)
            if tag is not None:
                tag[0].master_view(tag[1]).copy_(v[name])
            p.copy_(v[name].to(p.dtype))

    # ------------------------------------------------------------ stepping
    def _launch(self, batch: int, apply_update: bool, first_mom: bool, parity: int, gather_self: bool) -> None:
        hp = self.hyper()
        c = parity
        mf.fused_step(self.X, self.Y, self.ring, self.cursor, self.stage, self.loss_ring, self.P[c],
                      self.P[1 - c], self.G[1 - c], self.G[c], self.M[c], self.M[1 - c], self.layout, batch,
                      self.own_tiles, self.act, self.loss, apply_update, 1.0 / self.ws, hp, 1.0, first_mom,
                      parity=c, gather_self=gather_self)
        if gather_self:
            self.cursor.add_(1)
        if self.ws > 1 or self.allreduce_world1:
            self._allreduce(self.G[c])

    def _allreduce(self, t: torch.Tensor) -> None:
        if hasattr(self.comm, "all_reduce_inline"):
            self.comm.all_reduce_inline(t, "sum")
        else:
            self.comm.all_reduce(t, op="sum")

    def _eager_step(self, batch: int) -> None:
        first_mom = self.use_mom and self.pending and not self.mom_started
        self._launch(batch, self.pending, first_mom, self.parity, gather_self=not self.staged)
        if self.pending and self.use_mom:
            self.mom_started = True
        self.pending = True
        self.staged = True
        self.parity ^= 1

    def _graph(self, parity: int) -> torch.cuda.CUDAGraph:
        g = self._graphs.get(parity)
        if g is not None:
            return g
        # steady state only: pending update present, momentum already started
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                p = parity
                for _ in range(self.graph_steps):
                    self._launch(self.B, True, False, p, gather_self=False)
                    p ^= 1
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._graphs[parity] = g
        return g

    # ------------------------------------------------------------ indices
    def seek_epoch(self, epoch: int) -> None:
        """Position the index stream at ``epoch`` (only between epochs)."""
        if self.host_step != self.launched:
            raise RuntimeError("seek_epoch with uploaded-but-unrun steps")
        self.next_epoch = epoch
        self.staged = False

    def _upload_epoch(self) -> None:
        e = self.next_epoch
        S, B, R = self.steps_per_epoch, self.B, self.R
        # slots of steps still to run are never overwritten; with side-stream uploads
        # the launch in flight (from _last_start on) must keep its slots as well
        side = self._up_stream is not None and self.persistent  # (calibration may pick the per-step form)
        floor = self._last_start if side else self.launched
        assert self.host_step + S - R <= floor, "index ring overrun"
        self.loader.sampler.set_epoch(e)
        idx = self.loader.epoch_indices().to(torch.int32)
        host = self._pinned_buffer(S, B)
        host.view(-1)[: idx.numel()] = idx
        host.view(-1)[idx.numel():] = 0
        last = idx.numel() - (S - 1) * B
        r0 = self.host_step % R
        n1 = min(S, R - r0)
        up = self._up_stream if side else None
        compute = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(up) if up is not None else contextlib.nullcontext():
            if up is not None and self._up_fence_at != self.launched:
                # the overwritten slots belong to launches before the current one (ring
                # assertion above); waiting for every launch enqueued so far is a superset
                # that needs one event per upload batch instead of one per launch (an event
                # behind every launch would add a marker packet to each timed region)
                fence = torch.cuda.Event()
                fence.record(compute)
                up.wait_event(fence)
                self._up_fence_at = self.launched
            self.ring[r0:r0 + n1].copy_(host[:n1], non_blocking=True)
            if n1 < S:
                self.ring[0:S - n1].copy_(host[n1:], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        if up is not None:
            self._up_done = ev
        self._staging.append((host, ev))
        for j in range(S):
            self._batch_of[self.host_step + j] = B if j < S - 1 else last
        self.host_step += S
        self.next_epoch += 1

    def _pinned_buffer(self, S: int, B: int) -> torch.Tensor:
        """A pinned [S, B] int32 host buffer whose previous H2D copy has run
        (pinned allocation costs ~ms: buffers are recycled, not re-allocated)."""
        keep = []
        free = None
        for h, ev in self._staging:
            if free is None and ev.query():
                free = h
            else:
                keep.append((h, ev))
        self._staging = keep
        if free is None:
            free = torch.empty(S, B, dtype=torch.int32).pin_memory()
        return free

    def _ensure(self, upto: int) -> None:
        while self.host_step < upto:
            self._upload_epoch()

    # ------------------------------------------------------------ stepping API
    def _run_persistent(self, n: int) -> None:
        # (no autograd context: only native launches and plain copies happen here, and
        # the timed region of a short bench call is a few dozen microseconds)
        _T = [time.perf_counter()] if _TRACE else None
        end = self.launched + n
        first_call = self.launched == 0
        g = self.opt.param_groups[0]
        hkey = (g["lr"], g.get("momentum", 0.0), g.get("dampening", 0.0), g.get("weight_decay", 0.0),
                g.get("nesterov", False), g.get("maximize", False))
        if self.launched == 0 and self._up_stream is not None:
            # first call (warm-up): upload two launches of indices before the first
            # launch, so later short calls find them in place and the device is not
            # left idle between the warm-up launch and the next call
            self._ensure(min(2 * self.chunk_steps, self.R - self.steps_per_epoch))
        while self.launched < end:
            k = min(end - self.launched, self.chunk_steps)
            if first_call and self.launched < _WARM_SPLIT and end - self.launched > 1:
                # the first call (the warm-up) runs its steps as 1 + rest launches (_WARM_SPLIT single-step
                # launches first): on the gpurun boxes the SECOND launch of the program paid ~14-17 us inside
                # hipLaunchKernel (the third ~1 us), which otherwise lands on the first timed call.
                # Warm-up accounting only -- the per-step kernel time is unchanged
                # (profiles/headline_split_first_launch.txt)
                k = 1
            self._ensure(self.launched + k)
            if self._up_done is not None:
                # an upload that already landed needs no cross-stream dependency (a wait
                # packet ahead of the launch costs dispatch latency on the timed path)
                if not self._up_done.query():
                    torch.cuda.current_stream(self.device).wait_event(self._up_done)
                self._up_done = None
            key = (id(self._xinfo), hkey)
            if self._plaunch is None or self._plaunch[0] != key:
                hp = self.hyper()
                self._plaunch = (key, mf.persistent_prepare(
                    self.Xp, self.Y, self.ring, self.cursor, self.loss_ring, self.loss_cursor, self.mom_started_dev,
                    self.P[0], self.M[0], self.layout, self.B, self.act, self.loss, 1.0 / self.ws, hp,
                    xinfo=self._xinfo))
            if _T is not None:
                _T.append(time.perf_counter())
            self._plaunch[1].launch(k)
            if _T is not None:
                _T.append(time.perf_counter())
            self._last_start = self.launched
            for j in range(k):
                self._batch_of.pop(self.launched + j, None)
            self.launched += k
            self._prefetch()
        if _T is not None:
            _T.append(time.perf_counter())
            print("[fused_mlp] run_persistent us:", [round(1e6 * (b - a), 1) for a, b in zip(_T, _T[1:])],
                  file=sys.stderr)

    def _prefetch(self) -> None:
        """Pipelined index loading: while a launch runs, upload the indices of
        the next one (host sampler work + H2D on the side stream), so the next
        ``run_steps`` call -- e.g. the first after a warm-up -- finds them ready.
        The sampler's epoch is left as it was."""
        if self._up_stream is None or not self.persistent:
            return
        # hysteresis: top up only below one launch of indices ahead, then fill to two,
        # so a short run_steps call (e.g. a 20-step timed region after warm-up) finds
        # everything uploaded and does no host sampler work behind its launch
        if self.host_step - self.launched >= self.chunk_steps:
            return
        S = self.steps_per_epoch
        upto = min(self.launched + 2 * self.chunk_steps, self._last_start + self.R - S)
        sampler = self.loader.sampler
        ep = getattr(sampler, "epoch", None)
        self._ensure(upto)
        if ep is not None:
            sampler.set_epoch(ep)

    def run_steps(self, n: int) -> None:
        """Enqueue ``n`` training steps (crossing epochs as needed)."""
        if self.persistent:
            self._run_persistent(n)
            return
        self._run_eager(n)

    @torch.no_grad()
    def _run_eager(self, n: int) -> None:
        end = self.launched + n
        while self.launched < end:
            U = self.graph_steps
            steady = self.pending and self.staged and (self.mom_started or not self.use_mom)
            if steady and end - self.launched >= U:
                self._ensure(self.launched + U + 1)  # +1: the last step stages its successor
                if all(self._batch_of[self.launched + j] == self.B for j in range(U)):
                    self._graph(self.parity).replay()
                    for j in range(U):
                        self._batch_of.pop(self.launched + j, None)
                    self.launched += U  # parity unchanged (even number of steps)
                    continue
            self._ensure(self.launched + 2)
            self._eager_step(self._batch_of.pop(self.launched))
            self.launched += 1

    def run_epoch(self, epoch: int) -> int:
        S = self.steps_per_epoch
        ahead = (self.host_step - self.launched) // S  # whole epochs uploaded ahead (prefetch)
        if self.launched % S == 0 and self.next_epoch - ahead != epoch:
            # the prefetched epochs are not the requested one: drop them (nothing has
            # read their ring slots) and restart the index stream at ``epoch``
            for j in range(self.launched, self.host_step):
                self._batch_of.pop(j, None)
            self.host_step = self.launched
            self.seek_epoch(epoch)
        self.run_steps(S)
        return S

    def last_losses(self, n: int) -> torch.Tensor:
        """Losses of the last ``n`` launched steps (oldest first)."""
        L = self.loss_ring.numel()
        idx = [(self.launched - 1 - k) % L for k in range(min(n, self.launched, L))]
        return self.loss_ring[idx].flip(0) if idx else torch.zeros(0)
