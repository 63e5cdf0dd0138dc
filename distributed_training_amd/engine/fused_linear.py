"""Fused step program for the reference's default model.

The reference trains ONE ``nn.Linear(20, 1)`` with ``F.cross_entropy`` against
float targets, fp32, ``torch.optim.SGD`` and DDP (src/distributed_trainer.py:
160-165, 199-200; conf/model/default.yaml).  Its step is ~15 small ATen
launches plus the DDP reducer.  Here:

* one rank: ``csrc/linear_step.hip`` runs a whole epoch of complete steps
  (sampler-order gather, forward, loss, backward, SGD) in ONE launch with the
  parameters resident in LDS;
* several ranks: one launch per step (pending SGD update from the previous
  step's all-reduced gradients + gather + forward + loss + backward, gradients
  pre-scaled by 1/world_size) followed by the all-reduce of the 84-byte
  gradient bucket (the p2p one-shot all-reduce for small buckets on xGMI, or
  RCCL), the epoch's steps captured once into a hipGraph and replayed.

Numerics are fp32 like the reference; batches follow ``DistributedSampler``
order exactly (indices uploaded per epoch into a device ring).
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List, Optional

import torch
import torch.nn as nn

from ..ops import native

logger = logging.getLogger(__name__)

LOSS_KINDS = {"mse": 0, "cross_entropy": 1}


def linear_eligible(module: nn.Module, optimizer: Any, loader: Any, loss: str, device: torch.device) -> Optional[str]:
    """None when the fused Linear program applies, else the reason it does not."""
    from ..data.datasets import DeviceDataLoader

    if device.type != "cuda":
        return "not a GPU run"
    if type(module) is not nn.Linear or module.bias is None:
        return "model is not a single nn.Linear with bias"
    if loss not in LOSS_KINDS:
        return f"loss {loss} not fused"
    if not isinstance(loader, DeviceDataLoader) or not hasattr(loader.dataset, "X"):
        return "loader is not a device-resident feature loader"
    if len(optimizer.param_groups) != 1:
        return "optimizer has several param groups"
    g = optimizer.param_groups[0]
    if "momentum" not in g or "betas" in g:
        return "optimizer is not SGD"
    C, I = module.weight.shape
    if not native().linear_step_supported(I, C, loader.batch_size, False):
        return "shape outside the fused kernel's limits"
    return None


class FusedLinearProgram:
    def __init__(self, module: nn.Linear, optimizer: Any, loader: Any, comm: Any, loss: str = "cross_entropy",
                 loss_len: int = 4096) -> None:
        self.module = module
        self.opt = optimizer
        self.loader = loader
        self.comm = comm
        self.loss_kind = LOSS_KINDS[loss]
        self.ws = comm.world_size
        self.device = dev = loader.device
        C, I = module.weight.shape
        self.C, self.I, self.B = C, I, loader.batch_size
        self.NP = C * I + C
        self.P = torch.zeros(self.NP, device=dev)
        self.use_mom = bool(self.hyper()["momentum"])
        self.M = torch.zeros(self.NP, device=dev) if self.use_mom else None
        self.G = torch.zeros(self.NP, device=dev) if self.ws > 1 else None
        X, Y = loader.tensors()
        self.X = X.float().contiguous()
        self.T = Y.float().reshape(Y.shape[0], -1).contiguous()
        if self.T.shape[1] != C:
            raise ValueError(f"targets have {self.T.shape[1]} columns, the model {C} outputs")
        self.S = max(1, len(loader))  # steps per epoch
        self.R = 2 * self.S           # two epochs of index slots: upload e+1 while e may still run
        self.ring = torch.zeros(self.R, self.B, dtype=torch.int32, device=dev)
        self.counts = torch.zeros(self.R, dtype=torch.int32, device=dev)
        self.cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self.flags = torch.zeros(2, dtype=torch.int32, device=dev)  # momentum started, update pending
        self.loss_ring = torch.zeros(loss_len, device=dev)
        self.loss_cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self.launched = 0
        self._next_epoch = 0
        self._graph = None
        self._graph_key = None
        self._staging: List = []
        self.load_from_module()

    # ------------------------------------------------------------ state sync
    def hyper(self) -> Any:
        g = self.opt.param_groups[0]
        return {"lr": g["lr"], "momentum": g.get("momentum", 0.0), "dampening": g.get("dampening", 0.0),
                "weight_decay": g.get("weight_decay", 0.0), "nesterov": bool(g.get("nesterov", False)),
                "maximize": bool(g.get("maximize", False))}

    def _views(self) -> Any:
        C, I = self.C, self.I
        return {"weight": self.P[:C * I].view(C, I), "bias": self.P[C * I:]}

    def _mom_views(self) -> Dict[str, torch.Tensor]:
        assert self.M is not None
        C, I = self.C, self.I
        return {"weight": self.M[:C * I].view(C, I), "bias": self.M[C * I:]}

    @torch.no_grad()
    def load_from_module(self) -> None:
        v = self._views()
        for name, p in self.module.named_parameters():
            tag = getattr(p, "_dta_flat", None)  # fp32 master of the DDP engine, if it keeps one
            src = tag[0].master_view(tag[1]) if tag is not None else p.detach()
            v[name].copy_(src.float())
        if self.M is not None:
            # the momentum lives in the program's buffer while it runs and in the optimizer's
            # state (so in a checkpoint's OPTIM_STATE) between runs: a resumed run continues it
            mv = self._mom_views()
            started = False
            for name, p in self.module.named_parameters():
                buf = self.opt.state.get(p, {}).get("momentum_buffer")
                if buf is not None:
                    mv[name].copy_(buf.reshape(mv[name].shape).float())
                    started = True
            self.flags[0] = int(started)

    @torch.no_grad()
    def flush(self) -> None:
        """Apply a pending update (several ranks: the last step's all-reduced gradients)."""
        if self.G is not None:
            self._kernel(0, g_out=False)

    @torch.no_grad()
    def store_to_module(self) -> None:
        self.flush()
        if hasattr(self.comm, "check_errors"):
            self.comm.check_errors()
        v = self._views()
        for name, p in self.module.named_parameters():
            tag = getattr(p, "_dta_flat", None)
            if tag is not None:
                tag[0].master_view(tag[1]).copy_(v[name])
            p.copy_(v[name].to(p.dtype))
        if self.M is not None and int(self.flags[0].item()):
            mv = self._mom_views()
            for name, p in self.module.named_parameters():
                self.opt.state[p]["momentum_buffer"] = mv[name].reshape(p.shape).clone()

    # ------------------------------------------------------------ stepping
    def _kernel(self, nsteps: int, g_out: bool) -> None:
        hp = self.hyper()
        native().linear_step(self.X, self.T, self.ring, self.counts, self.cursor, self.P, self.M, self.flags,
                             self.G, self.G if g_out else None, self.loss_ring, self.loss_cursor, int(nsteps),
                             self.loss_kind, hp["lr"], hp["momentum"], hp["dampening"], hp["weight_decay"],
                             1.0 / self.ws, hp["nesterov"], hp["maximize"], -1)

    def _allreduce(self) -> None:
        if hasattr(self.comm, "all_reduce_inline"):
            self.comm.all_reduce_inline(self.G, "sum")
        else:
            self.comm.all_reduce(self.G, op="sum")

    def _upload(self, epoch: int) -> None:
        S, B = self.S, self.B
        assert self.launched % S == 0, "epochs are uploaded whole"
        self.loader.sampler.set_epoch(epoch)
        idx = self.loader.epoch_indices().to(torch.int32)
        n = idx.numel()
        if n and (int(idx.min()) < 0 or int(idx.max()) >= self.X.shape[0]):
            raise IndexError("sampler index outside the dataset")
        # one pinned block: [S, B] indices then the S per-step batch sizes
        host = torch.zeros(S * B + S, dtype=torch.int32).pin_memory()
        host[:n] = idx
        host[S * B:] = B
        host[S * B + S - 1] = n - (S - 1) * B
        base = self.launched % self.R
        self.ring[base:base + S].copy_(host[:S * B].view(S, B), non_blocking=True)
        self.counts[base:base + S].copy_(host[S * B:], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        # keep each pinned block alive until its copies ran
        self._staging = [(h, e) for h, e in self._staging if not e.query()] + [(host, ev)]

    def _epoch_graph(self) -> torch.cuda.CUDAGraph:
        key = tuple(sorted(self.hyper().items()))
        if self._graph is not None and self._graph_key == key:
            return self._graph
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(self.S):
                    self._kernel(1, g_out=True)
                    self._allreduce()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._graph, self._graph_key = g, key
        return g

    @torch.no_grad()
    def run_steps(self, n: int) -> None:
        """Enqueue ``n`` training steps, crossing epochs (sampler epochs 0, 1, ... or
        from the epoch given to :meth:`run_epoch`)."""
        while n > 0:
            off = self.launched % self.S
            if off == 0:
                self._upload(self._next_epoch)
                self._next_epoch += 1
            k = min(n, self.S - off)
            if self.ws == 1:
                self._kernel(k, g_out=False)
            elif off == 0 and k == self.S and self.launched > 0:
                self._epoch_graph().replay()  # (the first epoch runs eagerly: graph capture needs warm communicators)
            else:
                for _ in range(k):
                    self._kernel(1, g_out=True)
                    self._allreduce()
            self.launched += k
            n -= k

    def run_epoch(self, epoch: int) -> int:
        if self.launched % self.S:
            raise RuntimeError("run_epoch in the middle of an epoch")
        self._next_epoch = epoch
        self.run_steps(self.S)
        return self.S

    def last_losses(self, n: int) -> torch.Tensor:
        L = self.loss_ring.numel()
        idx = [(self.launched - 1 - k) % L for k in range(min(n, self.launched, L))]
        return self.loss_ring[idx].flip(0) if idx else torch.zeros(0)
