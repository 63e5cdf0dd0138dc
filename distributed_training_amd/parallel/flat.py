"""Flat, HBM-resident parameter / gradient storage.

MI355X-first layout: every trainable parameter of a module lives as a view
into ONE contiguous fp32 master buffer (and, under bf16 mixed precision, one
bf16 compute buffer), and every gradient is a view into ONE contiguous
gradient buffer.  Consequences:

* DDP buckets are plain slices of the gradient buffer ("grads as bucket
  views"): no flatten/unflatten copies (the reference's DDP Reducer copies
  grad x 1/ws into the bucket and back);
* the fused optimizer updates the whole model with ONE kernel over the flat
  buffer (fp32 master -> bf16 compute copy in the same pass);
* every region starts on a 64-byte boundary so kernels use 16-byte accesses.

Parameters keep their identity (``nn.Parameter`` objects are not replaced:
only ``.data`` is re-pointed), so an optimizer created before wrapping -- as
the reference does (src/distributed_trainer.py:195-201 creates SGD before
Trainer wraps the model) -- keeps working.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch

ALIGN_ELEMS = 16


def _align(n: int, a: int = ALIGN_ELEMS) -> int:
    return (n + a - 1) // a * a


@dataclass
class Bucket:
    index: int
    start: int            # element offset in the flat buffers
    end: int
    param_ids: List[int]  # indices into FlatParamGroup.params


class FlatParamGroup:
    def __init__(self, params: Sequence[torch.nn.Parameter], device: torch.device,
                 param_dtype: torch.dtype = torch.float32, grad_dtype: Optional[torch.dtype] = None,
                 names: Optional[Sequence[str]] = None, pad_after: Optional[Dict[int, int]] = None,
                 pin_memory: bool = False) -> None:
        self.params: List[torch.nn.Parameter] = list(params)
        self.names = list(names) if names is not None else [f"p{i}" for i in range(len(self.params))]
        self.device = device
        self.param_dtype = param_dtype
        self.grad_dtype = grad_dtype or param_dtype
        self.shapes = [tuple(p.shape) for p in self.params]
        self.numels = [p.numel() for p in self.params]
        self.offsets: List[int] = []
        off = 0
        pad_after = pad_after or {}
        for i, n in enumerate(self.numels):
            self.offsets.append(off)
            off = _align(off + n, pad_after.get(i, ALIGN_ELEMS))  # bucket ends: world_size x 64 elements
        self.total = max(off, ALIGN_ELEMS)
        self.pad_after = dict(pad_after)
        self.master = torch.zeros(self.total, dtype=torch.float32, device=device)
        if pin_memory and self.master.device.type == "cpu":  # host-resident shards (FSDP cpu_offload)
            self.master = self.master.pin_memory()
        with torch.no_grad():
            for p, o, n in zip(self.params, self.offsets, self.numels):
                self.master[o:o + n].copy_(p.detach().reshape(-1).to(torch.float32))
        self.mixed = param_dtype != torch.float32
        self.compute = self.master if not self.mixed else self.master.to(param_dtype)
        self.grad = torch.zeros(self.total, dtype=self.grad_dtype, device=device)
        if pin_memory and self.grad.device.type == "cpu":
            self.grad = self.grad.pin_memory()
        # set by an engine whose backward hooks move fresh gradients into the
        # flat buffer (DDP): zero_grad(set_to_none=True) may then drop the views
        self.steal_ok = False
        # set by an engine that writes every gradient slice itself in the next
        # backward (FSDP reduce-scatters into the slices): zero_grad(set_to_none)
        # then drops the gradients and calls it instead of zero-filling the buffer
        self.fresh_hook: Optional[Callable[[], None]] = None
        # parameters whose gradient a backward already wrote straight into its
        # slice since the last zero_grad(set_to_none) (ops/lm.py _grad_dest)
        self.direct_claimed: set = set()
        for i, p in enumerate(self.params):
            p.data = self.param_view(i)
            if self.grad_dtype != param_dtype and hasattr(p, "grad_dtype"):
                p.grad_dtype = None  # fp32 gradients of bf16 compute copies (FSDP reduce_dtype=fp32)
            p.grad = self.grad_view(i)
            p._dta_flat = (self, i)  # noqa: SLF001 - tag read by the fused optimizers

    # -------------------------------------------------------------- views
    def _view(self, buf: torch.Tensor, i: int) -> torch.Tensor:
        o, n = self.offsets[i], self.numels[i]
        return buf[o:o + n].view(self.shapes[i])

    def param_view(self, i: int) -> torch.Tensor:
        return self._view(self.compute, i)

    def master_view(self, i: int) -> torch.Tensor:
        return self._view(self.master, i)

    def grad_view(self, i: int) -> torch.Tensor:
        return self._view(self.grad, i)

    def index_of(self, p: torch.nn.Parameter) -> int:
        tag = getattr(p, "_dta_flat", None)
        if tag is None or tag[0] is not self:
            raise KeyError("parameter does not belong to this flat group")
        return tag[1]

    # ------------------------------------------------------------ helpers
    def rebind_grad(self, i: int) -> None:
        """Make ``params[i].grad`` the flat view again (after a torch optimizer
        set it to None or autograd stole a fresh tensor)."""
        p = self.params[i]
        view = self.grad_view(i)
        g = p.grad
        if g is None:
            view.zero_()
        elif g.data_ptr() != view.data_ptr():
            view.copy_(g)
        p.grad = view

    def grad_is_view(self, i: int) -> bool:
        g = self.params[i].grad
        return g is not None and g.data_ptr() == self.grad_view(i).data_ptr()

    def zero_grad(self, set_to_none: bool = False) -> None:
        """``set_to_none``: drop the gradients (autograd then hands fresh
        tensors over without an accumulate kernel; the DDP engine moves them
        into the flat buffer in one batched copy per bucket).  Otherwise zero
        the flat buffer and keep the views."""
        if set_to_none and (self.steal_ok or self.fresh_hook is not None):
            self.direct_claimed.clear()
            for p in self.params:
                p.grad = None
            if self.fresh_hook is not None:
                self.fresh_hook()
            return
        self.grad.zero_()
        for i, p in enumerate(self.params):
            if p.grad is None or p.grad.data_ptr() != self.grad_view(i).data_ptr():
                p.grad = self.grad_view(i)

    def prepare_grads_for_step(self) -> bool:
        """Before a flat optimizer step: make every gradient its flat view
        (normally already true after a DDP backward).  Returns False when no
        parameter has a gradient (torch optimizers skip such parameters)."""
        if all(self.grad_is_view(i) for i in range(len(self.params))):
            return True
        if all(p.grad is None for p in self.params):
            return False
        for i in range(len(self.params)):
            self.rebind_grad(i)
        return True

    def sync_compute_from_master(self) -> None:
        if self.mixed:
            from ..ops.optim import cast_into

            cast_into(self.master, self.compute)

    def sync_master_from_compute(self) -> None:
        if self.mixed:
            self.master.copy_(self.compute.float())

    def buckets_from_plan(self, plan: Sequence[Sequence[int]]) -> List[Bucket]:
        """Buckets of :func:`plan_buckets` (each ends at its last parameter's padded end)."""
        out = []
        for ids in plan:
            last = ids[-1]
            end = _align(self.offsets[last] + self.numels[last], self.pad_after.get(last, ALIGN_ELEMS))
            out.append(Bucket(len(out), self.offsets[ids[0]], end, list(ids)))
        return out

    def make_buckets(self, order: Sequence[int], cap_bytes: int, first_cap_bytes: int) -> List[Bucket]:
        """Contiguous buckets over the flat buffer (params are laid out in
        ``order``, which callers choose as reverse registration order so the
        first bucket fills first during backward)."""
        esize = torch.empty((), dtype=self.grad_dtype).element_size()
        buckets: List[Bucket] = []
        cur: List[int] = []
        start = None
        cap = first_cap_bytes
        for i in order:
            o, n = self.offsets[i], self.numels[i]
            if start is None:
                start = o
            cur.append(i)
            end = _align(o + n)
            if (end - start) * esize >= cap:
                buckets.append(Bucket(len(buckets), start, end, cur))
                cur, start, cap = [], None, cap_bytes
        if cur:
            end = _align(self.offsets[cur[-1]] + self.numels[cur[-1]])
            buckets.append(Bucket(len(buckets), start, end, cur))
        return buckets


@torch.no_grad()
def clip_flat_grad_norm_(fg: FlatParamGroup, max_norm: float, comm: Any = None, sharded: bool = False) -> torch.Tensor:
    """Global-norm gradient clipping over ONE flat gradient buffer (what
    ``torch.nn.utils.clip_grad_norm_`` computes over the module's parameters).

    ``sharded``: the buffer holds this rank's shard only (FSDP), so the squared
    norm is all-reduced (sum) over ``comm`` before the coefficient is formed --
    every rank then scales its shard by the SAME coefficient.  Replicated
    buffers (DDP after the all-reduce) need no collective.  No host sync: the
    coefficient stays on the device.  Padding between parameters is zero and
    does not change the norm.  Returns the total norm (0-dim tensor)."""
    if not fg.prepare_grads_for_step():
        return torch.zeros((), device=fg.grad.device)
    g = fg.grad
    if g.is_cuda and g.dtype == torch.float32:
        from ..ops import native

        sq = torch.zeros(1, dtype=torch.float32, device=g.device)
        native().flat_sumsq(g, sq, -1)
    else:
        sq = g.float().pow(2).sum().reshape(1)
    if sharded and comm is not None and comm.world_size > 1:
        dev = getattr(comm, "device", None)
        if dev is not None and sq.device != torch.device(dev):  # host-resident shards, device communicator
            sq_d = sq.to(dev)
            comm.all_reduce(sq_d, op="sum")
            sq = sq_d.to(sq.device)
        else:
            comm.all_reduce(sq, op="sum")
    norm = sq.sqrt()
    coef = (float(max_norm) / (norm + 1e-6)).clamp(max=1.0)
    g.mul_(coef.to(g.dtype))
    return norm.reshape(())


def plan_buckets(numels: Sequence[int], esize: int, cap_bytes: int, first_cap_bytes: int) -> List[List[int]]:
    """Bucket membership over parameters in layout order: the first bucket closes
    at ``first_cap_bytes``, later ones at ``cap_bytes`` (torch Reducer rule)."""
    plan: List[List[int]] = []
    cur: List[int] = []
    size, cap = 0, first_cap_bytes
    for i, n in enumerate(numels):
        cur.append(i)
        size += _align(n) * esize
        if size >= cap:
            plan.append(cur)
            cur, size, cap = [], 0, cap_bytes
    if cur:
        plan.append(cur)
    return plan


# xGMI model for DDP bucket sizing: one MI355X has 7 point-to-point
# links of ~153 GB/s; RCCL's multi-channel ring all-reduce reaches a bus bandwidth
# of roughly 2 links' worth, and each collective costs a fixed ~20 us (launch +
# protocol latency).  A ring all-reduce of S bytes over N ranks moves 2 (N-1)/N S.
XGMI_BUS_BW = 300e9
XGMI_COLL_LATENCY = 20e-6


def xgmi_bucket_caps(world_size: int, grad_bytes: int, min_buckets: int = 6) -> Tuple[int, int]:
    """(first_cap_bytes, cap_bytes) for DDP buckets on one xGMI node:
    * a steady bucket large enough that the fixed latency is <= 10 % of its
      transfer time: S >= 10 * latency * bus_bw / (2 (N-1) / N);
    * but at least ``min_buckets`` buckets per backward so the all-reduces
      overlap the remaining backward; clamped to [4, 64] MiB;
    * a first bucket of cap / 16 (>= 1 MiB) so the first collective starts after
      the last layer's gradients, early in backward."""
    MiB = 1 << 20
    n = max(2, world_size)
    s_lat = 10 * XGMI_COLL_LATENCY * XGMI_BUS_BW / (2.0 * (n - 1) / n)
    cap = min(s_lat, grad_bytes / max(1, min_buckets))
    cap = int(min(64 * MiB, max(4 * MiB, cap)))
    first = max(1 * MiB, cap // 16)
    return first, cap


def fit_alpha_beta(points: Sequence[Tuple[float, float]]) -> Optional[Tuple[float, float]]:
    """Least-squares fit of ``t = alpha + S / beta`` over measured ``(S bytes, t seconds)`` points:
    ``(alpha seconds, beta bytes/s of message size)``, or None when the points do not give a positive
    slope (noise, too few sizes).  ``alpha`` is clamped at >= 0."""
    pts = [(float(s), float(t)) for s, t in points if s > 0 and t > 0 and math.isfinite(t)]
    if len({s for s, _ in pts}) < 2:
        return None
    n = len(pts)
    ms = sum(s for s, _ in pts) / n
    mt = sum(t for _, t in pts) / n
    var = sum((s - ms) ** 2 for s, _ in pts)
    slope = sum((s - ms) * (t - mt) for s, t in pts) / var
    if slope <= 0:
        return None
    alpha = max(0.0, mt - slope * ms)
    return alpha, 1.0 / slope


def measured_bucket_caps(grad_bytes: int, alpha: float, beta: float, min_buckets: int = 6) -> Tuple[int, int]:
    """(first_cap_bytes, cap_bytes) from a MEASURED all-reduce cost ``t(S) = alpha + S / beta`` (the
    α/β fit of the routed communicator's wrap-time calibration, :meth:`.routed.RoutedComm.alpha_beta`):
    the same rule as :func:`xgmi_bucket_caps` -- a steady bucket whose fixed cost is <= 10 % of its
    transfer time (``S >= 10 alpha beta``), but >= ``min_buckets`` buckets per backward for overlap,
    clamped to [4, 64] MiB; a first bucket of cap / 16 (>= 1 MiB)."""
    MiB = 1 << 20
    cap = min(10.0 * alpha * beta, grad_bytes / max(1, min_buckets))
    cap = int(min(64 * MiB, max(4 * MiB, cap)))
    first = max(1 * MiB, cap // 16)
    return first, cap


def bucket_caps_for(comm: Any, world_size: int, grad_bytes: int, dtype: Any) -> Tuple[int, int, str]:
    """DDP's ``bucket_cap_mb="auto"``: measured caps when the communicator timed its all-reduce at wrap
    (``alpha_beta``), else the assumed xGMI constants (the no-calibration fallback).  Returns
    ``(first_cap_bytes, cap_bytes, source)``."""
    ab = None
    fn = getattr(comm, "alpha_beta", None) if world_size > 1 else None
    if fn is not None:
        try:
            ab = fn("all_reduce", dtype)
        except Exception:  # noqa: BLE001 - a communicator without usable timings: the model
            ab = None
    if ab is not None:
        first, cap = measured_bucket_caps(grad_bytes, *ab)
        return first, cap, f"measured: alpha {ab[0] * 1e6:.1f} us, beta {ab[1] / 1e9:.1f} GB/s"
    first, cap = xgmi_bucket_caps(world_size, grad_bytes)
    return first, cap, "xgmi model (assumed constants)"


def build_flat_group(params_with_names: Sequence[Tuple[str, torch.nn.Parameter]], device: torch.device,
                     param_dtype: Any = torch.float32, grad_dtype: Any = None, reverse: bool = True,
                     pad_after: Optional[Dict[int, int]] = None) -> FlatParamGroup:
    items = list(params_with_names)
    if reverse:
        items = items[::-1]
    names = [n for n, _ in items]
    params = [p for _, p in items]
    return FlatParamGroup(params, device, param_dtype=param_dtype, grad_dtype=grad_dtype, names=names,
                          pad_after=pad_after)


def param_flat_tags(params: Any) -> Dict[int, Tuple[FlatParamGroup, int]]:
    out = {}
    for p in params:
        tag = getattr(p, "_dta_flat", None)
        if tag is not None:
            out[id(p)] = tag
    return out
