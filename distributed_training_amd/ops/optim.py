"""Fused optimizers (drop-in ``torch.optim.SGD`` / ``AdamW`` / ``Adam``).

GPU parameters are updated by the hand-written HIP kernels of
``csrc/optim.hip``.  When the parameters belong to a :class:`FlatParamGroup`
(DDP/FSDP engines) the whole group is updated by ONE launch over the flat
buffer, including the fp32-master -> bf16 compute copy under mixed precision.
CPU parameters (gloo plumbing path) use the same math in plain PyTorch.

Semantics follow torch.optim exactly (tested against it), so the reference's
``torch.optim.SGD(model.parameters(), lr=cfg.train.learning_rate)``
(src/distributed_trainer.py:200) maps 1:1 onto :class:`FusedSGD`.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import torch

from . import native


def cast_into(src: torch.Tensor, dst: torch.Tensor) -> None:
    if src.is_cuda and src.dtype == torch.float32 and dst.dtype == torch.bfloat16:
        native().cast_f32_bf16(src, dst, -1)
    else:
        dst.copy_(src)


def _grad32(fg_grad: torch.Tensor) -> torch.Tensor:
    return fg_grad if fg_grad.dtype == torch.float32 else fg_grad.float()


def _split_params(group_params: Any) -> Any:
    flats: Dict[int, list] = {}
    flat_objs = {}
    singles = []
    for p in group_params:
        tag = getattr(p, "_dta_flat", None)
        if tag is not None and p.is_cuda:
            fg = tag[0]
            flats.setdefault(id(fg), []).append(p)
            flat_objs[id(fg)] = fg
        else:
            singles.append(p)
    return [(flat_objs[k], v) for k, v in flats.items()], singles


def _cpu_target(p: torch.Tensor) -> Any:
    """The tensor a CPU-side update must write for parameter ``p``: under bf16 mixed precision a
    DDP / FSDP flat-group parameter is the bf16 COMPUTE view, and the update belongs in its fp32
    master (which checkpoints save), then copied back -- updating the compute view alone left the
    master, and every snapshot of a CPU mixed-precision run, at the initial weights."""
    tag = getattr(p, "_dta_flat", None)
    if tag is not None and getattr(tag[0], "mixed", False):
        return tag[0].master_view(tag[1]), True
    return p, False


def _sgd_ref(p: torch.Tensor, g: torch.Tensor, buf: Optional[torch.Tensor], lr: float, momentum: float,
             dampening: float, wd: float, nesterov: bool, maximize: bool, first: bool) -> None:
    d = -g if maximize else g
    if wd:
        d = d.add(p, alpha=wd)
    if momentum:
        if first:
            buf.copy_(d)
        else:
            buf.mul_(momentum).add_(d, alpha=1 - dampening)
        d = d.add(buf, alpha=momentum) if nesterov else buf
    p.add_(d, alpha=-lr)


def _saved_state_by_param(opt: torch.optim.Optimizer, state_dict: dict) -> Dict[torch.nn.Parameter, dict]:
    """Map a ``torch.optim.Optimizer.state_dict()`` onto this optimizer's parameters
    (same param-group structure), restoring the groups' hyper-parameters.  Unlike
    torch's ``load_state_dict`` nothing is cast to the parameter dtype: under bf16
    mixed precision the parameters are bf16 compute copies while the optimizer
    state is fp32 and lives in flat buffers beside the fp32 master."""
    saved_groups = state_dict["param_groups"]
    if len(saved_groups) != len(opt.param_groups) or any(
            len(g["params"]) != len(sg["params"]) for g, sg in zip(opt.param_groups, saved_groups)):
        raise ValueError("optimizer state dict does not match the optimizer's parameter groups")
    saved = state_dict["state"]
    out: Dict[torch.nn.Parameter, dict] = {}
    for g, sg in zip(opt.param_groups, saved_groups):
        for k, v in sg.items():
            if k != "params":
                g[k] = v
        for p, pid in zip(g["params"], sg["params"]):
            st = saved.get(pid, saved.get(str(pid)))
            if st:
                out[p] = st
    return out


def _restore_flat(fg: Any, by_param: Dict[torch.nn.Parameter, dict], key: str) -> Optional[torch.Tensor]:
    """A fresh flat fp32 buffer (the layout of ``fg.master``) filled with each
    parameter's saved ``key`` tensor; None when no parameter has one."""
    if not any(key in by_param.get(p, {}) for p in fg.params):
        return None
    flat = torch.zeros_like(fg.master)
    for i, p in enumerate(fg.params):
        v = by_param.get(p, {}).get(key)
        if v is not None:
            fg._view(flat, i).copy_(v.reshape(fg.shapes[i]).to(flat.device, torch.float32))
    return flat


def _stepped_in_backward(fg: Any) -> bool:
    """True (once) when the DDP engine already ran this step bucket by bucket inside the
    backward (parallel/ddp.py ``overlap_optimizer``): ``step()`` then has nothing to do."""
    if getattr(fg, "stepped_in_backward", False):
        fg.stepped_in_backward = False
        return True
    return False


def _covers(params: Any, fg: Any) -> bool:
    ids = {id(p) for p in params}
    return len(ids) == len(fg.params) and all(id(p) in ids for p in fg.params)


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, params: Any, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, maximize: bool = False) -> None:
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, maximize=maximize)
        super().__init__(params, defaults)
        self._flat_state: Dict[int, dict] = {}

    def hyper(self, group: Any = None) -> dict:
        g = group or self.param_groups[0]
        return {k: g[k] for k in ("lr", "momentum", "dampening", "weight_decay", "nesterov", "maximize")}

    @torch.no_grad()
    def step(self, closure: Any = None) -> Any:
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, mom, damp, wd = group["lr"], group["momentum"], group["dampening"], group["weight_decay"]
            nest, maxi = group["nesterov"], group["maximize"]
            flats, singles = _split_params(group["params"])
            for fg, ps in flats:
                if _stepped_in_backward(fg):
                    continue
                if len(ps) == len(fg.params):
                    if not fg.prepare_grads_for_step():
                        continue
                    st = self._flat_state.setdefault(id(fg), {"first": True})
                    if mom and "mom" not in st:
                        st["mom"] = torch.zeros_like(fg.master)
                        for i, p in enumerate(fg.params):
                            self.state[p]["momentum_buffer"] = fg._view(st["mom"], i)
                    pb = fg.compute if fg.mixed else None
                    native().flat_sgd(fg.master, fg.master, _grad32(fg.grad), st.get("mom"), pb, lr, mom, damp, wd,
                                      1.0, nest, maxi, st["first"], -1)
                    st["first"] = False
                else:
                    fg.prepare_grads_for_step()
                    for p in ps:
                        self._single_gpu(fg, p, lr, mom, damp, wd, nest, maxi)
            for p in singles:
                if p.grad is None:
                    continue
                state = self.state[p]
                first = "momentum_buffer" not in state or state["momentum_buffer"] is None
                if mom and first:
                    state["momentum_buffer"] = torch.zeros_like(p, dtype=torch.float32)
                buf = state.get("momentum_buffer") if mom else None
                if p.is_cuda:
                    if p.dtype != torch.float32:
                        raise TypeError("FusedSGD on GPU needs fp32 parameters (or a FlatParamGroup with a master)")
                    native().flat_sgd(p.view(-1), p.view(-1), p.grad.float().contiguous().view(-1),
                                      None if buf is None else buf.view(-1), None, lr, mom, damp, wd, 1.0, nest,
                                      maxi, first, -1)
                else:
                    tgt, sync = _cpu_target(p)
                    _sgd_ref(tgt, p.grad.to(tgt.dtype), buf, lr, mom, damp, wd, nest, maxi, first)
                    if sync:
                        p.copy_(tgt)
        return loss

    # -------------------------------------------------- step split over DDP buckets
    def range_capable(self, fg: Any) -> bool:
        return len(self.param_groups) == 1 and _covers(self.param_groups[0]["params"], fg)

    @torch.no_grad()
    def step_range(self, fg: Any, lo: int, hi: int, first: bool, max_blocks: int = 0) -> None:
        """Update elements ``[lo, hi)`` of the flat group ``fg`` (one DDP bucket, on the
        current stream): the same per-element math as :meth:`step` over the whole buffer,
        so a step split into ranges is bit-identical.  ``first``: the step's first range
        (``max_blocks``: accepted for the interface, the SGD update keeps its grid)."""
        g = self.param_groups[0]
        st = self._flat_state.setdefault(id(fg), {"first": True})
        if g["momentum"] and "mom" not in st:
            st["mom"] = torch.zeros_like(fg.master)
            for i, p in enumerate(fg.params):
                self.state[p]["momentum_buffer"] = fg._view(st["mom"], i)
        mom = st.get("mom")
        native().flat_sgd(fg.master[lo:hi], fg.master[lo:hi], _grad32(fg.grad[lo:hi]),
                          None if mom is None else mom[lo:hi], fg.compute[lo:hi] if fg.mixed else None,
                          g["lr"], g["momentum"], g["dampening"], g["weight_decay"], 1.0, g["nesterov"],
                          g["maximize"], st["first"], -1)

    def end_ranges(self, fg: Any) -> None:
        """Every range of this step launched."""
        self._flat_state.setdefault(id(fg), {"first": True})["first"] = False

    @torch.no_grad()
    def load_state_dict(self, state_dict: dict) -> None:
        """Resume: momentum buffers go back into the flat fp32 state (resumable after a
        checkpoint written by ``state_dict()``)."""
        by_param = _saved_state_by_param(self, state_dict)
        for group in self.param_groups:
            flats, singles = _split_params(group["params"])
            for fg, ps in flats:
                flat = _restore_flat(fg, by_param, "momentum_buffer")
                if flat is None:
                    continue
                if len(ps) == len(fg.params):
                    self._flat_state[id(fg)] = {"first": False, "mom": flat}
                    for i, p in enumerate(fg.params):
                        self.state[p]["momentum_buffer"] = fg._view(flat, i)
                else:
                    for p in ps:
                        i = fg.index_of(p)
                        self.state[p]["momentum_buffer"] = fg._view(flat, i).reshape(-1).clone()
            for p in singles:
                v = by_param.get(p, {}).get("momentum_buffer")
                if v is not None:
                    self.state[p]["momentum_buffer"] = v.to(p.device, torch.float32).reshape(p.shape).clone()

    def _single_gpu(self, fg: Any, p: Any, lr: float, mom: float, damp: float, wd: float, nest: bool,
                    maxi: bool) -> None:
        i = fg.index_of(p)
        state = self.state[p]
        first = "momentum_buffer" not in state or state["momentum_buffer"] is None
        if mom and first:
            state["momentum_buffer"] = torch.zeros(fg.numels[i], device=p.device)
        buf = state.get("momentum_buffer") if mom else None
        m = fg.master_view(i).view(-1)
        g = fg.grad_view(i).view(-1).float()
        pb = fg.param_view(i).view(-1) if fg.mixed else None
        native().flat_sgd(m, m, g, None if buf is None else buf.view(-1), pb, lr, mom, damp, wd, 1.0, nest, maxi,
                          first, -1)

    def zero_grad(self, set_to_none: bool = True) -> None:
        flats_done = set()
        for group in self.param_groups:
            flats, singles = _split_params(group["params"])
            for fg, _ in flats:
                if id(fg) not in flats_done:
                    fg.zero_grad(set_to_none)  # views kept unless the engine moves fresh grads in

                    flats_done.add(id(fg))
            for p in singles:
                tag = getattr(p, "_dta_flat", None)
                if tag is not None:
                    tag[0].zero_grad(set_to_none)
                elif p.grad is not None:
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.zero_()


def _adam_ref(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, vmax: torch.Tensor, step: int,
              lr: float, b1: float, b2: float, eps: float, wd: float, adamw: bool, maximize: bool,
              amsgrad: bool) -> None:
    g = -g if maximize else g
    if wd:
        if adamw:
            p.mul_(1 - lr * wd)
        else:
            g = g.add(p, alpha=wd)
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    vv = v
    if amsgrad:
        torch.maximum(vmax, v, out=vmax)
        vv = vmax
    denom = (vv.sqrt() / (bc2 ** 0.5)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


class FusedAdamW(torch.optim.Optimizer):
    """AdamW (``adamw=True``, default) or Adam with L2 (``adamw=False``)."""

    def __init__(self, params: Any, lr: float = 1e-3, betas: Any = (0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, amsgrad: bool = False, maximize: bool = False, adamw: bool = True) -> None:
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                        maximize=maximize, adamw=adamw)
        super().__init__(params, defaults)
        self._flat_state: Dict[int, dict] = {}

    @torch.no_grad()
    def step(self, closure: Any = None) -> Any:
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            ams, maxi, adamw = group["amsgrad"], group["maximize"], group["adamw"]
            flats, singles = _split_params(group["params"])
            for fg, ps in flats:
                if len(ps) != len(fg.params):
                    raise ValueError("FusedAdamW: a FlatParamGroup must be optimised as a whole by one param group")
                if _stepped_in_backward(fg):
                    continue
                if not fg.prepare_grads_for_step():
                    continue
                st = self._flat(fg, ams)
                pb = fg.compute if fg.mixed else None
                native().flat_adam(fg.master, fg.grad, st["m"], st["v"], st["vmax"], pb, st["step"], lr, b1,
                                   b2, eps, wd, 1.0, adamw, maxi, ams, True, -1)
            for p in singles:
                if p.grad is None:
                    continue
                state = self.state[p]
                if not state:
                    state["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                    state["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                    state["step"] = torch.zeros(1, device=p.device) if p.is_cuda else torch.zeros(())
                    if ams:
                        state["max_exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                if p.is_cuda:
                    if p.dtype != torch.float32:
                        raise TypeError("FusedAdamW on GPU needs fp32 parameters (or a FlatParamGroup with a master)")
                    native().flat_adam(p.view(-1), p.grad.float().contiguous().view(-1), state["exp_avg"].view(-1),
                                       state["exp_avg_sq"].view(-1),
                                       state["max_exp_avg_sq"].view(-1) if ams else None, None, state["step"], lr,
                                       b1, b2, eps, wd, 1.0, adamw, maxi, ams, True, -1)
                else:
                    state["step"] += 1
                    tgt, sync = _cpu_target(p)
                    _adam_ref(tgt, p.grad.to(tgt.dtype), state["exp_avg"], state["exp_avg_sq"],
                              state.get("max_exp_avg_sq"), float(state["step"]), lr, b1, b2, eps, wd, adamw, maxi, ams)
                    if sync:
                        p.copy_(tgt)
        return loss

    zero_grad = FusedSGD.zero_grad

    def _flat(self, fg: Any, ams: bool) -> dict:
        st = self._flat_state.get(id(fg))
        if st is None:
            st = {"m": torch.zeros_like(fg.master), "v": torch.zeros_like(fg.master),
                  "vmax": torch.zeros_like(fg.master) if ams else None,
                  "step": torch.zeros(1, device=fg.master.device)}
            self._flat_state[id(fg)] = st
            for i, p in enumerate(fg.params):
                self.state[p]["exp_avg"] = fg._view(st["m"], i)
                self.state[p]["exp_avg_sq"] = fg._view(st["v"], i)
                self.state[p]["step"] = st["step"]
                if ams:
                    self.state[p]["max_exp_avg_sq"] = fg._view(st["vmax"], i)
        return st

    # -------------------------------------------------- step split over DDP buckets
    range_capable = FusedSGD.range_capable

    @torch.no_grad()
    def step_range(self, fg: Any, lo: int, hi: int, first: bool, max_blocks: int = 0) -> None:
        """Update elements ``[lo, hi)`` of the flat group ``fg`` (one DDP bucket / FSDP unit, on
        the current stream); ``first`` bumps the device step counter (the step's first range);
        ``max_blocks`` > 0 caps the grid (an update running beside the backward's kernels).
        Element-wise math identical to :meth:`step`: a split step is bit-identical."""
        g = self.param_groups[0]
        (b1, b2), ams = g["betas"], g["amsgrad"]
        st = self._flat(fg, ams)
        native().flat_adam(fg.master[lo:hi], fg.grad[lo:hi], st["m"][lo:hi], st["v"][lo:hi],
                           None if st["vmax"] is None else st["vmax"][lo:hi],
                           fg.compute[lo:hi] if fg.mixed else None, st["step"], g["lr"], b1, b2, g["eps"],
                           g["weight_decay"], 1.0, g["adamw"], g["maximize"], ams, first, -1, max_blocks)

    def end_ranges(self, fg: Any) -> None:
        pass

    @torch.no_grad()
    def load_state_dict(self, state_dict: dict) -> None:
        """Resume: first / second moments and the step count go back into the flat fp32
        state (the fused step keeps them there, not in per-parameter tensors)."""
        by_param = _saved_state_by_param(self, state_dict)
        for group in self.param_groups:
            flats, singles = _split_params(group["params"])
            for fg, _ps in flats:
                m = _restore_flat(fg, by_param, "exp_avg")
                if m is None:
                    continue
                v = _restore_flat(fg, by_param, "exp_avg_sq")
                vmax = _restore_flat(fg, by_param, "max_exp_avg_sq") if group["amsgrad"] else None
                if group["amsgrad"] and vmax is None:
                    vmax = torch.zeros_like(fg.master)
                steps = [by_param[p]["step"] for p in fg.params if p in by_param and "step" in by_param[p]]
                step = torch.zeros(1, device=fg.master.device)
                if steps:
                    step.fill_(float(torch.as_tensor(steps[0]).reshape(-1)[0]))
                st = {"m": m, "v": v if v is not None else torch.zeros_like(fg.master), "vmax": vmax, "step": step}
                self._flat_state[id(fg)] = st
                for i, p in enumerate(fg.params):
                    self.state[p]["exp_avg"] = fg._view(st["m"], i)
                    self.state[p]["exp_avg_sq"] = fg._view(st["v"], i)
                    self.state[p]["step"] = st["step"]
                    if vmax is not None:
                        self.state[p]["max_exp_avg_sq"] = fg._view(vmax, i)
            for p in singles:
                sv = by_param.get(p)
                if not sv:
                    continue
                st = self.state[p]
                for k in ("exp_avg", "exp_avg_sq", "max_exp_avg_sq"):
                    if k in sv:
                        st[k] = sv[k].to(p.device, torch.float32).reshape(p.shape).clone()
                if "step" in sv:
                    st["step"] = (torch.zeros(1, device=p.device) if p.is_cuda else torch.zeros(())).fill_(
                        float(torch.as_tensor(sv["step"]).reshape(-1)[0]))


def build_optimizer(name: str, params: Any, **kw: Any) -> torch.optim.Optimizer:
    name = name.lower()
    if name == "sgd":
        return FusedSGD(params, **kw)
    if name == "adamw":
        return FusedAdamW(params, adamw=True, **kw)
    if name == "adam":
        return FusedAdamW(params, adamw=False, **{"weight_decay": 0.0, **kw})
    raise ValueError(f"unknown optimizer {name!r}")


def optimizer_hparams(opt: torch.optim.Optimizer) -> Dict[str, object]:
    """Hyper-parameters of param group 0 (works for torch and fused optimizers)."""
    g = opt.param_groups[0]
    return {k: v for k, v in g.items() if k != "params"}


def same_kind_optimizer(opt: torch.optim.Optimizer, params: List[torch.nn.Parameter]) -> torch.optim.Optimizer:
    """Rebuild ``opt`` (same class / hyper-parameters) over ``params``."""
    hp = optimizer_hparams(opt)
    cls = type(opt)
    if cls is torch.optim.SGD:
        keep = {k: hp[k] for k in ("lr", "momentum", "dampening", "weight_decay", "nesterov", "maximize") if k in hp}
        return FusedSGD(params, **keep)
    if cls in (torch.optim.AdamW, torch.optim.Adam):
        keep = {k: hp[k] for k in ("lr", "betas", "eps", "weight_decay", "amsgrad", "maximize") if k in hp}
        return FusedAdamW(params, adamw=cls is torch.optim.AdamW, **keep)
    if cls is FusedSGD:
        keep = {k: hp[k] for k in ("lr", "momentum", "dampening", "weight_decay", "nesterov", "maximize")}
        return FusedSGD(params, **keep)
    if cls is FusedAdamW:
        keep = {k: hp[k] for k in ("lr", "betas", "eps", "weight_decay", "amsgrad", "maximize", "adamw")}
        return FusedAdamW(params, **keep)
    return cls(params, **hp)
