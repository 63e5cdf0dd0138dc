"""Thin Python wrapper of the fused 2-layer-MLP train-step kernel
(``csrc/mlp_fused.hip``) plus its fp32 PyTorch reference.

Flat parameter layout (fp32, each region 64-byte aligned)::

    [ W1 (hidden x in) | b1 (hidden) | W2 (out x hidden) | b2 (out) ]

Names match ``nn.Linear`` state-dict order of the MLP model
(``models/mlp.py``: ``fc1.weight, fc1.bias, fc2.weight, fc2.bias``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from . import native

ACTIVATIONS = {"none": 0, "identity": 0, "relu": 1, "gelu": 2, "gelu_tanh": 2, "silu": 3}
LOSSES = {"mse": 0, "cross_entropy": 1}
ALIGN = 16  # floats (64 bytes)

LDS_LIMIT = 160 * 1024


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass(frozen=True)
class MlpLayout:
    in_dim: int
    hidden: int
    out_dim: int
    o_w1: int
    o_b1: int
    o_w2: int
    o_b2: int
    total: int

    @property
    def offsets(self) -> Any:
        return [self.o_w1, self.o_b1, self.o_w2, self.o_b2]

    def views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        H, I, O = self.hidden, self.in_dim, self.out_dim
        return {
            "fc1.weight": flat[self.o_w1:self.o_w1 + H * I].view(H, I),
            "fc1.bias": flat[self.o_b1:self.o_b1 + H],
            "fc2.weight": flat[self.o_w2:self.o_w2 + O * H].view(O, H),
            "fc2.bias": flat[self.o_b2:self.o_b2 + O],
        }


def make_layout(in_dim: int, hidden: int, out_dim: int) -> MlpLayout:
    o_w1 = 0
    o_b1 = _align(o_w1 + hidden * in_dim)
    o_w2 = _align(o_b1 + hidden)
    # LDS banks: in the persistent loop's SGD one instruction updates b1[h] (one
    # lane) and W2[h] (another): keep the two 4 banks apart, not on one bank
    if (o_w2 - o_b1) % 32 == 0:
        o_w2 += 4
    o_b2 = _align(o_w2 + out_dim * hidden)
    total = _align(o_b2 + out_dim)
    return MlpLayout(in_dim, hidden, out_dim, o_w1, o_b1, o_w2, o_b2, total)


def lds_bytes(in_dim: int, hidden: int, out_dim: int, batch: int, momentum: bool = False) -> int:
    """LDS footprint: fp32 image of the flat params (+ momentum image) + bf16 X
    tiles + wave-private transpose / dY tiles (host mirror of the kernel's)."""
    rt = (batch + 31) // 32
    bpad = 32 if rt <= 1 else (64 if rt <= 2 else 128)
    total = make_layout(in_dim, hidden, out_dim).total
    return (total * 4 * (2 if momentum else 1) + bpad * 80 + 32 * (bpad + 8) * 2 + 8 * 2 * 32 * 40 * 2
            + 2 * bpad * 32 + 8 * bpad * 32)


def supported(in_dim: int, hidden: int, out_dim: int, batch: int, momentum: bool = False) -> bool:
    """Shapes covered by the fused kernel (host mirror of the kernel's limits)."""
    return (
        1 <= in_dim <= 31
        and 1 <= out_dim <= 8
        and hidden >= 32
        and hidden % 32 == 0
        and 1 <= batch <= 128
        and lds_bytes(in_dim, hidden, out_dim, batch, momentum) <= LDS_LIMIT
    )


def persistent_supported(in_dim: int, hidden: int, out_dim: int, batch: int, momentum: bool = False,
                         world: int = 1) -> bool:
    """Shapes served by the persistent single-workgroup loop (csrc/mlp_persistent.hip);
    SGD momenta take LDS only with several ranks (one rank keeps them in registers)."""
    if not (1 <= in_dim and in_dim + 1 + out_dim <= 32 and out_dim == 1 and hidden % 32 == 0
            and 32 <= hidden <= 512 and 1 <= batch <= 32):
        return False
    total = make_layout(in_dim, hidden, out_dim).total
    return native().mlp_persistent_lds_bytes(total, hidden, out_dim, int(momentum and world > 1)) <= LDS_LIMIT


def pad_features(X: torch.Tensor) -> torch.Tensor:
    """[N, in] -> bf16 [N, 32] = (X | 1 | 0): the persistent kernel's row format
    (the ones column carries the bias gradient)."""
    N, I = X.shape
    Xp = torch.zeros(N, 32, dtype=torch.bfloat16, device=X.device)
    Xp[:, :I] = X.to(torch.bfloat16)
    Xp[:, I] = 1.0
    return Xp


def persistent_steps(Xp: torch.Tensor, T: torch.Tensor, idx_ring: torch.Tensor, cursor: torch.Tensor,
                     loss_ring: torch.Tensor, loss_cursor: torch.Tensor, mom_started: torch.Tensor, P: torch.Tensor,
                     M: torch.Tensor, layout: MlpLayout,
                     batch: int, nsteps: int, act: str, loss: str, grad_scale: float, sgd: Dict[str, float],
                     stream: Any = None, dbg: Any = None, dbg_step: int = 0, xinfo: Any = None) -> None:
    """``nsteps`` complete training steps (gather, forward, loss, backward, SGD) in ONE launch.
    ``xinfo`` (from :func:`exchange_info`): DDP gradient exchange across ranks inside the loop."""
    native().mlp_persistent(
        Xp, T, idx_ring, cursor, loss_ring, loss_cursor, mom_started, P, M, layout.offsets, layout.total,
        layout.in_dim, layout.hidden, layout.out_dim, int(batch), int(nsteps), ACTIVATIONS[act], LOSSES[loss],
        float(grad_scale), float(sgd.get("lr", 1e-3)), float(sgd.get("momentum", 0.0)),
        float(sgd.get("dampening", 0.0)), float(sgd.get("weight_decay", 0.0)), bool(sgd.get("nesterov", False)),
        bool(sgd.get("maximize", False)), -1 if stream is None else int(stream.cuda_stream), dbg, int(dbg_step),
        list(xinfo) if xinfo else [])


def persistent_prepare(Xp: torch.Tensor, T: torch.Tensor, idx_ring: torch.Tensor, cursor: torch.Tensor,
                       loss_ring: torch.Tensor, loss_cursor: torch.Tensor, mom_started: torch.Tensor, P: torch.Tensor,
                       M: torch.Tensor, layout: MlpLayout, batch: int, act: str, loss: str, grad_scale: float,
                       sgd: Dict[str, float], xinfo: Any = None) -> Any:
    """:func:`persistent_steps` with its arguments checked and packed once: returns a
    native object whose ``launch(nsteps, stream=-1)`` enqueues the loop (host cost of
    one kernel launch)."""
    return native().mlp_persistent_prepare(
        Xp, T, idx_ring, cursor, loss_ring, loss_cursor, mom_started, P, M, layout.offsets, layout.total,
        layout.in_dim, layout.hidden, layout.out_dim, int(batch), ACTIVATIONS[act], LOSSES[loss],
        float(grad_scale), float(sgd.get("lr", 1e-3)), float(sgd.get("momentum", 0.0)),
        float(sgd.get("dampening", 0.0)), float(sgd.get("weight_decay", 0.0)), bool(sgd.get("nesterov", False)),
        bool(sgd.get("maximize", False)), list(xinfo) if xinfo else [])


XMODES = {"oneshot": 1, "rsag": 2, "helpers": 3}


def helper_elems(hidden: int, out_dim: int) -> int:
    """Exchange array of the helper form: fragment order [hidden/32 tiles][16][64] + the b2 gradients."""
    return (hidden // 32) * 1024 + 64 * (-(-out_dim // 64))


def exchange_info(p2p: Any, xepoch: torch.Tensor, slot_elems: int, mode: str = "oneshot",
                  timeout_iters: int = 1 << 24, helper: Any = None) -> Any:
    """Flatten a :class:`~..parallel.p2p.P2PAllReduce` (dedicated to this loop) into the
    kernel's exchange descriptor.  ``slot_elems``: slot stride (>= the parameter count,
    >= the helper exchange array); ``mode``: "oneshot" (every gradient to every rank),
    "rsag" (reduce-scatter to an owner rank + all-gather of the sums; needs 2 (world + 1)
    slots per rank) or "helpers" (``helper`` = (xg_out, xg_red, xready, xdone, nh, xe):
    helper workgroups run the one-shot exchange off the loop's CU)."""
    peers, local, rank, world, slot, err, _ = p2p._h.ll_info()
    cap = 2 * world * slot  # LL elements per rank's buffer
    info = [world, rank, int(slot_elems), local, err, xepoch.data_ptr(), int(timeout_iters), XMODES[mode],
            cap] + list(peers)
    if mode == "helpers":
        info += [int(v) for v in helper]  # xg_out, xg_red, xready, xdone (device addresses), nh, xe
    return info


def helper_buffers(p2p: Any, hidden: int, out_dim: int) -> Any:
    """The helper form's hand-off buffers, carved from the p2p buffer's uncached data
    and flag regions (unused by the LL protocol): plain stores there reach memory
    before an s_waitcnt returns, so a relaxed flag suffices -- no L2 write-back or
    invalidate per step.  Returns (xg_out, xg_red, xready, xdone, nh, xe)."""
    xe = helper_elems(hidden, out_dim)
    nh = -(-xe // 512)  # 512 elements (one per thread) per helper: two per 32-unit hidden tile + the output bias
    data, dbytes, flags, fbytes = p2p._h.regions()
    if 4 * xe * 4 > dbytes or (16 + nh) * 4 > fbytes or nh > 255 or out_dim > 64:
        return None
    return (data, data + 2 * xe * 4, flags, flags + 16 * 4, nh, xe)  # xready [2][8 waves], xdone [nh]


STAGE_ROWS, STAGE_COLS = 128, 32


def make_stage(device: Any) -> Any:
    """Double-buffered staging slots for the pipelined batch gather."""
    return (torch.zeros(2, STAGE_ROWS, STAGE_COLS, dtype=torch.bfloat16, device=device),
            torch.zeros(2, STAGE_ROWS, 8, dtype=torch.float32, device=device),
            torch.zeros(1, dtype=torch.int32, device=device))  # loss cursor


def fused_step(
    X: torch.Tensor, T: torch.Tensor, idx_ring: torch.Tensor, cursor: torch.Tensor, stage: torch.Tensor,
    loss_ring: torch.Tensor, p_in: torch.Tensor, p_out: torch.Tensor, g_prev: torch.Tensor, g_out: torch.Tensor,
    mom_in: torch.Tensor, mom_out: torch.Tensor,
    layout: MlpLayout, batch: int, own_tiles: int, act: str, loss: str, apply_update: bool,
    grad_scale: float, sgd: Dict[str, float], prev_grad_scale: float, first_step: bool, stream: Any = None,
    dbg_stamps: Any = None, parity: int = 0, gather_self: bool = True,
) -> None:
    """One fused step.  ``gather_self`` reads this step's batch straight from the
    index ring at ``cursor`` (and leaves the cursor for the caller to advance);
    otherwise the batch comes from staging slot ``parity``, which the previous
    step filled, and the kernel advances the cursor itself.  Either way the next
    step's batch is staged into slot ``1 - parity``."""
    C = native()
    C.mlp2_fused_step(
        X, T, idx_ring, cursor, stage[2], stage[0], stage[1], loss_ring, p_in, p_out, g_prev, g_out, mom_in, mom_out,
        layout.offsets, layout.in_dim, layout.hidden, layout.out_dim, int(batch), int(own_tiles),
        ACTIVATIONS[act], LOSSES[loss], bool(apply_update), int(parity), bool(gather_self), float(grad_scale),
        float(sgd.get("lr", 1e-3)), float(sgd.get("momentum", 0.0)), float(sgd.get("dampening", 0.0)),
        float(sgd.get("weight_decay", 0.0)), float(prev_grad_scale), bool(sgd.get("nesterov", False)),
        bool(sgd.get("maximize", False)), bool(first_step), -1 if stream is None else int(stream.cuda_stream),
        dbg_stamps,
    )


def _act(x: torch.Tensor, act: str) -> torch.Tensor:
    if act == "relu":
        return F.relu(x)
    if act in ("gelu", "gelu_tanh"):
        return F.gelu(x, approximate="tanh")
    if act == "silu":
        return F.silu(x)
    return x


def loss_fn(y: torch.Tensor, t: torch.Tensor, loss: str) -> torch.Tensor:
    if loss == "mse":
        return F.mse_loss(y, t)
    return F.cross_entropy(y, t)


def reference_step(
    X: torch.Tensor, T: torch.Tensor, idx: torch.Tensor, params: Dict[str, torch.Tensor], act: str, loss: str,
    emulate_bf16: bool = False,
) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """fp32 autograd reference of one step on the gathered batch.

    With ``emulate_bf16`` the forward MFMA operands are rounded to bf16 exactly
    as the kernel does (X, W1 for layer 1; act(H), W2 for layer 2)."""
    p = {k: v.detach().clone().float().requires_grad_(True) for k, v in params.items()}
    x = X[idx.long()].float()
    t = T[idx.long()].float()
    w1 = p["fc1.weight"]
    if emulate_bf16:
        h = x.bfloat16().float() @ w1.bfloat16().float().t() + p["fc1.bias"]
    else:
        h = x @ w1.t() + p["fc1.bias"]
    a = _act(h, act)
    if emulate_bf16:
        y = a.bfloat16().float() @ p["fc2.weight"].bfloat16().float().t() + p["fc2.bias"]
    else:
        y = a @ p["fc2.weight"].t() + p["fc2.bias"]
    lv = loss_fn(y, t, loss)
    lv.backward()
    return lv.detach(), {k: v.grad.detach() for k, v in p.items()}


def apply_sgd_reference(p: torch.Tensor, g: torch.Tensor, buf: Optional[torch.Tensor], sgd: Dict[str, float],
                        first_step: bool) -> torch.Tensor:
    """torch.optim.SGD single-tensor math (for tests)."""
    lr = sgd.get("lr", 1e-3)
    mom = sgd.get("momentum", 0.0)
    damp = sgd.get("dampening", 0.0)
    wd = sgd.get("weight_decay", 0.0)
    d = -g if sgd.get("maximize", False) else g.clone()
    if wd:
        d = d + wd * p
    if mom:
        if first_step:
            buf.copy_(d)
        else:
            buf.mul_(mom).add_(d, alpha=1 - damp)
        d = d + mom * buf if sgd.get("nesterov", False) else buf
    return p - lr * d
