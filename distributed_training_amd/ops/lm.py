"""Autograd ops for the transformer models, backed by the gfx950 kernels of
``csrc/attention.hip`` and ``csrc/lm_ops.hip``.

GPU tensors always take the HIP kernels (bf16 activations required -- the
models run under bf16 mixed precision on GPU; anything else raises).  CPU
tensors use the equivalent PyTorch math, which is also the numerics reference
of the GPU tests.  Plain GEMMs (the projections) stay on ``F.linear``
(hipBLASLt), as the build rules allow for unfused library GEMMs.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F
from torch.autograd import Function

from . import native


def _need_bf16(*ts):
    for t in ts:
        if t.dtype != torch.bfloat16:
            raise TypeError(f"GPU transformer ops need bf16 tensors (got {t.dtype}); "
                            "train the LM configs with mixed_precision=bf16")


# ------------------------------------------------------------------ attention
def attention_reference(q, k, v, causal: bool = True, scale: Optional[float] = None) -> torch.Tensor:
    """[B, S, H, D] / [B, S, Hkv, D] -> [B, S, H, D], fp32 math."""
    B, S, H, D = q.shape
    Hkv = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    if Hkv != H:
        kf = kf.repeat_interleave(H // Hkv, dim=1)
        vf = vf.repeat_interleave(H // Hkv, dim=1)
    s = (qf @ kf.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    return (p @ vf).transpose(1, 2).to(q.dtype)


class _FlashAttn(Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = native().attn_fwd(q, k, v, bool(causal), float(scale), -1)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        do = do.contiguous()
        dq, dk, dv = native().attn_bwd(do, q, k, v, o, lse, bool(ctx.causal), float(ctx.scale), -1)
        return dq, dk, dv, None, None


def attention(q, k, v, causal: bool = True, scale: Optional[float] = None) -> torch.Tensor:
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if q.is_cuda:
        _need_bf16(q, k, v)
        return _FlashAttn.apply(q, k, v, causal, scale)
    return attention_reference(q, k, v, causal, scale)


# ------------------------------------------------------------------ norms
class _Norm(Function):
    @staticmethod
    def forward(ctx, x, w, b, rms, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, mean, rstd = native().norm_fwd(x2, w.contiguous(), None if rms else b.contiguous(), rms, eps, -1)
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.rms, ctx.shape = rms, shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = native().norm_bwd(dy.reshape(x2.shape).contiguous(), x2, w.contiguous(), mean, rstd, ctx.rms,
                                       -1)
        return dx.view(ctx.shape), dw, (None if ctx.rms else db), None, None


def layer_norm(x, w, b, eps: float = 1e-5):
    if x.is_cuda:
        _need_bf16(x, w, b)
        return _Norm.apply(x, w, b, False, eps)
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def rms_norm(x, w, eps: float = 1e-5):
    if x.is_cuda:
        _need_bf16(x, w)
        return _Norm.apply(x, w, None, True, eps)
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype) * w


# ------------------------------------------------------------------ activations
class _Gelu(Function):
    @staticmethod
    def forward(ctx, x):
        xc = x.contiguous()
        ctx.save_for_backward(xc)
        return native().gelu_fwd(xc, -1)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return native().gelu_bwd(dy.contiguous(), x, -1)


def gelu(x):
    if x.is_cuda:
        _need_bf16(x)
        return _Gelu.apply(x)
    return F.gelu(x, approximate="tanh")


class _SwiGLU(Function):
    @staticmethod
    def forward(ctx, ab):
        abc = ab.contiguous()
        ctx.save_for_backward(abc)
        return native().swiglu_fwd(abc, -1)

    @staticmethod
    def backward(ctx, dy):
        (ab,) = ctx.saved_tensors
        return native().swiglu_bwd(dy.contiguous(), ab, -1)


def swiglu(ab):
    """``silu(a) * b`` for ``ab = [a | b]`` along the last dim."""
    if ab.is_cuda:
        _need_bf16(ab)
        return _SwiGLU.apply(ab)
    a, b = ab.chunk(2, dim=-1)
    return F.silu(a) * b


# ------------------------------------------------------------------ rotary
def rope_tables(seq_len: int, head_dim: int, theta: float = 10000.0, device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(seq_len, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def rope_reference(x, cos, sin):
    S, D = x.shape[1], x.shape[-1]
    c = cos[:S].view(1, S, 1, D // 2).to(torch.float32)
    s = sin[:S].view(1, S, 1, D // 2).to(torch.float32)
    x1, x2 = x.float()[..., : D // 2], x.float()[..., D // 2:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)


class _Rope(Function):
    @staticmethod
    def forward(ctx, x, cos, sin):
        y = x.contiguous().clone()
        native().rope_(y, cos, sin, False, -1)
        ctx.save_for_backward(cos, sin)
        return y

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        dx = dy.contiguous().clone()
        native().rope_(dx, cos, sin, True, -1)
        return dx, None, None


def apply_rope(x, cos, sin):
    """Rotate-half RoPE on [B, S, heads, D]."""
    if x.is_cuda:
        _need_bf16(x)
        return _Rope.apply(x, cos, sin)
    return rope_reference(x, cos, sin)


# ------------------------------------------------------------------ loss
class _CrossEntropy(Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):
        # no host sync: the valid-token count stays on the device
        count = (target != ignore_index).sum().clamp_min(1).float()
        dlogits = torch.empty_like(logits)
        loss_rows = native().cross_entropy_fwd_bwd(logits, dlogits, target, 1.0, ignore_index, -1)
        ctx.save_for_backward(dlogits, count)
        return loss_rows.sum() / count

    @staticmethod
    def backward(ctx, g):
        dlogits, count = ctx.saved_tensors
        return dlogits * (g / count).to(dlogits.dtype), None, None


def cross_entropy(logits, target, ignore_index: int = -100):
    """Mean token cross-entropy over ``logits [N, V]`` (fused fwd+bwd kernel on GPU)."""
    if logits.is_cuda:
        _need_bf16(logits)
        return _CrossEntropy.apply(logits.contiguous(), target.contiguous(), ignore_index)
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index)
