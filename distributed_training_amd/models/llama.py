"""Llama-3 (8B by default), random init, for the Llama-3 8B FSDP configuration
of BASELINE.json.

RMSNorm pre-norm blocks, grouped-query attention (32 query / 8 key-value heads)
with rotary embeddings (theta 500000), SwiGLU FFN (14336), untied output head,
vocab 128256.  The QKV and gate/up projections are fused (one GEMM each); on
GPU the non-GEMM work runs on the gfx950 kernels of ``ops/lm.py``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any, List, Optional, Tuple

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint

from ..ops import lm


@dataclass
class LlamaConfig:
    n_layer: int = 32
    n_head: int = 32
    n_kv_head: int = 8
    n_embd: int = 4096
    ffn_hidden: int = 14336
    vocab_size: int = 128256
    block_size: int = 8192
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    tie_weights: bool = False

    @staticmethod
    def from_cfg(c: Any) -> "LlamaConfig":
        g = c.get if hasattr(c, "get") else (lambda k, d=None: getattr(c, k, d))
        return LlamaConfig(int(g("n_layer", 32)), int(g("n_head", 32)), int(g("n_kv_head", 8)),
                           int(g("n_embd", 4096)), int(g("ffn_hidden", 14336)), int(g("vocab_size", 128256)),
                           int(g("block_size", 8192)), float(g("rope_theta", 500000.0)),
                           float(g("norm_eps", 1e-5)), bool(g("tie_weights", False)))


class RMSNorm(nn.Module):
    def __init__(self, n: int, eps: float) -> None:
        super().__init__()
        self.weight = nn.Parameter(torch.ones(n))
        self.eps = eps

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return lm.rms_norm(x, self.weight, self.eps)

    def add_forward(self, x: torch.Tensor, res: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """``(x + res, RMSNorm(x + res))`` in one kernel; ``res=None`` -> ``(x, RMSNorm(x))``."""
        if res is None:
            return x, self(x)
        return lm.add_rms_norm(x, res, self.weight, self.eps)


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig) -> None:
        super().__init__()
        self.H, self.Hkv = cfg.n_head, cfg.n_kv_head
        self.D = cfg.n_embd // cfg.n_head
        self.wqkv = lm.Linear(cfg.n_embd, (self.H + 2 * self.Hkv) * self.D, bias=False)
        self.wo = lm.Linear(self.H * self.D, cfg.n_embd, bias=False)

    def forward(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
        B, S, _ = x.shape
        # RoPE + GQA attention on the packed projection output (one packed dQKV in backward)
        y = lm.attention_packed(self.wqkv(x), self.H, self.Hkv, causal=True, rope=(cos, sin), rope_inplace=True)
        return self.wo(y.reshape(B, S, self.H * self.D))


class FeedForward(nn.Module):
    def __init__(self, cfg: LlamaConfig) -> None:
        super().__init__()
        self.w13 = lm.Linear(cfg.n_embd, 2 * cfg.ffn_hidden, bias=False)
        self.w2 = lm.Linear(cfg.ffn_hidden, cfg.n_embd, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # w2(swiglu(.)) as one op: its input gradient carries the SwiGLU backward in the GEMM epilogue
        return lm.swiglu_linear(self.w13(x), self.w2.weight)


class Block(nn.Module):
    def __init__(self, cfg: LlamaConfig) -> None:
        super().__init__()
        self.attention_norm = RMSNorm(cfg.n_embd, cfg.norm_eps)
        self.attention = Attention(cfg)
        self.ffn_norm = RMSNorm(cfg.n_embd, cfg.norm_eps)
        self.feed_forward = FeedForward(cfg)

    def forward(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, h: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Residual adds fused into the norms (see GPT-2 ``Block``); returns ``(x, h)``."""
        x, y = self.attention_norm.add_forward(x, h)
        x, y = self.ffn_norm.add_forward(x, self.attention(y, cos, sin))
        return x, self.feed_forward(y)


class Llama(nn.Module):
    block_class = Block

    def __init__(self, cfg: LlamaConfig) -> None:
        super().__init__()
        self.cfg = cfg
        self.vocab_size = cfg.vocab_size
        self.tok_embeddings = lm.Embedding(cfg.vocab_size, cfg.n_embd)
        self.layers = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.norm = RMSNorm(cfg.n_embd, cfg.norm_eps)
        self.output = lm.LMHead(cfg.n_embd, cfg.vocab_size, bias=False)
        if cfg.tie_weights:
            self.output.weight = self.tok_embeddings.weight
        cos, sin = lm.rope_tables(cfg.block_size, cfg.n_embd // cfg.n_head, cfg.rope_theta)
        self.register_buffer("rope_cos", cos, persistent=False)
        self.register_buffer("rope_sin", sin, persistent=False)
        self.activation_checkpointing = False
        std = 0.02
        for n, p in self.named_parameters():
            if p.dim() >= 2:
                s = std / math.sqrt(2 * cfg.n_layer) if n.endswith(("wo.weight", "w2.weight")) else std
                nn.init.normal_(p, 0.0, s)

    def init_param(self, name: str, t: torch.Tensor, gen: torch.Generator) -> None:
        """The initial value of parameter ``name`` (the distributions of ``__init__``) drawn into ``t``:
        materialisation of a model built on the meta device (models/init.py)."""
        if t.dim() >= 2:
            std = 0.02 / math.sqrt(2 * self.cfg.n_layer) if name.endswith(("wo.weight", "w2.weight")) else 0.02
            t.normal_(0.0, std, generator=gen)
        else:  # RMSNorm weights
            t.fill_(1.0)

    def init_buffers(self, device: torch.device) -> None:
        """The RoPE tables (non-persistent buffers), computed on the host in fp64 and moved."""
        cos, sin = lm.rope_tables(self.cfg.block_size, self.cfg.n_embd // self.cfg.n_head, self.cfg.rope_theta,
                                  device=device)
        self.rope_cos, self.rope_sin = cos, sin

    def enable_activation_checkpointing(self, on: bool = True) -> None:
        self.activation_checkpointing = on

    def fsdp_extra_units(self) -> List[nn.Module]:
        """Modules that are FSDP units of their own besides the blocks (parallel/fsdp.py
        ``lm_wrap_policy``): the embedding and the output head, 525 M parameters each at 8B --
        in the root unit they would be gathered synchronously before the forward and held
        through the whole backward.  Tied (one weight, used first and last): kept in the root."""
        return [] if self.cfg.tie_weights else [self.tok_embeddings, self.output]

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def forward(self, idx: torch.Tensor, targets: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Logits; with ``targets``, the mean token cross-entropy (head + loss fused)."""
        x = self.tok_embeddings(idx)
        cos, sin = self.rope_cos, self.rope_sin
        h = None
        for blk in self.layers:
            if self.activation_checkpointing and torch.is_grad_enabled():
                x, h = checkpoint(blk, x, cos, sin, h, use_reentrant=False)
            else:
                x, h = blk(x, cos, sin, h)
        _, y = self.norm.add_forward(x, h)
        return self.output(y, targets)

    def activation_bytes_per_token(self, checkpointed: bool = False) -> int:
        """Bytes the forward keeps for the backward, per token (bf16 activations; estimate for the
        ``activation_checkpointing: auto`` decision, app.py).  Per block: block input, norm outputs,
        packed QKV, attention output, residual sum, gate|up and the SwiGLU output, plus the fp32 row
        statistics; checkpointed: the block input only.  The LM head's logits (rewritten in place as
        the logit gradient) come on top in both cases."""
        c = self.cfg
        d = c.n_embd // c.n_head
        qkv = (c.n_head + 2 * c.n_kv_head) * d
        per_block = 2 * (c.n_embd * 5 + qkv + 3 * c.ffn_hidden) + 4 * (4 + c.n_head)
        if checkpointed:
            per_block = 2 * c.n_embd
        return c.n_layer * per_block + 2 * c.vocab_size + 2 * c.n_embd

    def flops_per_token(self, seq_len: int) -> float:
        c = self.cfg
        n = self.num_params() - self.tok_embeddings.weight.numel()
        return 6 * n + 12 * c.n_layer * c.n_embd * seq_len
