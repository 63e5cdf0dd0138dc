"""GPT-2 (124M "small" by default), random init, for the GPT-2 DDP / FSDP
configurations of BASELINE.json.

Architecture as GPT-2 / nanoGPT: learned token + position embeddings, pre-LN
blocks (LayerNorm -> causal self-attention -> residual, LayerNorm -> GELU MLP ->
residual), final LayerNorm, lm_head tied to the token embedding.  On GPU the
non-GEMM work runs on the gfx950 kernels of ``ops/lm.py`` (flash attention,
LayerNorm, GELU, fused cross-entropy); the projections are plain bf16 GEMMs.
The vocabulary is padded to a multiple of 64 (50257 -> 50304) so the logits
rows are 16-byte aligned.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from ..ops import lm


@dataclass
class GPT2Config:
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    vocab_size: int = 50257
    block_size: int = 1024
    dropout: float = 0.0
    tie_weights: bool = True

    @property
    def padded_vocab(self) -> int:
        return (self.vocab_size + 63) // 64 * 64

    @staticmethod
    def from_cfg(c: Any) -> "GPT2Config":
        g = c.get if hasattr(c, "get") else (lambda k, d=None: getattr(c, k, d))
        return GPT2Config(int(g("n_layer", 12)), int(g("n_head", 12)), int(g("n_embd", 768)),
                          int(g("vocab_size", 50257)), int(g("block_size", 1024)), float(g("dropout", 0.0) or 0.0),
                          bool(g("tie_weights", True)))


class LayerNorm(nn.Module):
    def __init__(self, n: int, eps: float = 1e-5) -> None:
        super().__init__()
        self.weight = nn.Parameter(torch.ones(n))
        self.bias = nn.Parameter(torch.zeros(n))
        self.eps = eps

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return lm.layer_norm(x, self.weight, self.bias, self.eps)

    def add_forward(self, x: torch.Tensor, res: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """``(x + res, LN(x + res))`` in one kernel; ``res=None`` -> ``(x, LN(x))``."""
        if res is None:
            return x, self(x)
        return lm.add_layer_norm(x, res, self.weight, self.bias, self.eps)


class CausalSelfAttention(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        self.n_head = cfg.n_head
        self.c_attn = lm.Linear(cfg.n_embd, 3 * cfg.n_embd)
        self.c_proj = lm.Linear(cfg.n_embd, cfg.n_embd)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, S, C = x.shape
        # q/k/v are read in place from the projection output; dq/dk/dv land in one packed buffer
        y = lm.attention_packed(self.c_attn(x), self.n_head, self.n_head, causal=True)
        return self.c_proj(y.reshape(B, S, C))


class MLP(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        self.c_fc = lm.Linear(cfg.n_embd, 4 * cfg.n_embd)
        self.c_proj = lm.Linear(4 * cfg.n_embd, cfg.n_embd)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # c_proj(gelu(c_fc(x))): the GELU in c_fc's GEMM epilogue (pre-activation and activation stored
        # in one pass), its backward folded into c_proj's input-gradient GEMM
        h, a = lm.linear_gelu(x, self.c_fc.weight, self.c_fc.bias)
        return lm.gelu_linear(h, self.c_proj.weight, self.c_proj.bias, a=a)


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        self.ln_1 = LayerNorm(cfg.n_embd)
        self.attn = CausalSelfAttention(cfg)
        self.ln_2 = LayerNorm(cfg.n_embd)
        self.mlp = MLP(cfg)

    def forward(self, x: torch.Tensor, h: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """``h``: the previous block's MLP output, not yet added to the
        residual stream -- the add is fused into this block's ln_1 (and this
        block's MLP output is handed on the same way), so no residual add runs
        as a separate kernel, forward or backward.  Returns ``(x, h)``."""
        x, y = self.ln_1.add_forward(x, h)
        x, y = self.ln_2.add_forward(x, self.attn(y))
        return x, self.mlp(y)


class GPT2(nn.Module):
    block_class = Block

    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        self.cfg = cfg
        self.vocab_size = cfg.vocab_size
        V = cfg.padded_vocab
        self.wte = nn.Embedding(V, cfg.n_embd)
        self.wpe = nn.Embedding(cfg.block_size, cfg.n_embd)
        self.h = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = LayerNorm(cfg.n_embd)
        self.lm_head = nn.Linear(cfg.n_embd, V, bias=False)
        if cfg.tie_weights:
            self.lm_head.weight = self.wte.weight
        self.activation_checkpointing = False
        self.apply(self._init)
        for n, p in self.named_parameters():
            if n.endswith("c_proj.weight"):
                nn.init.normal_(p, 0.0, 0.02 / math.sqrt(2 * cfg.n_layer))

    @staticmethod
    def _init(m: Any) -> None:
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, 0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, 0.02)

    def init_param(self, name: str, t: torch.Tensor, gen: torch.Generator) -> None:
        """The initial value of parameter ``name`` (the same distributions as ``__init__``) drawn into
        ``t`` -- materialisation of a model built on the meta device (models/init.py)."""
        if name.endswith("c_proj.weight"):
            t.normal_(0.0, 0.02 / math.sqrt(2 * self.cfg.n_layer), generator=gen)
        elif t.dim() >= 2:  # embeddings and Linear weights
            t.normal_(0.0, 0.02, generator=gen)
        elif name.endswith("bias"):
            t.zero_()
        else:  # LayerNorm weights
            t.fill_(1.0)

    def enable_activation_checkpointing(self, on: bool = True) -> None:
        self.activation_checkpointing = on

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def forward(self, idx: torch.Tensor, targets: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Logits ``[B, S, V]``; with ``targets``, the mean token cross-entropy
        (LM head and loss fused: the logits are never materialised twice)."""
        B, S = idx.shape
        # (the token rows' gradient is added straight into the tied head's gradient slice; the
        # positions 0..S-1 are wpe's first S rows: added as a view, no position ids)
        x = lm.add_position(lm.embedding(idx, self.wte.weight), self.wpe.weight)
        h = None
        for blk in self.h:
            if self.activation_checkpointing and torch.is_grad_enabled():
                x, h = checkpoint(blk, x, h, use_reentrant=False)
            else:
                x, h = blk(x, h)
        _, y = self.ln_f.add_forward(x, h)
        if targets is not None:
            return lm.linear_cross_entropy(y, self.lm_head.weight, targets)
        return self.lm_head(y)

    def activation_bytes_per_token(self, checkpointed: bool = False) -> int:
        """Bytes the forward keeps for the backward, per token (bf16; estimate for the
        ``activation_checkpointing: auto`` decision, app.py): per block the input, two LayerNorm
        outputs, qkv, the attention output, the residual sum, the MLP pre-activation and its GELU
        (16 C), plus fp32 row statistics; checkpointed: the block input only.  Logits on top."""
        c = self.cfg
        per_block = 2 * 16 * c.n_embd + 4 * (4 + c.n_head)
        if checkpointed:
            per_block = 2 * c.n_embd
        return c.n_layer * per_block + 2 * c.padded_vocab + 2 * c.n_embd

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs per token (6N + attention), PaLM-style accounting."""
        n = self.num_params() - self.wpe.weight.numel()
        c = self.cfg
        return 6 * n + 12 * c.n_layer * c.n_embd * seq_len
