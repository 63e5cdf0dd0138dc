"""MLP models.

The reference's "toy MLP" is a single ``torch.nn.Linear(20, 1)``
(src/distributed_trainer.py:199, conf/model/default.yaml) -- kept as the
default model for parity.  :class:`MLP` is the multi-layer model named by the
benchmark configs ("2-layer MLP", BASELINE.json): ``Linear(in, hidden) ->
act -> Linear(hidden, out)`` with ``fc1``/``fc2`` parameter names; its
training step has a dedicated fused gfx950 kernel (``ops/mlp_fused.py``).
"""
from __future__ import annotations

from typing import Any, List, Sequence, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

ACTS = {
    "relu": F.relu,
    "gelu": lambda x: F.gelu(x, approximate="tanh"),
    "gelu_tanh": lambda x: F.gelu(x, approximate="tanh"),
    "silu": F.silu,
    "none": lambda x: x,
}


class MLP(nn.Module):
    def __init__(self, input_size: int = 20, hidden_size: Union[int, Sequence[int]] = 512, output_size: int = 1,
                 activation: str = "relu") -> None:
        super().__init__()
        hidden: List[int] = [hidden_size] if isinstance(hidden_size, int) else list(hidden_size)
        dims = [input_size] + hidden + [output_size]
        self.activation = activation
        self._act = ACTS[activation]
        for i in range(len(dims) - 1):
            self.add_module(f"fc{i + 1}", nn.Linear(dims[i], dims[i + 1]))
        self.num_layers = len(dims) - 1
        self.input_size, self.output_size = input_size, output_size
        self.hidden = hidden

    def layers(self) -> List[nn.Linear]:
        return [getattr(self, f"fc{i + 1}") for i in range(self.num_layers)]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        ls = self.layers()
        for layer in ls[:-1]:
            x = self._act(layer(x))
        return ls[-1](x)

    def is_fused_eligible(self) -> bool:
        """2-layer shape covered by the fused train-step kernel."""
        return self.num_layers == 2


def build_mlp(cfg_model: Any) -> nn.Module:
    """``cfg.model`` -> module.  No ``hidden_size`` => the reference's Linear."""
    get = cfg_model.get if hasattr(cfg_model, "get") else (lambda k, d=None: getattr(cfg_model, k, d))
    hidden = get("hidden_size", None)
    in_size = int(get("input_size", 20))
    out_size = int(get("output_size", 1))
    if not hidden:
        return nn.Linear(in_size, out_size)
    return MLP(in_size, hidden, out_size, activation=str(get("activation", "relu")))
