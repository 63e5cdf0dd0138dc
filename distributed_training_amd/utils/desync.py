"""Cross-rank replica consistency check (race / desync detector).

The reference has none (its only aid is the playground's
per-rank norm logs, src/playground/ddp_script.py:155-164).  Data-parallel
replicas must hold bit-identical parameters after every optimizer step; this
all-reduces a per-parameter checksum (sum and sum of squares, fp64) with MAX
and MIN and raises if any rank differs.
"""
from __future__ import annotations

import logging
from typing import Any, List

import torch

logger = logging.getLogger(__name__)


class DesyncError(RuntimeError):
    pass


@torch.no_grad()
def param_checksums(model: torch.nn.Module) -> torch.Tensor:
    vals: List[torch.Tensor] = []
    for p in model.parameters():
        x = p.detach().double()
        vals.append(x.sum())
        vals.append((x * x).sum())
    if not vals:
        return torch.zeros(0, dtype=torch.float64)
    return torch.stack(vals)


@torch.no_grad()
def check_replicas_in_sync(model: torch.nn.Module, env: Any, rtol: float = 0.0) -> None:
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    if hasattr(model, "full_state_dict"):  # FSDP: shards differ by construction
        return
    c = param_checksums(model)
    dev = env.torch_device if env.is_gpu and dist.get_backend() == "nccl" else torch.device("cpu")
    hi = c.to(dev).clone()
    lo = c.to(dev).clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    diff = (hi - lo).abs()
    tol = rtol * hi.abs()
    bad = (diff > tol).nonzero().flatten().tolist()
    if bad:
        raise DesyncError(f"replicas out of sync at checksum entries {bad[:8]} (max diff {diff.max().item():.3e})")
    logger.debug("replicas in sync (%d checksums)", c.numel())
