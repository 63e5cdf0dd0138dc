"""Checkpoint manager.

Reference: ``ModelCheckpoint`` (src/distributed_trainer.py:73-105) and the
strategies' ``save_checkpoint``/``load_checkpoint``
(src/dist_strategy/ddp_strategy.py:23-32, fsdp_strategy.py:28-46).

Format (unchanged, byte-compatible): a ``torch.save`` of
``{"MODEL_STATE": OrderedDict[str, Tensor], "EPOCHS_RUN": int}`` -- DDP keys
``module.<name>``, FSDP keys unprefixed -- loadable with
``torch.load(..., weights_only=True)``.  Optional extra keys (``OPTIM_STATE``:
the complete optimizer state -- FSDP's gathered from every rank's shards and
keyed by parameter name -- restored on resume) do not break reference loaders.

Fixes: the model state is collected on ALL ranks (the
FSDP full-state-dict gather is a collective), only global rank 0 writes, the
write goes to a temporary file + ``os.replace`` (atomic), then all ranks meet
at a barrier so nobody resumes from a half-written file.
"""
from __future__ import annotations

import logging
import os
from pathlib import Path
from typing import Any, Optional, Tuple

import torch

logger = logging.getLogger("distributed_training_amd.trainer")


class ModelCheckpoint:
    """Handles model checkpointing operations."""

    def __init__(self, path: Path, env: Any, strategy: Any, save_optimizer: bool = False) -> None:
        self.path = Path(path)
        self.env = env
        self.strategy = strategy
        self.save_optimizer = save_optimizer

    def save(self, model: torch.nn.Module, epoch: int, optimizer: Optional[torch.optim.Optimizer] = None) -> None:
        # collective on every rank (FSDP full-state gather), write on rank 0
        model_state = self.strategy.model_state(model)
        optim_state = None
        if self.save_optimizer and optimizer is not None:  # collective too (FSDP gathers its shards)
            optim_state = self.strategy.optim_state(model, optimizer)
        if self.env.global_rank == 0:
            state_dict = {"MODEL_STATE": model_state, "EPOCHS_RUN": epoch}
            if optim_state is not None:
                state_dict["OPTIM_STATE"] = optim_state
            self.strategy.save_checkpoint(model, state_dict, str(self.path))
            logger.info(f"Epoch {epoch} | Training snapshot saved at {self.path}")
        self.env.barrier()

    def load(self, model: torch.nn.Module, device: Any,
             optimizer: Optional[torch.optim.Optimizer] = None) -> Tuple[torch.nn.Module, int]:
        if not self.path.exists():
            return model, 0
        logger.info("Loading snapshot")
        # tensors stay on the host: the strategy copies each into place (an 8B-parameter
        # FSDP snapshot would otherwise be materialised on every rank's GPU at once)
        # memory-mapped: each rank pages in only what it copies (an FSDP rank reads its shard ranges)
        try:
            snapshot = torch.load(self.path, map_location="cpu", weights_only=True, mmap=True)
        except RuntimeError:  # legacy (non-zip) format cannot be mapped
            snapshot = torch.load(self.path, map_location="cpu", weights_only=True)
        model, epochs = self.strategy.load_checkpoint(model, snapshot, device)
        if optimizer is not None and "OPTIM_STATE" in snapshot:
            self.strategy.load_optim_state(model, optimizer, snapshot["OPTIM_STATE"])
            logger.info("Optimizer state restored")
        return model, epochs


def atomic_torch_save(obj: Any, path: str) -> None:
    p = Path(path)
    if p.parent and not p.parent.exists():
        p.parent.mkdir(parents=True, exist_ok=True)
    tmp = p.with_name(p.name + f".tmp{os.getpid()}")
    torch.save(obj, tmp)
    os.replace(tmp, p)
