"""DistributedSampler-compatible index generation.

Produces exactly the index order of ``torch.utils.data.DistributedSampler``
(``randperm(n, generator.manual_seed(seed + epoch))`` if shuffle, pad by
wrapping to ``ceil(n / ws) * ws`` (or truncate with ``drop_last``), stride
``rank::ws``) -- SURVEY.md §7.4 item 6; the reference uses it at
src/distributed_trainer.py:204-211 with ``set_epoch`` at :175.

Unlike torch's sampler it can hand out whole epochs as int32 tensors so the
device-resident loader can upload them in one copy.
"""
from __future__ import annotations

import math
from typing import Any, Iterator, Optional

import torch
from torch.utils.data import Sampler


class DistributedSampler(Sampler):
    """Drop-in for ``torch.utils.data.distributed.DistributedSampler``."""

    def __init__(self, dataset: Any, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False) -> None:
        if num_replicas is None or rank is None:
            import torch.distributed as dist

            if dist.is_available() and dist.is_initialized():
                num_replicas = dist.get_world_size() if num_replicas is None else num_replicas
                rank = dist.get_rank() if rank is None else rank
            else:
                num_replicas = 1 if num_replicas is None else num_replicas
                rank = 0 if rank is None else rank
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.n = len(dataset)
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        self.shuffle = shuffle
        self.seed = seed
        if self.drop_last and self.n % self.num_replicas != 0:
            self.num_samples = math.ceil((self.n - self.num_replicas) / self.num_replicas)
        else:
            self.num_samples = math.ceil(self.n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def epoch_indices(self, epoch: Optional[int] = None) -> torch.Tensor:
        """This rank's indices for ``epoch`` (default: current) as int64."""
        ep = self.epoch if epoch is None else epoch
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + ep)
            indices = torch.randperm(self.n, generator=g)
        else:
            indices = torch.arange(self.n)
        if not self.drop_last:
            pad = self.total_size - indices.numel()
            if pad > 0:
                if pad <= indices.numel():
                    indices = torch.cat([indices, indices[:pad]])
                else:
                    reps = math.ceil(pad / indices.numel())
                    indices = torch.cat([indices, indices.repeat(reps)[:pad]])
        else:
            indices = indices[: self.total_size]
        assert indices.numel() == self.total_size
        out = indices[self.rank:self.total_size:self.num_replicas]
        assert out.numel() == self.num_samples
        return out

    def __iter__(self) -> Iterator[int]:
        return iter(self.epoch_indices().tolist())

    def __len__(self) -> int:
        return self.num_samples
