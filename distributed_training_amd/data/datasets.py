"""Synthetic datasets and the device-resident data loader.

Reference: ``MyTrainDataset`` (src/data_utils.py:7-16) builds a Python list of
``(torch.rand(20), torch.rand(1))`` pairs; ``prepare_dataloader``
(src/distributed_trainer.py:204-211) wraps it in ``DataLoader(batch_size,
pin_memory=True, shuffle=False, sampler=DistributedSampler(dataset))``, and the
trainer copies every batch host->device (:176-182).

Here the dataset is stored as two contiguous tensors (identical values: the
generator draws in the same per-sample order), and :class:`DeviceDataLoader`
keeps them resident in HBM: a batch is an on-device gather by the sampler's
indices -- identical batches to the torch DataLoader, no collate, no pinned
copies, no host round trip.
"""
from __future__ import annotations

import math
from typing import Any, Iterator, Optional, Tuple

import torch
from torch.utils.data import Dataset

from ..parallel.sampler import DistributedSampler


class MyTrainDataset(Dataset):
    """``size`` samples of ``(rand(input_size), rand(output_size))``.

    With ``seed=None`` the global torch RNG is used exactly like the reference
    (unseeded: every rank draws its own data).  Values are drawn sample by
    sample, so for the same RNG state the data equals the reference's list.
    """

    def __init__(self, size: int, input_size: int = 20, output_size: int = 1, seed: Optional[int] = None,
                 vectorized: Optional[bool] = None) -> None:
        self.size = int(size)
        gen = None
        if seed is not None:
            gen = torch.Generator()
            gen.manual_seed(int(seed))
        if vectorized is None:
            vectorized = self.size > 200_000
        if vectorized:  # fast path for big synthetic sets (different draw order)
            self.X = torch.rand(self.size, input_size, generator=gen)
            self.Y = torch.rand(self.size, output_size, generator=gen)
        else:
            self.X = torch.empty(self.size, input_size)
            self.Y = torch.empty(self.size, output_size)
            for i in range(self.size):
                self.X[i] = torch.rand(input_size, generator=gen)
                self.Y[i] = torch.rand(output_size, generator=gen)

    @property
    def data(self) -> Any:
        return list(zip(self.X, self.Y))

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, index: int) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.X[index], self.Y[index]


class SyntheticTokens(Dataset):
    """Random token sequences for the GPT-2 / Llama benchmark configs
    (random-init weights, synthetic data: there is no dataset download)."""

    def __init__(self, size: int, seq_len: int, vocab_size: int, seed: int = 0) -> None:
        g = torch.Generator()
        g.manual_seed(seed)
        self.seq_len = seq_len
        self.tokens = torch.randint(0, vocab_size, (size, seq_len + 1), generator=g, dtype=torch.int64)

    def __len__(self) -> int:
        return self.tokens.shape[0]

    def __getitem__(self, i: int) -> Any:
        t = self.tokens[i]
        return t[:-1], t[1:]


class DeviceDataLoader:
    """DataLoader-compatible iterator over device-resident tensors.

    Yields exactly the batches ``DataLoader(ds, batch_size, shuffle=False,
    sampler=sampler, drop_last=drop_last)`` would, already on ``device``.
    """

    def __init__(self, dataset: Any, batch_size: int, sampler: Optional[DistributedSampler] = None,
                 device: Optional[torch.device] = None, drop_last: bool = False) -> None:
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.sampler = sampler if sampler is not None else DistributedSampler(dataset)
        self.drop_last = drop_last
        self.device = torch.device("cpu") if device is None else torch.device(device)
        self.pin_memory = False
        self._tensors = None

    def to(self, device: Any) -> "DeviceDataLoader":
        self.device = torch.device(device)
        self._tensors = None
        return self

    def tensors(self) -> Tuple[torch.Tensor, ...]:
        """The dataset's columns, resident on ``self.device``."""
        if self._tensors is None:
            ds = self.dataset
            if hasattr(ds, "X") and hasattr(ds, "Y"):
                cols = (ds.X, ds.Y)
            elif hasattr(ds, "tokens"):
                cols = (ds.tokens,)
            else:
                items = [ds[i] for i in range(len(ds))]
                cols = tuple(torch.stack([it[c] for it in items]) for c in range(len(items[0])))
            self._tensors = tuple(c.to(self.device).contiguous() for c in cols)
        return self._tensors

    def __len__(self) -> int:
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def epoch_indices(self) -> torch.Tensor:
        return self.sampler.epoch_indices()

    def __iter__(self) -> Iterator:
        cols = self.tensors()
        idx = self.epoch_indices().to(self.device)
        nb = len(self)
        is_tokens = hasattr(self.dataset, "tokens") and not hasattr(self.dataset, "X")
        for b in range(nb):
            sl = idx[b * self.batch_size:(b + 1) * self.batch_size]
            if is_tokens:
                t = cols[0].index_select(0, sl)
                yield t[:, :-1], t[:, 1:]
            else:
                yield tuple(c.index_select(0, sl) for c in cols)
