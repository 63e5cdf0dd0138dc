"""Distributed environment: rank/device discovery, process-group bring-up,
and the communicator used by the parallel engines.

Reference: ``DistributedEnvironment`` in src/distributed_trainer.py:42-70
(same public attributes: ``device, is_gpu, global_rank, local_rank,
world_size``; ``setup()``).  Differences, each deliberate:

* the ``LOCAL_RANK``/``RANK`` check happens BEFORE ``init_process_group``
  (reference raises after init);
* ``torch.cuda.set_device`` happens before the process group is created so
  RCCL binds to the right GPU;
* a collective timeout is configurable (reference: library default);
* ``comm`` is the native RCCL communicator on GPU (gloo/torch on CPU).
"""
from __future__ import annotations

import datetime
import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

from .comm import Communicator, TorchComm, make_comm

logger = logging.getLogger(__name__)


def _determine_device(device: str) -> str:
    if device == "auto":
        return "cuda" if torch.cuda.is_available() else "cpu"
    return device


class DistributedEnvironment:
    """Manages distributed training setup and environment variables."""

    def __init__(self, device: str = "auto", backend: Optional[str] = None, timeout_s: Optional[float] = None,
                 comm: str = "auto") -> None:
        self.device = _determine_device(device)
        self.is_gpu = self.device == "cuda"
        self.global_rank = int(os.environ.get("RANK", 0))
        # reference quirk kept: local rank is forced to 0 on CPU
        self.local_rank = int(os.environ.get("LOCAL_RANK", 0)) if self.is_gpu else 0
        self.world_size = int(os.environ.get("WORLD_SIZE", 1))
        self.backend = backend
        self.timeout_s = timeout_s
        self.comm_pref = comm
        self._comm: Optional[Communicator] = None
        self._owns_pg = False

    @staticmethod
    def _determine_device(device: str) -> str:
        return _determine_device(device)

    @property
    def torch_device(self) -> torch.device:
        from .ipc import device_index

        return torch.device("cuda", device_index(self.local_rank)) if self.is_gpu else torch.device("cpu")

    def setup(self) -> None:
        if self.is_gpu and ("LOCAL_RANK" not in os.environ or "RANK" not in os.environ):
            if self.world_size > 1:
                raise ValueError("LOCAL_RANK and RANK environment variables must be set for GPU training")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("LOCAL_RANK", "0")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        os.environ.setdefault("RANK", str(self.global_rank))
        os.environ.setdefault("WORLD_SIZE", str(self.world_size))
        if self.is_gpu:
            torch.cuda.set_device(self.torch_device)
        from .ipc import dist_backend

        backend = self.backend or dist_backend(self.is_gpu)
        if not dist.is_initialized():
            kwargs = {}
            if self.timeout_s:
                kwargs["timeout"] = datetime.timedelta(seconds=float(self.timeout_s))
            if self.is_gpu and backend == "nccl":
                kwargs["device_id"] = self.torch_device
            dist.init_process_group(backend=backend, **kwargs)
            self._owns_pg = True
        self.global_rank = dist.get_rank()
        self.world_size = dist.get_world_size()

    @property
    def comm(self) -> Communicator:
        """Communicator for the parallel engines (created lazily, collective)."""
        if self._comm is None:
            if self.is_gpu:
                self._comm = make_comm(self.torch_device, prefer=self.comm_pref)
            else:
                self._comm = TorchComm(device=torch.device("cpu"))
        return self._comm

    def barrier(self) -> None:
        if dist.is_initialized() and dist.get_world_size() > 1:
            if self.is_gpu and dist.get_backend() == "nccl":
                dist.barrier(device_ids=[self.torch_device.index])
            else:
                dist.barrier()

    def teardown(self) -> None:
        if self._comm is not None and hasattr(self._comm, "destroy"):
            try:
                self._comm.destroy()
            except Exception:  # noqa: BLE001
                pass
            self._comm = None
        if dist.is_initialized():
            dist.destroy_process_group()
