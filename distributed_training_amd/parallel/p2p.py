"""One-shot intra-node all-reduce over xGMI peer memory (``csrc/p2p_allreduce.hip``).

Used by :class:`~.comm.RcclComm` for small fp32 buckets (the headline MLP's
~45 KB gradient): one kernel pushes the bucket into every
peer's receive slot and sums the slots locally, instead of RCCL's 2(W-1)-hop
ring.  Enabled only when every rank is on this node (``LOCAL_WORLD_SIZE ==
WORLD_SIZE``) and after a numerical self-test agreed on all ranks; otherwise
RCCL is used.  ``DTA_P2P_ALLREDUCE=0`` disables it.
"""
from __future__ import annotations

import logging
import os
from typing import Any, Optional

import torch

logger = logging.getLogger(__name__)

DEFAULT_MAX_ELEMS = 1 << 18        # 1 MiB of fp32 per slot
DEFAULT_TIMEOUT_ITERS = 1 << 26    # ~ seconds of s_sleep polling before the error flag is raised


class P2PAllReduce:
    """Collective constructor: every rank publishes its IPC handle in the
    store (an empty value if allocation failed) before anything can raise, so
    no rank is left waiting on a key that never appears."""

    _seq: dict = {}

    def __init__(self, rank: int, world_size: int, device: torch.device, store: Any, tag: str = "default",
                 max_elems: int = DEFAULT_MAX_ELEMS, timeout_iters: int = DEFAULT_TIMEOUT_ITERS,
                 protocol: str = "ll") -> None:
        from ..ops import native

        self.rank, self.world_size, self.device = rank, world_size, device
        self.timeout_iters = int(timeout_iters)
        # one store key per construction: every rank builds its buffers in the same
        # order, so the n-th construction with a tag agrees across ranks (a reused
        # key could hand a peer the previous buffer's handle)
        seq = P2PAllReduce._seq.get(tag, 0)
        P2PAllReduce._seq[tag] = seq + 1
        key = f"dta_p2p/{tag}/{seq}"
        self._h = None
        err = None
        try:
            with torch.cuda.device(device):
                self._h = native().P2PAllReduce(rank, world_size, int(max_elems))
            mine = self._h.handle()
        except Exception as e:  # noqa: BLE001
            err, mine = e, b""
        store.set(f"{key}/{rank}", mine)
        handles = [store.get(f"{key}/{r}") for r in range(world_size)]
        if err is not None:
            raise err
        if any(len(h) == 0 for h in handles):
            self._h.destroy()
            raise RuntimeError("a peer could not allocate its p2p buffer")
        self.max_elems = self._h.max_elems
        with torch.cuda.device(device):
            self._h.open(handles)
        if protocol not in ("ll", "flag"):
            raise ValueError(f"unknown p2p protocol {protocol!r}")
        self.protocol = protocol
        self._h.set_ll(protocol == "ll")  # identical on every rank (same argument everywhere)

    def supports(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and 0 < t.numel() <= self.max_elems
                and t.data_ptr() % 16 == 0)

    def all_reduce(self, t: torch.Tensor, scale: float = 1.0, stream: Optional[torch.cuda.Stream] = None) -> None:
        s = stream or torch.cuda.current_stream(self.device)
        self._h.all_reduce(t, float(scale), self.timeout_iters, int(s.cuda_stream))

    def check(self) -> None:
        """Raise if any launch timed out waiting for a peer (host sync)."""
        if self._h.error():
            raise RuntimeError(f"rank {self.rank}: p2p all-reduce timed out waiting for a peer")

    def poll(self) -> None:
        """Raise if an all-reduce launch timed out (host-mapped flag: no device sync)."""
        if self._h.error_nosync():
            raise RuntimeError(f"rank {self.rank}: p2p all-reduce timed out waiting for a peer; "
                               "gradients of that step are partial")

    def destroy(self) -> None:
        self._h.destroy()


def intra_node() -> bool:
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(ws)))
    return lws == ws


def maybe_create(rank: int, world_size: int, device: torch.device, store: Any, verify_comm: Any,
                 tag: str = "default") -> Optional[P2PAllReduce]:
    """Create + self-test the p2p path on every rank (collective).  Returns
    None (all ranks agree) when disabled, not intra-node, or the test fails."""
    if world_size < 2 or world_size > 8 or os.environ.get("DTA_P2P_ALLREDUCE", "1") == "0" or not intra_node():
        return None
    ok = 1.0
    p2p = None
    try:
        p2p = P2PAllReduce(rank, world_size, device, store, tag=tag,
                           protocol=os.environ.get("DTA_P2P_PROTOCOL", "ll"))
        for n in (5, 4099, 70001):  # scalar tail, 1 and many workgroups
            x = torch.arange(n, device=device, dtype=torch.float32) * (rank + 1)
            p2p.all_reduce(x, 1.0)
            want = torch.arange(n, device=device, dtype=torch.float32) * (world_size * (world_size + 1) / 2)
            torch.cuda.synchronize(device)
            p2p.check()
            if not torch.equal(x, want):
                ok = 0.0
    except Exception as e:  # noqa: BLE001 - any failure falls back to RCCL
        logger.warning("p2p all-reduce unavailable (%s); using RCCL", e)
        ok = 0.0
    flag = torch.tensor([ok], device=device)
    verify_comm(flag)  # MIN over ranks
    if float(flag.item()) < 1.0:
        if p2p is not None:
            p2p.destroy()
        return None
    logger.debug("p2p one-shot all-reduce enabled (%d ranks, %d elems/slot)", world_size, p2p.max_elems)
    return p2p
