"""Size-selected routing between RCCL and the IPC push data plane.

A ring all-reduce over xGMI is per-link bound (one outgoing link per GPU per ring);
the IPC collectives of ``csrc/ipc_coll.hip`` push each rank's chunk to every peer
over all 7 point-to-point links in one hop.  Which of the two is faster depends on
the op, the dtype and the message size, and on the node -- so it is MEASURED, once,
when the communicator is built:

* both data planes are built and self-tested (IpcComm checks every op exactly on
  known values); any failure on any rank -> RCCL for everything;
* every (op, dtype, size class) -- all-reduce / all-gather / reduce-scatter, fp32 /
  bf16, 1 / 4 / 16 / 64 MiB -- is timed on both, the per-rank times are MAX-reduced
  over the ranks (so every rank takes the SAME decision: collectives are issued in the
  same order on every rank of each data plane), and the faster one (IPC only when it
  wins by ``margin``) serves every message of that class;
* each message then goes to the route of the smallest class at least its size (the
  largest class beyond).  Broadcast, all-to-all and barrier stay on the primary.

The routes of the table are logged and exposed (:meth:`routes`: bench_lm.py emits
them in its JSON).  Anything the router does not route -- the fused programs'
``all_reduce_inline``, the p2p one-shot, ``check_errors`` -- is the primary's.

Reference call sites served: the DDP bucket all-reduce (src/dist_strategy/ddp_strategy.py:18)
and FSDP's all-gather / reduce-scatter (src/dist_strategy/fsdp_strategy.py:20).
"""
from __future__ import annotations

import logging
import time
from typing import Any, Dict, List, Optional, Tuple

import torch

from .comm import CommWork, Communicator

logger = logging.getLogger(__name__)

MiB = 1 << 20
SIZES = (1 * MiB, 4 * MiB, 16 * MiB, 64 * MiB)
OPS = ("all_reduce", "all_gather", "reduce_scatter")
DTYPES = (torch.float32, torch.bfloat16)


class RoutedComm(Communicator):
    name = "routed"

    def __init__(self, primary: Communicator, fast: Communicator, sizes: Tuple[int, ...] = SIZES,
                 margin: float = 0.9, calibrate: bool = True, iters: int = 5,
                 table: Optional[Dict[Tuple[str, torch.dtype], List[str]]] = None) -> None:
        """``primary``: the default data plane (RCCL); ``fast``: the IPC push collectives.
        ``table`` (tests): a fixed route table instead of the calibration."""
        self.primary, self.fast = primary, fast
        self.rank, self.world_size, self.device = primary.rank, primary.world_size, primary.device
        self.sizes = tuple(sizes)
        self.margin = float(margin)
        self.timings: Dict[str, float] = {}
        if table is not None:
            self.table = dict(table)
        elif calibrate:
            self.table = self._calibrate(iters)
        else:
            self.table = {(op, dt): ["primary"] * len(self.sizes) for op in OPS for dt in DTYPES}
        self.counts = {"primary": 0, "fast": 0}

    # ------------------------------------------------------------ routing
    def _route(self, op: str, dtype: torch.dtype, nbytes: int) -> Communicator:
        routes = self.table.get((op, dtype))
        if routes is None:
            return self.primary
        k = next((i for i, s in enumerate(self.sizes) if nbytes <= s), len(self.sizes) - 1)
        r = routes[k]
        self.counts[r] += 1
        return self.fast if r == "fast" else self.primary

    def routes(self) -> Dict[str, str]:
        """``"all_reduce bf16 <=4MiB" -> "ipc" | "rccl"`` for the log / bench JSON."""
        out = {}
        pn = getattr(self.primary, "name", "primary")
        fn = getattr(self.fast, "name", "fast")
        for (op, dt), rs in sorted(self.table.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
            for s, r in zip(self.sizes, rs):
                out[f"{op} {str(dt).replace('torch.', '')} <={s // MiB}MiB"] = fn if r == "fast" else pn
        return out

    # ------------------------------------------------------------ calibration
    def _time(self, comm: Communicator, op: str, dt: torch.dtype, nbytes: int, iters: int) -> float:
        W = self.world_size
        n = max(8 * W, nbytes // torch.empty((), dtype=dt).element_size() // (8 * W) * (8 * W))
        dev = self.device
        if op == "all_reduce":
            x = torch.ones(n, dtype=dt, device=dev)
            fn = lambda: comm.all_reduce(x, "sum")  # noqa: E731
        elif op == "all_gather":
            inp = torch.ones(n // W, dtype=dt, device=dev)
            out = torch.empty(n, dtype=dt, device=dev)
            fn = lambda: comm.all_gather_into(out, inp)  # noqa: E731
        else:
            inp = torch.ones(n, dtype=dt, device=dev)
            out = torch.empty(n // W, dtype=dt, device=dev)
            fn = lambda: comm.reduce_scatter_into(out, inp, "sum")  # noqa: E731

        def sync() -> None:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)

        for _ in range(2):
            fn()
        sync()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        sync()
        return (time.perf_counter() - t0) / iters

    def _calibrate(self, iters: int) -> Dict[Tuple[str, torch.dtype], List[str]]:
        keys = [(op, dt, s) for op in OPS for dt in DTYPES for s in self.sizes]
        t = torch.zeros(2 * len(keys), dtype=torch.float64)
        ok = 1.0
        try:
            for i, (op, dt, s) in enumerate(keys):
                t[2 * i] = self._time(self.primary, op, dt, s, iters)
                t[2 * i + 1] = self._time(self.fast, op, dt, s, iters)
        except Exception as e:  # noqa: BLE001 - a failing route: every rank falls back to the primary
            logger.warning("routed comm calibration failed on rank %d (%s); primary data plane only", self.rank, e)
            ok = 0.0
        tt = torch.cat([t, torch.tensor([-ok], dtype=torch.float64)]).to(
            self.device if self.device.type == "cuda" else "cpu")
        self.primary.all_reduce(tt, "max")  # every rank: the slowest rank's time, and whether any failed
        tt = tt.cpu()
        table: Dict[Tuple[str, torch.dtype], List[str]] = {}
        failed = float(tt[-1]) > -1.0
        for i, (op, dt, s) in enumerate(keys):
            tp, tf = float(tt[2 * i]), float(tt[2 * i + 1])
            self.timings[f"{op} {str(dt).replace('torch.', '')} {s // MiB}MiB"] = (round(tp * 1e6, 1),
                                                                                  round(tf * 1e6, 1))
            r = "fast" if (not failed and tf < self.margin * tp) else "primary"
            table.setdefault((op, dt), []).append(r)
        logger.info("routed comm table (rank %d): %s", self.rank, self.routes_from(table))
        return table

    def routes_from(self, table: Any) -> str:
        saved, self.table = getattr(self, "table", None), table
        try:
            return ", ".join(f"{k}: {v}" for k, v in self.routes().items())
        finally:
            if saved is not None:
                self.table = saved

    # ------------------------------------------------------------ Communicator API
    def supports_avg(self) -> bool:
        return self.primary.supports_avg() and self.fast.supports_avg()

    def all_reduce(self, t: Any, op: str = "sum", async_op: bool = False) -> Optional[CommWork]:
        c = self._route("all_reduce", t.dtype, t.numel() * t.element_size()) if op in ("sum", "avg") \
            else self.primary
        return c.all_reduce(t, op=op, async_op=async_op)

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False) -> Optional[CommWork]:
        c = self._route("all_gather", inp.dtype, out.numel() * out.element_size())
        return c.all_gather_into(out, inp, async_op=async_op)

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum",
                            async_op: bool = False) -> Optional[CommWork]:
        c = self._route("reduce_scatter", inp.dtype, inp.numel() * inp.element_size()) if op in ("sum", "avg") \
            else self.primary
        return c.reduce_scatter_into(out, inp, op=op, async_op=async_op)

    def broadcast(self, t: Any, src: int = 0, async_op: bool = False) -> Optional[CommWork]:
        return self.primary.broadcast(t, src=src, async_op=async_op)

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        self.primary.all_to_all_single(out, inp)

    def barrier(self) -> None:
        self.primary.barrier()

    def poll_errors(self) -> None:
        for c in (self.primary, self.fast):
            poll = getattr(c, "poll_errors", None)
            if poll is not None:
                poll()

    def watch_stream(self, stream: Any, desc: str) -> None:
        watch = getattr(self.primary, "watch_stream", None)
        if watch is not None:
            watch(stream, desc)

    def destroy(self) -> None:
        for c in (self.fast, self.primary):
            d = getattr(c, "destroy", None)
            if d is not None:
                d()

    # everything else (all_reduce_inline, _p2p, check_errors, ...): the primary's
    def __getattr__(self, name: str) -> Any:
        if name in ("primary", "fast"):
            raise AttributeError(name)
        return getattr(self.primary, name)
