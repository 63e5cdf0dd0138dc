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
* each message then goes to the route of the smallest class at least its size.  The engines
  know every message they will send when they wrap the model -- DDP its bucket sizes, FSDP its
  unit sizes (436 MB per Llama-3 8B layer, 1.05 GB for the embedding / head) -- and hand them to
  :meth:`RoutedComm.prepare` there: every message larger than the default classes gets a class
  of its own (its size rounded up to 16 MiB), calibrated at wrap time for the (op, dtype) pairs
  that will use it -- before the first step, outside any capture, while no activation is
  allocated.  A message past every class that was NOT prepared still adds a class on first use
  (the next power of two; a logged fallback -- it times multi-GB scratch inside a running
  step); inside a graph capture the largest class is used instead.  Broadcast, all-to-all and
  barrier stay on the primary.
* calibration failures are agreed on key by key (a MIN of the success flag over the ranks
  after each timed key), so every rank stops timing the fast plane at the same key.

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
                 table: Optional[Dict[Tuple[str, torch.dtype], List[str]]] = None,
                 lazy_max: int = 4 << 30) -> None:
        """``primary``: the default data plane (RCCL); ``fast``: the IPC push collectives.
        ``table`` (tests): a fixed route table instead of the calibration.  ``lazy_max``: the largest
        class a message may add on first use (0: no lazy classes)."""
        self.primary, self.fast = primary, fast
        self.rank, self.world_size, self.device = primary.rank, primary.world_size, primary.device
        self.sizes = list(sizes)
        self.margin = float(margin)
        self.iters = int(iters)
        self.timings: Dict[str, float] = {}
        self.failed = False
        self.lazy_max = int(lazy_max) if calibrate and table is None else 0
        if table is not None:
            self.table = {k: list(v) for k, v in table.items()}
        elif calibrate:
            self.table = self._calibrate(self.sizes, iters)
        else:
            self.table = {(op, dt): ["primary"] * len(self.sizes) for op in OPS for dt in DTYPES}
        self.counts = {"primary": 0, "fast": 0}
        self.prepared_log: List[Dict[str, Any]] = []  # classes added after construction (bench_lm.py JSON)

    # ------------------------------------------------------------ routing
    def _route(self, op: str, dtype: torch.dtype, nbytes: int) -> Communicator:
        routes = self.table.get((op, dtype))
        if routes is None:
            return self.primary
        if nbytes > self.sizes[-1] and self.lazy_max and nbytes <= self.lazy_max \
                and not (self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            logger.warning("routed comm: %s %s message of %.1f MiB is past every prepared size class: "
                           "calibrating a class inside the running step (the engine should prepare() it "
                           "at wrap)", op, str(dtype).replace("torch.", ""), nbytes / MiB)
            self._add_class(1 << (int(nbytes) - 1).bit_length())
            routes = self.table[(op, dtype)]
        k = next((i for i, s in enumerate(self.sizes) if nbytes <= s), len(self.sizes) - 1)
        r = routes[k]
        self.counts[r] += 1
        return self.fast if r == "fast" else self.primary

    def route_of(self, op: str, dtype: torch.dtype, nbytes: int) -> str:
        """``"primary"`` / ``"fast"`` for a message (no counting, no lazy class)."""
        routes = self.table.get((op, dtype))
        if routes is None:
            return "primary"
        k = next((i for i, s in enumerate(self.sizes) if nbytes <= s), len(self.sizes) - 1)
        return routes[k]

    def _add_class(self, size: int, pairs: Optional[List[Tuple[str, torch.dtype]]] = None,
                   why: str = "on first use") -> None:
        """A new size class, kept in ascending order: the (op, dtype) ``pairs`` (default: every one)
        calibrated at ``size``; the other pairs take the route of the next smaller class."""
        new = self._calibrate([size], self.iters, pairs)
        k = next((i for i, s in enumerate(self.sizes) if size < s), len(self.sizes))
        self.sizes.insert(k, size)
        for key, rs in self.table.items():
            rs.insert(k, new[key][0] if key in new else rs[max(k - 1, 0)])
        self.prepared_log.append({"MiB": size // MiB, "when": why,
                                  "routes": {f"{op} {str(dt).replace('torch.', '')}": r[0]
                                             for (op, dt), r in new.items()}})
        logger.info("routed comm: size class %d MiB added %s (rank %d): %s", size // MiB, why, self.rank,
                    self.prepared_log[-1]["routes"])

    def prepare(self, messages: Any) -> List[int]:
        """Calibrate, now, a size class for every message of ``messages`` -- ``(op, dtype, nbytes)``
        triples, the collectives an engine will send each step -- that is larger than every class,
        so no calibration runs inside a step.  COLLECTIVE: every rank passes the same messages
        (the engines derive them from the model structure, identical on every rank).  Returns the
        sizes of the classes added."""
        if not self.lazy_max:  # (fixed table / calibration off: nothing is ever timed)
            return []
        want: Dict[int, List[Tuple[str, torch.dtype]]] = {}
        for op, dt, n in messages:
            if op not in OPS or (op, dt) not in self.table or int(n) <= self.sizes[-1] or int(n) > self.lazy_max:
                continue
            gran = min(16 * MiB, max(4096, self.sizes[-1] // 4))  # (16 MiB past the default 64 MiB classes)
            size = -(-int(n) // gran) * gran
            if size in self.sizes:
                continue
            pairs = want.setdefault(size, [])
            if (op, dt) not in pairs:
                pairs.append((op, dt))
        added = []
        for size in sorted(want):
            self._add_class(size, sorted(want[size], key=lambda p: (p[0], str(p[1]))), why="at wrap")
            added.append(size)
        return added

    def alpha_beta(self, op: str = "all_reduce", dtype: torch.dtype = torch.bfloat16) -> Optional[Tuple[float, float]]:
        """``(alpha s, beta B/s)`` of ``t(S) = alpha + S / beta`` fitted over the calibration's timings of
        (op, dtype) -- per size class the time of the route the class takes (the MAX over the ranks, so
        every rank fits the same numbers and derives the same DDP bucket plan).  None without timings.
        parallel/flat.py ``bucket_caps_for`` sizes DDP's buckets from it."""
        from .flat import fit_alpha_beta

        routes = self.table.get((op, dtype))
        if routes is None:
            return None
        pts = []
        for s, r in zip(self.sizes, routes):
            t = self.timings.get(f"{op} {str(dtype).replace('torch.', '')} {s // MiB}MiB")
            if t is not None:
                pts.append((s, (t[1] if r == "fast" else t[0]) * 1e-6))
        return fit_alpha_beta(pts)

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

    def _calibrate(self, sizes: List[int], iters: int, pairs: Optional[List[Tuple[str, torch.dtype]]] = None
                   ) -> Dict[Tuple[str, torch.dtype], List[str]]:
        """Time every (op, dtype, size) (``pairs``: only those (op, dtype)) on both planes; per key the
        ranks agree (MAX of the times, MIN of the success flag) before the next key is timed, so a
        failure on one rank stops the timing of the fast plane on every rank at that key (no rank
        left waiting inside an IPC collective)."""
        pairs = pairs if pairs is not None else [(op, dt) for op in OPS for dt in DTYPES]
        keys = [(op, dt, s) for op, dt in pairs for s in sizes]
        table: Dict[Tuple[str, torch.dtype], List[str]] = {}
        dev = self.device if self.device.type == "cuda" else torch.device("cpu")
        for op, dt, s in keys:
            tp = tf = float("inf")
            ok = 0.0 if self.failed else 1.0
            if ok:
                try:
                    tp = self._time(self.primary, op, dt, s, iters)
                    tf = self._time(self.fast, op, dt, s, iters)
                except Exception as e:  # noqa: BLE001 - a failing route: every rank falls back to the primary
                    logger.warning("routed comm calibration failed on rank %d at %s %s %d MiB (%s); primary "
                                   "data plane only", self.rank, op, dt, s // MiB, e)
                    ok = 0.0
                    tp = tf = 0.0
            tt = torch.tensor([tp if ok else 0.0, tf if ok else 0.0, -ok], dtype=torch.float64, device=dev)
            self.primary.all_reduce(tt, "max")  # the slowest rank's times, and whether any rank failed
            tt = tt.cpu()
            if float(tt[2]) > -1.0:
                self.failed = True
            tpa, tfa = float(tt[0]), float(tt[1])
            self.timings[f"{op} {str(dt).replace('torch.', '')} {s // MiB}MiB"] = (round(tpa * 1e6, 1),
                                                                                    round(tfa * 1e6, 1))
            r = "fast" if (not self.failed and tfa < self.margin * tpa) else "primary"
            table.setdefault((op, dt), []).append(r)
        if self.failed:  # (a failure at a later key also retracts the fast routes of earlier keys)
            table = {k: ["primary"] * len(v) for k, v in table.items()}
        logger.info("routed comm table (rank %d): %s", self.rank, self.routes_from(table, sizes))
        return table

    def routes_from(self, table: Any, sizes: Optional[List[int]] = None) -> str:
        saved, self.table = getattr(self, "table", None), table
        saved_sizes = self.sizes
        if sizes is not None:
            self.sizes = list(sizes)
        try:
            return ", ".join(f"{k}: {v}" for k, v in self.routes().items())
        finally:
            self.sizes = saved_sizes
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
