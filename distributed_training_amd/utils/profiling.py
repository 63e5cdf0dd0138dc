"""Tracing helpers: roctx ranges + HIP-event step timer.

``roctx`` ranges (``libroctx64``, resolved at run time with ctypes) mark step
phases so ``rocprofv3 --marker-trace`` timelines show forward / backward /
all-reduce / optimizer; without the library the ranges are no-ops.  The
reference has no tracing at all.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from typing import Any, Dict, List, Optional

import torch

_roctx = None


def _load_roctx() -> Any:
    global _roctx
    if _roctx is not None:
        return _roctx if _roctx else None
    # rocprofiler-sdk's roctx first: rocprofv3 --marker-trace intercepts that one
    for name in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so",
                 "libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            return lib
        except OSError:
            continue
    _roctx = False
    return None


_ENABLED: Optional[bool] = None


def enabled() -> bool:
    """``DTA_ROCTX=1`` and libroctx64 loadable (read once per process: the ranges sit on
    per-bucket / per-unit hot paths, so a disabled range costs one global lookup)."""
    global _ENABLED
    if _ENABLED is None:
        _ENABLED = os.environ.get("DTA_ROCTX", "0") == "1" and _load_roctx() is not None
    return _ENABLED


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on) and _load_roctx() is not None


class _Range:
    __slots__ = ("name",)

    def __init__(self, name: str) -> None:
        self.name = name

    def __enter__(self) -> Any:
        _roctx.roctxRangePushA(self.name.encode())
        return self

    def __exit__(self, *exc: Any) -> None:
        _roctx.roctxRangePop()
        return False


_NULL = contextlib.nullcontext()


def range_(name: str) -> Any:
    """Context manager: a named roctx range around host work (enqueue of kernels /
    collectives); a shared no-op context when tracing is off."""
    return _Range(name) if enabled() else _NULL


def push(name: str) -> None:
    if enabled():
        _roctx.roctxRangePushA(name.encode())


def pop() -> None:
    if enabled():
        _roctx.roctxRangePop()


def mark(name: str) -> None:
    if enabled():
        _roctx.roctxMarkA(name.encode())


class StepTimer:
    """Wall-clock step timer with device synchronisation at the boundaries."""

    def __init__(self, device: Optional[torch.device] = None) -> None:
        self.device = device
        self.times: List[float] = []
        self._t0 = None

    def _sync(self) -> None:
        if self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def start(self) -> None:
        self._sync()
        self._t0 = time.perf_counter()

    def stop(self, n_steps: int = 1) -> float:
        self._sync()
        dt = time.perf_counter() - self._t0
        self.times.append(dt / max(1, n_steps))
        return dt

    def summary(self) -> Dict[str, float]:
        if not self.times:
            return {}
        ts = sorted(self.times)
        return {"mean_s": sum(ts) / len(ts), "median_s": ts[len(ts) // 2], "min_s": ts[0]}
