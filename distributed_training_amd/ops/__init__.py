"""Native op layer: loads the in-tree ``_C`` extension (gfx950 HIP kernels +
RCCL communicator).

Policy (no silent fallback on the GPU): GPU tensors are ALWAYS processed by
the HIP kernels.  If the extension is missing while a GPU is visible,
:func:`native` raises.  CPU tensors (the gloo plumbing path and unit tests on
hosts without a GPU) are handled by plain PyTorch reference math in the
individual op modules.
"""
from __future__ import annotations

import importlib
import os
from pathlib import Path
from typing import Any, Optional

_native: Optional[Any] = None
_native_err: Optional[BaseException] = None


def _try_import() -> None:
    global _native, _native_err
    if _native is not None or _native_err is not None:
        return
    try:
        _native = importlib.import_module("distributed_training_amd._C")
    except BaseException as e:  # noqa: BLE001 - remember the reason for the error message
        _native_err = e


def has_native() -> bool:
    _try_import()
    return _native is not None


def native() -> Any:
    """Return the ``_C`` module or raise a descriptive error."""
    _try_import()
    if _native is None:
        raise RuntimeError(
            "distributed_training_amd native extension (_C) is not built or failed to load: "
            f"{_native_err!r}. Build it with `python -m distributed_training_amd.ops._build` "
            "(hipcc --offload-arch=gfx950)."
        )
    return _native


_rccl_ready = False


def ensure_rccl() -> Any:
    """Resolve the RCCL API from the librccl.so PyTorch ships (one RCCL runtime
    per process)."""
    global _rccl_ready
    C = native()
    if _rccl_ready or C.rccl_loaded():
        _rccl_ready = True
        return C
    import torch

    cands = [
        os.environ.get("DTA_RCCL_LIB", ""),
        str(Path(torch.__file__).resolve().parent / "lib" / "librccl.so"),
        "/opt/rocm/lib/librccl.so",
    ]
    errs = []
    for c in cands:
        if not c or not Path(c).exists():
            continue
        err = C.rccl_load(c)
        if not err:
            _rccl_ready = True
            return C
        errs.append(f"{c}: {err}")
    raise RuntimeError("could not load librccl: " + "; ".join(errs or ["no candidate found"]))


def stream_handle(stream: Any = None) -> int:
    """HIP stream handle for a torch stream (-1 = current torch stream)."""
    if stream is None:
        return -1
    return int(stream.cuda_stream)
