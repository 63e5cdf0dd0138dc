"""Deferred ("meta") initialisation of the transformer models.

The reference builds its model on the host and moves it (``load_train_objs`` +
``model.to(device)``, src/distributed_trainer.py:195-201,137-138).  At Llama-3 8B that is
32 GB of fp32 per rank initialised single-threaded on the host (256 GB across an 8-GPU
node) before FSDP shards it.  Here the LM configs are built on the ``meta`` device
(shapes only) and materialised where they live:

* DDP: :func:`materialize_` -- ``to_empty`` on the GPU, then every parameter initialised
  on the device (the engine broadcasts rank 0's copy at wrap time anyway);
* FSDP: the engine calls :func:`init_param_` per unit into its flat fp32 staging buffer
  on the GPU (rank 0 only when the unit is broadcast from rank 0), keeps this rank's
  shard and frees the unit -- the full model never exists on the host, and on the
  device only one unit at a time (parallel/fsdp.py).

Each parameter draws from its own generator, seeded by (process seed, parameter
name): the initial model is the same whatever the world size, wrap policy or
materialisation order.  Models opt in by defining ``init_param(name, tensor,
generator)`` (and ``init_buffers(device)`` for non-persistent buffers such as RoPE tables).
"""
from __future__ import annotations

import zlib
from typing import Any, Optional

import torch
import torch.nn as nn


def is_meta(module: nn.Module) -> bool:
    """Any parameter or buffer of ``module`` still on the meta device."""
    return any(t.is_meta for t in module.parameters()) or any(b.is_meta for b in module.buffers())


def supports_meta_init(module: nn.Module) -> bool:
    return callable(getattr(module, "init_param", None))


def _generator(device: torch.device, name: str, base_seed: Optional[int]) -> torch.Generator:
    base = torch.initial_seed() if base_seed is None else int(base_seed)
    g = torch.Generator(device=device)
    g.manual_seed((base * 1_000_003 + zlib.crc32(name.encode())) % (1 << 62))
    return g


@torch.no_grad()
def init_param_(model: nn.Module, name: str, t: torch.Tensor, base_seed: Optional[int] = None) -> None:
    """Initialise ``t`` (any device, any dtype) as parameter ``name`` of ``model``."""
    fn = getattr(model, "init_param", None)
    if fn is None:
        raise RuntimeError(f"{type(model).__name__} has no init_param: cannot materialise meta parameter {name}")
    if t.dtype == torch.float32:
        fn(name, t, _generator(t.device, name, base_seed))
    else:  # (draw in fp32, as a host-built model converted afterwards would hold)
        tmp = torch.empty(t.shape, dtype=torch.float32, device=t.device)
        fn(name, tmp, _generator(t.device, name, base_seed))
        t.copy_(tmp)


@torch.no_grad()
def init_buffers_(model: nn.Module, device: torch.device) -> None:
    """Buffers onto ``device``: recomputed by the model's ``init_buffers`` when it has one (after
    ``to_empty`` their values are garbage), else moved (meta buffers without it are an error)."""
    fn = getattr(model, "init_buffers", None)
    if fn is not None:
        fn(device)
        return
    for m in model.modules():
        for k, b in m._buffers.items():
            if b is None:
                continue
            if b.is_meta:
                raise RuntimeError(f"{type(model).__name__} has meta buffers but no init_buffers")
            m._buffers[k] = b.to(device)


@torch.no_grad()
def materialize_(model: nn.Module, device: Any, base_seed: Optional[int] = None) -> nn.Module:
    """Allocate every meta parameter / buffer of ``model`` on ``device`` and initialise it there.

    Each Parameter OBJECT is materialised in place (``torch.utils.swap_tensors``: same Python object,
    new device storage), once however many modules hold it -- so tied weights stay tied (GPT-2's
    ``lm_head.weight is wte.weight``) and an optimizer built over the meta model stays valid.
    ``nn.Module.to_empty`` would instead give every owning module a NEW Parameter (a meta tensor
    cannot take a device tensor through ``.data``): the tie silently broken, the head trained as a
    second [V, C] matrix (GPT-2 at the entrypoint: 163 M parameters instead of 124 M)."""
    device = torch.device(device)
    done = set()
    for name, p in model.named_parameters():  # (deduplicated: a tied weight appears once, first owner's name)
        if id(p) in done:
            continue
        done.add(id(p))
        if p.is_meta:
            torch.utils.swap_tensors(p, nn.Parameter(torch.empty_like(p, device=device), requires_grad=p.requires_grad))
            init_param_(model, name, p.data, base_seed)
    for m in model.modules():  # (buffers: moved / recomputed below; meta ones get device storage first)
        for k, b in m._buffers.items():
            if b is not None and b.is_meta:
                m._buffers[k] = torch.empty_like(b, device=device)
    init_buffers_(model, device)
    return model
