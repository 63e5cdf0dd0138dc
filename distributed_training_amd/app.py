"""Application layer: config -> objects -> training (the Hydra ``main``).

Reference: ``load_train_objs`` (src/distributed_trainer.py:195-201),
``prepare_dataloader`` (:204-211) and ``main`` (:243-276).  ``main`` keeps the
reference flow and log lines (``"Training failed: ..."`` then re-raise;
``destroy_process_group`` in ``finally``).
"""
from __future__ import annotations

import logging
from typing import Any, Tuple

import torch
from torch.utils.data import Dataset

from .data.datasets import DeviceDataLoader, MyTrainDataset, SyntheticTokens
from .engine.trainer import Trainer, TrainingConfig
from .parallel.env import DistributedEnvironment
from .parallel.sampler import DistributedSampler
from .utils.logging_utils import setup_logging

logger = logging.getLogger("distributed_training_amd.trainer")


def _get(node: Any, key: str, default: Any = None) -> Any:
    if node is None:
        return default
    if hasattr(node, "get"):
        return node.get(key, default)
    return getattr(node, key, default)


_LM_NAMES = ("gpt2", "gpt2_small", "llama", "llama3", "llama3_8b")


def build_model(cfg_model: Any) -> torch.nn.Module:
    name = str(_get(cfg_model, "name", "") or "")
    if name in ("gpt2", "gpt2_small"):
        from .models.gpt2 import GPT2, GPT2Config

        return GPT2(GPT2Config.from_cfg(cfg_model))
    if name in ("llama", "llama3", "llama3_8b"):
        from .models.llama import Llama, LlamaConfig

        return Llama(LlamaConfig.from_cfg(cfg_model))
    from .models.mlp import build_mlp

    return build_mlp(cfg_model)


def build_optimizer(cfg_train: Any, params: Any) -> Any:
    from .ops.optim import build_optimizer as _b

    name = str(_get(cfg_train, "optimizer", "sgd"))
    lr = float(_get(cfg_train, "learning_rate", 1e-3))
    wd = float(_get(cfg_train, "weight_decay", 0.0) or 0.0)
    if name == "sgd":
        return _b("sgd", params, lr=lr, momentum=float(_get(cfg_train, "momentum", 0.0) or 0.0), weight_decay=wd)
    betas = tuple(_get(cfg_train, "betas", (0.9, 0.95)))
    return _b(name, params, lr=lr, betas=betas, weight_decay=wd)


def load_train_objs(cfg: Any) -> Tuple[Dataset, torch.nn.Module, torch.optim.Optimizer]:
    seed = _get(cfg.train, "seed", None)
    if seed is not None:
        torch.manual_seed(int(seed))
    name = str(_get(cfg.model, "name", "") or "")
    if name in _LM_NAMES and bool(_get(cfg.train, "meta_init", True)):
        # shapes only: the Trainer materialises on the device (DDP) or unit by unit into the shards
        # (FSDP) -- never 32 GB of fp32 per rank on the host at 8B (models/init.py)
        with torch.device("meta"):
            model = build_model(cfg.model)
    else:
        model = build_model(cfg.model)
    if hasattr(model, "vocab_size"):
        train_set = SyntheticTokens(int(cfg.train.dataset_size), int(_get(cfg.train, "seq_len", 1024)),
                                    model.vocab_size, seed=int(seed or 0))
    else:
        train_set = MyTrainDataset(cfg.train.dataset_size, int(_get(cfg.model, "input_size", 20)),
                                   int(_get(cfg.model, "output_size", 1)))
    optimizer = build_optimizer(cfg.train, model.parameters())
    return train_set, model, optimizer


def prepare_dataloader(dataset: Dataset, batch_size: int) -> DeviceDataLoader:
    return DeviceDataLoader(dataset, batch_size=batch_size, sampler=DistributedSampler(dataset))


def _wrap_policy(name: str, model: Any) -> Any:
    if not name:
        return None
    if name == "block":  # blocks + the model's extra units (Llama: embedding, output head)
        if getattr(model, "block_class", None) is None:
            return None
        from .parallel.fsdp import lm_wrap_policy

        return lm_wrap_policy(model)
    if name == "block_only":  # blocks only (embedding / head in the root unit)
        return getattr(model, "block_class", None) and {model.block_class}
    return None


def _mb(v: Any) -> Any:
    """Bucket size knob: a number of MiB, or "auto" / None (derived for xGMI)."""
    if v is None or str(v).lower() in ("auto", "none", "null"):
        return None if v is None or str(v).lower() in ("none", "null") else "auto"
    return float(v)


def training_config_from(cfg: Any, model: Any = None) -> TrainingConfig:
    t = cfg.train
    return TrainingConfig(
        max_epochs=t.total_epochs,
        save_every=t.save_every,
        batch_size=t.batch_size,
        learning_rate=t.learning_rate,
        snapshot_path=t.snapshot_path,
        device=_get(t, "device", "auto"),
        parallel_strategy=_get(t, "parallel_strategy", "ddp"),
        loss=_get(t, "loss", "cross_entropy"),
        fused_step=bool(_get(t, "fused_step", True)),
        graph_steps=int(_get(t, "graph_steps", 32)),
        bucket_cap_mb=_mb(_get(t, "bucket_cap_mb", "auto")),
        first_bucket_mb=_mb(_get(t, "first_bucket_mb", None)),
        mixed_precision=_get(t, "mixed_precision", None),
        fsdp_wrap=_wrap_policy(_get(t, "fsdp_wrap", None), model),
        log_throughput=bool(_get(t, "log_throughput", False)),
        grad_clip=_get(t, "grad_clip", None),
        save_optimizer=bool(_get(t, "save_optimizer", False)),
        desync_check_every=int(_get(t, "desync_check_every", 0) or 0),
        fault_injection=_get(t, "fault_injection", None),
        cpu_offload=bool(_get(t, "cpu_offload", False)),
        reduce_dtype=_get(t, "reduce_dtype", None),
        fsdp_sharding=str(_get(t, "fsdp_sharding", "full") or "full"),
        hybrid_shard_size=_get(t, "hybrid_shard_size", None),
        optimizer_in_backward=bool(_get(t, "optimizer_in_backward", False)),
        step_graph=bool(_get(t, "step_graph", False)),
    )


def estimate_peak_bytes(model: Any, cfg_train: Any, world_size: int, checkpointed: bool) -> int:
    """Per-rank training memory estimate (bytes): the optimizer state, the master and compute
    copies of the parameters and the gradients (all sharded under FSDP), the gathered units in
    flight (FSDP at world size > 1: the largest unit, twice -- the prefetch), and the activations
    of one micro-batch (the model's ``activation_bytes_per_token``).  An estimate for the
    ``activation_checkpointing: auto`` decision, not an allocator trace."""
    n = sum(p.numel() for p in model.parameters())
    mixed = str(_get(cfg_train, "mixed_precision", "") or "").lower() == "bf16"
    opt = str(_get(cfg_train, "optimizer", "sgd"))
    moments = 8 if opt in ("adam", "adamw") else (4 if float(_get(cfg_train, "momentum", 0) or 0) else 0)
    per_param = 4 + moments + (2 + 2 if mixed else 4)  # master + optimizer + compute copy + gradient
    fsdp = str(_get(cfg_train, "parallel_strategy", "ddp")).lower() == "fsdp"
    state = n * per_param // (world_size if fsdp else 1)
    if fsdp and world_size > 1:
        largest = max((sum(p.numel() for p in m.parameters()) for m in getattr(model, "layers", getattr(model, "h", []))),
                      default=0)
        vocab_unit = getattr(model, "vocab_size", 0) * getattr(getattr(model, "cfg", None), "n_embd", 0)
        state += 2 * max(largest, vocab_unit) * (2 if mixed else 4)
    tokens = int(_get(cfg_train, "batch_size", 1)) * int(_get(cfg_train, "seq_len", 1024))
    act = tokens * int(model.activation_bytes_per_token(checkpointed)) if hasattr(
        model, "activation_bytes_per_token") else 0
    return state + act


def activation_checkpointing_wanted(cfg: Any, model: Any, env: Any) -> bool:
    """``train.activation_checkpointing``: true / false, or ``auto`` -- on only when the estimated
    peak (:func:`estimate_peak_bytes`) without it exceeds 90 % of the device memory.  On a 288 GB
    MI355X the Llama-3 8B config needs none even at one rank (~168 GB), and checkpointing costs
    ~45 % of its throughput (the whole forward again)."""
    v = _get(cfg.train, "activation_checkpointing", False)
    if str(v).lower() != "auto":
        return bool(v)
    if not (getattr(env, "is_gpu", False) and torch.cuda.is_available()):
        return False
    total = torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory
    need = estimate_peak_bytes(model, cfg.train, int(getattr(env, "world_size", 1)), checkpointed=False)
    on = need > 0.9 * total
    logger.info(f"activation checkpointing auto: estimated peak {need / 2**30:.1f} GiB of "
                f"{total / 2**30:.1f} GiB -> {'on' if on else 'off'}")
    return on


def run(cfg: Any) -> Trainer:
    """Main training entry point (reference ``main`` body)."""
    env = None
    try:
        setup_logging(cfg)
        env = DistributedEnvironment(_get(cfg.train, "device", "auto"),
                                     timeout_s=_get(cfg.train, "timeout_s", None))
        env.setup()
        dataset, model, optimizer = load_train_objs(cfg)
        if hasattr(model, "enable_activation_checkpointing") and \
                activation_checkpointing_wanted(cfg, model, env):
            model.enable_activation_checkpointing()
        head_chunk = _get(cfg.train, "head_ce_chunk", None)
        if head_chunk is not None:  # LM head + CE in row blocks (ops/lm.py _ChunkedLinearCrossEntropy)
            from .ops import lm as _lm_ops
            _lm_ops.set_head_ce_chunk(int(head_chunk))
        train_config = training_config_from(cfg, model)
        train_data = prepare_dataloader(dataset, train_config.batch_size)
        trainer = Trainer(model, train_data, optimizer, train_config, env)
        trainer.train(train_config.max_epochs)
        return trainer
    except Exception as e:
        logger.error(f"Training failed: {str(e)}")
        raise
    finally:
        if torch.distributed.is_initialized():
            if env is not None:
                env.teardown()
            else:
                torch.distributed.destroy_process_group()
