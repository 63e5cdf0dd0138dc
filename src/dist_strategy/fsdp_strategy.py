"""``FSDPStrategy(is_gpu)`` (reference: src/dist_strategy/fsdp_strategy.py:13-46),
backed by the native FSDP engine (flat shards, RCCL all-gather / reduce-scatter)."""
from distributed_training_amd.parallel.strategy import FSDPStrategy

__all__ = ["FSDPStrategy"]
