"""``DDPStrategy(local_rank, is_gpu)`` (reference: src/dist_strategy/ddp_strategy.py:10-32),
backed by the native DDP engine (flat gradient buckets, RCCL all-reduce over xGMI)."""
from distributed_training_amd.parallel.strategy import DDPStrategy

__all__ = ["DDPStrategy"]
