"""Strategy ABC (reference: src/dist_strategy/dist_strategy.py:8-26)."""
from distributed_training_amd.parallel.strategy import DistributedStrategy

__all__ = ["DistributedStrategy"]
