"""Reference-compatible data module (reference: src/data_utils.py:7-16).

``MyTrainDataset(size)`` -> ``(Tensor[20], Tensor[1])`` samples; backed by the
framework's contiguous, device-uploadable implementation.
"""
from distributed_training_amd.data.datasets import MyTrainDataset

__all__ = ["MyTrainDataset"]
