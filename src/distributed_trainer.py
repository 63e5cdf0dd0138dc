"""Reference-compatible training entrypoint (reference: src/distributed_trainer.py).

Same public names and signatures: ``TrainingConfig``,
``DistributedEnvironment``, ``ModelCheckpoint``, ``Trainer``,
``load_train_objs``, ``prepare_dataloader``, ``setup_logging``, ``main``.
``main`` is decorated with a Hydra-compatible loader (no hydra dependency):

    torchrun --nproc_per_node=8 src/distributed_trainer.py model=mlp2 train=mlp2_bf16
"""
import logging
import os
import sys
from typing import Any

if __package__ in (None, ""):  # executed as a script by torchrun
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_training_amd.app import load_train_objs, prepare_dataloader, run  # noqa: E402
from distributed_training_amd.config import main_decorator  # noqa: E402
from distributed_training_amd.engine.checkpoint import ModelCheckpoint  # noqa: E402
from distributed_training_amd.engine.trainer import Trainer, TrainingConfig  # noqa: E402
from distributed_training_amd.parallel.env import DistributedEnvironment  # noqa: E402
from distributed_training_amd.utils.logging_utils import setup_logging  # noqa: E402

logging.basicConfig(level=logging.INFO)
logger = logging.getLogger(__name__)

__all__ = ["TrainingConfig", "DistributedEnvironment", "ModelCheckpoint", "Trainer", "load_train_objs",
           "prepare_dataloader", "setup_logging", "main"]


@main_decorator(config_path="../conf", config_name="config", version_base=None)
def main(cfg: Any) -> None:
    """Main training entry point."""
    run(cfg)


if __name__ == "__main__":
    main()
