"""Logging set-up (reference: ``setup_logging``, src/distributed_trainer.py:214-240).

Same behaviour and format: a file handler at ``cfg.logging.file`` plus a
stdout handler on the root logger, format
``"%(asctime)s | %(levelname)s | %(message)s"`` / ``"%Y-%m-%d %H:%M:%S"``,
level from ``cfg.logging.level``; the "Logging setup complete" line is
emitted twice like the reference (once before the handlers exist).
"""
from __future__ import annotations

import logging
import sys
from pathlib import Path
from typing import Any

logger = logging.getLogger("distributed_training_amd.trainer")

FORMAT = "%(asctime)s | %(levelname)s | %(message)s"
DATEFMT = "%Y-%m-%d %H:%M:%S"


def setup_logging(cfg: Any) -> None:
    """Configure logging to write to both file and console."""
    logging.basicConfig(level=logging.INFO)
    logger.info(f"Logging setup complete. Log file: {cfg.logging.file}")
    log_file = Path(cfg.logging.file)
    log_file.parent.mkdir(parents=True, exist_ok=True)
    formatter = logging.Formatter(FORMAT, datefmt=DATEFMT)
    file_handler = logging.FileHandler(log_file)
    file_handler.setFormatter(formatter)
    console_handler = logging.StreamHandler(sys.stdout)
    console_handler.setFormatter(formatter)
    root_logger = logging.getLogger()
    root_logger.setLevel(cfg.logging.level)
    root_logger.addHandler(file_handler)
    root_logger.addHandler(console_handler)
    logger.info(f"Logging setup complete. Log file: {log_file}")
