"""Legacy torchrun entrypoint documented by the reference (README.md:57-61,89)
and launched by its cloud-init (cloud-init.tftpl:67,77) but missing from the
reference snapshot.

    torchrun --nnodes=N --node_rank=i --master_addr=A --master_port=29500 \\
        --nproc_per_node=8 src/multigpu_multi_node.py [EPOCHS] [SAVE_FREQUENCY] \\
        [--batch_size B] [key=value ...]

Positional ``EPOCHS``/``SAVE_FREQUENCY`` map to ``train.total_epochs`` /
``train.save_every``, ``--batch_size`` to ``train.batch_size`` (per GPU);
any Hydra-style ``key=value`` overrides are forwarded.  With no arguments it
trains the default config (what the cloud-init launcher does).
"""
import argparse
import os
import sys
from typing import Any

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_training_amd.config import compose, prepare_run_dir, split_argv  # noqa: E402

CONF_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conf")


def parse(argv: Any = None) -> Any:
    argv = list(sys.argv[1:] if argv is None else argv)
    overrides, rest = split_argv(argv)
    ap = argparse.ArgumentParser(description="simple distributed training job")
    ap.add_argument("total_epochs", nargs="?", type=int, help="Total epochs to train the model")
    ap.add_argument("save_every", nargs="?", type=int, help="How often to save a snapshot")
    ap.add_argument("--batch_size", "--batch-size", type=int, default=None,
                    help="Input batch size on each device (default: 32)")
    args = ap.parse_args(rest)
    if args.total_epochs is not None:
        overrides.append(f"train.total_epochs={args.total_epochs}")
    if args.save_every is not None:
        overrides.append(f"train.save_every={args.save_every}")
    if args.batch_size is not None:
        overrides.append(f"train.batch_size={args.batch_size}")
    return overrides


def main(argv: Any = None) -> Any:
    from distributed_training_amd.app import run

    overrides = parse(argv)
    cfg = compose(CONF_DIR, "config", overrides, runtime={"cwd": os.getcwd(), "config_dir": CONF_DIR})
    prepare_run_dir(cfg)
    return run(cfg)


if __name__ == "__main__":
    main()
