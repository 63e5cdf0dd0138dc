"""Data parallelism from scratch -- the educational playground.

Reference: src/playground/ddp_script.py: a Linear(10, 1)
model, a seeded ``randn`` dataset, ``torch.multiprocessing.spawn`` of
``--world-size`` workers, an explicit parameter broadcast from rank 0, and a
per-parameter gradient all-reduce + divide after ``backward()`` with
per-rank logs of every parameter's gradient / weight norm.

Same command line and log lines.  The collectives go through the framework's
communicator layer (``parallel/comm.py``): RCCL on GPU (each rank its own
MI355X), gloo on CPU.  ``--bucketed`` switches the per-parameter all-reduces
for ONE all-reduce over a flat gradient buffer (what the real DDP engine does)
so the two can be compared.

    python src/playground/ddp_script.py --world-size 2 --epochs 2 --num-workers 0
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
from pathlib import Path
from typing import Any, List, Tuple

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
from torch.utils.data import DataLoader, Dataset
from torch.utils.data.distributed import DistributedSampler

ROOT = Path(__file__).resolve().parents[2]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


class SimpleModel(nn.Module):
    def __init__(self) -> None:
        super().__init__()
        self.linear = nn.Linear(10, 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.linear(x)


class DummyDataset(Dataset):
    def __init__(self, size: int = 1000) -> None:
        self.size = size
        self.data = torch.randn(size, 10)
        self.labels = torch.randn(size, 1)

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.data[idx], self.labels[idx]


def rank_logger(rank: int, log_dir: str = "logs") -> logging.Logger:
    """One log file per rank (``<log_dir>/ddp_rank_<rank>.log``) + console."""
    Path(log_dir).mkdir(parents=True, exist_ok=True)
    logger = logging.getLogger(f"ddp_trainer_{rank}")
    logger.setLevel(logging.INFO)
    logger.propagate = False
    fmt = logging.Formatter("%(asctime)s - Rank %(rank)s - %(levelname)s - %(message)s",
                            datefmt="%Y-%m-%d %H:%M:%S")
    for h in (logging.FileHandler(str(Path(log_dir) / f"ddp_rank_{rank}.log")), logging.StreamHandler(sys.stdout)):
        h.setLevel(logging.INFO)
        h.setFormatter(fmt)
        logger.addHandler(h)
    return logger


class ManualDDP:
    """What DistributedDataParallel does, spelled out (no hooks, no overlap)."""

    def __init__(self, model: nn.Module, comm: Any, world_size: int, bucketed: bool = False) -> None:
        self.model = model
        self.comm = comm
        self.world_size = world_size
        self.bucketed = bucketed

    @torch.no_grad()
    def broadcast_parameters(self) -> None:
        for p in self.model.parameters():
            self.comm.broadcast(p.data, src=0)

    @torch.no_grad()
    def allreduce_gradients(self) -> None:
        params: List[nn.Parameter] = [p for p in self.model.parameters() if p.grad is not None]
        if self.bucketed:
            flat = torch.cat([p.grad.reshape(-1) for p in params])
            self.comm.all_reduce(flat, op="sum")
            flat /= self.world_size
            off = 0
            for p in params:
                n = p.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n
        else:
            for p in params:
                self.comm.all_reduce(p.grad, op="sum")
                p.grad /= self.world_size


def setup(rank: int, world_size: int, backend: str, addr: str, port: int) -> torch.device:
    os.environ["MASTER_ADDR"] = addr
    os.environ["MASTER_PORT"] = str(port)
    if torch.cuda.is_available() and backend == "nccl":
        torch.cuda.set_device(rank)
        device = torch.device("cuda", rank)
        dist.init_process_group("nccl", rank=rank, world_size=world_size, device_id=device)
    else:
        device = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world_size)
    return device


def train(rank: int, world_size: int, args: argparse.Namespace) -> None:
    logger = rank_logger(rank, args.log_dir)
    extra = {"rank": rank}
    torch.manual_seed(42)  # identical data + model on every rank
    device = setup(rank, world_size, args.backend, args.master_addr, args.port)
    from distributed_training_amd.parallel.comm import make_comm

    comm = make_comm(device)
    model = SimpleModel().to(device)
    ddp = ManualDDP(model, comm, world_size, bucketed=args.bucketed)
    ddp.broadcast_parameters()
    dataset = DummyDataset()
    sampler = DistributedSampler(dataset, num_replicas=world_size, rank=rank)
    loader = DataLoader(dataset, batch_size=args.batch_size, sampler=sampler, num_workers=args.num_workers)
    optimizer = torch.optim.SGD(model.parameters(), lr=args.learning_rate)
    criterion = nn.MSELoss()
    model.train()
    for epoch in range(args.epochs):
        sampler.set_epoch(epoch)
        total_loss = 0.0
        for batch_idx, (data, target) in enumerate(loader):
            data, target = data.to(device), target.to(device)
            optimizer.zero_grad()
            loss = criterion(model(data), target)
            loss.backward()
            ddp.allreduce_gradients()
            for name, param in model.named_parameters():
                logger.info(f"Epoch {epoch} - Parameter: {name}, Gradient: {torch.norm(param.grad)}", extra=extra)
                logger.info(f"Epoch {epoch} - Parameter: {name}, Weight: {torch.norm(param.data)}", extra=extra)
            optimizer.step()
            total_loss += loss.item()
            if batch_idx % args.log_interval == 0 and rank == 0:
                logger.info(f"Epoch: {epoch}, Batch: {batch_idx}, Loss: {loss.item():.6f}", extra=extra)
        if rank == 0:
            logger.info(f"Epoch: {epoch}, Average Loss: {total_loss / len(loader):.6f}", extra=extra)
    if hasattr(comm, "destroy"):
        comm.destroy()
    dist.destroy_process_group()


def get_argument_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="PyTorch DDP Training")
    p.add_argument("--batch-size", type=int, default=32, help="input batch size for training (default: 32)")
    p.add_argument("--epochs", type=int, default=10, help="number of epochs to train (default: 10)")
    p.add_argument("--learning-rate", type=float, default=0.01, help="learning rate (default: 0.01)")
    p.add_argument("--num-workers", type=int, default=4, help="data loading workers (default: 4)")
    p.add_argument("--backend", type=str, default="nccl", help="nccl (= RCCL on ROCm) or gloo (default: nccl)")
    p.add_argument("--log-interval", type=int, default=10, help="batches between loss logs")
    p.add_argument("--world-size", type=int,
                   default=torch.cuda.device_count() if torch.cuda.is_available() else 4,
                   help="number of processes for distributed training")
    p.add_argument("--log-dir", type=str, default="logs", help="directory to store log files (default: logs)")
    p.add_argument("--master-addr", type=str, default="127.0.0.1")
    p.add_argument("--port", type=int, default=12355)
    p.add_argument("--bucketed", action="store_true", help="one flat all-reduce instead of one per parameter")
    return p


def main(argv: Any = None) -> None:
    args = get_argument_parser().parse_args(argv)
    if not torch.cuda.is_available() and args.backend == "nccl":
        args.backend = "gloo"
    where = f"{args.world_size} GPUs" if args.backend == "nccl" else f"CPU with {args.world_size} processes"
    logging.basicConfig(level=logging.INFO)
    logging.info(f"Training on {where}")
    mp.spawn(train, args=(args.world_size, args), nprocs=args.world_size, join=True)


if __name__ == "__main__":
    main()
