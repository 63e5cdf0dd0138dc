#!/usr/bin/env python3
"""Headline benchmark: samples/sec (whole node) of the 2-layer MLP DDP bf16
training step, weak scaling (32 samples per GPU per step), on N GPUs.

    python bench.py                                   # N=1
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Config (BASELINE.json "2-layer MLP DDP bf16"): model Linear(20,512)-ReLU-
Linear(512,1), random init; synthetic data = the reference's MyTrainDataset
(2048 samples of rand(20), rand(1)) with DistributedSampler order; batch 32
per GPU; SGD lr 1e-3; MSE loss (the reference's cross-entropy on a 1-wide
output is identically zero).  Every timed step does the full
work: gather, forward, loss, backward, gradient exchange, SGD update.  The
exchange: at N > 1 the persistent program's in-kernel all-reduce of the 1 / N
pre-scaled gradients over xGMI peer memory (or RCCL, whichever form the
start-up calibration measured faster: "step_form" in the JSON); at N = 1 there
is no peer and the persistent program runs no exchange (an all-reduce over one
rank is the identity; torch's DDP at world size 1 still launches one -- so does
this program's per-step form, DTA_MLP_PERSISTENT=0, with ``--allreduce-world1 1``).
bf16 = MFMA operand precision (fp32 accumulate, fp32 master weights).

``--impl fused`` (default): this framework's fused gfx950 step program.
``--impl generic``: this framework's generic engine (autograd + native DDP
buckets + fused SGD) on the same model.
``--impl torch``: stock PyTorch-ROCm running the reference's loop (torch DDP,
DataLoader(pin_memory) + DistributedSampler, torch.optim.SGD, bf16 autocast)
-- the comparison baseline recorded in bench_baseline.json.

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path
from typing import TYPE_CHECKING, Any, Callable, Optional, Tuple

if TYPE_CHECKING:  # annotations only: torch is imported inside the functions (fast --help)
    import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "samples/sec (whole node) + DDP scaling efficiency, toy MLP at 1/2/4/8 MI355X"
# (step_fn(n): run n steps, finish(): last loss, the communicator or None)
Runner = Tuple[Callable[[int], None], Callable[[], float], Optional[object]]


def parse() -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2048)
    ap.add_argument("--warmup", type=int, default=256)
    ap.add_argument("--impl", choices=["fused", "generic", "torch"], default="fused")
    ap.add_argument("--model", choices=["mlp2", "linear"], default="mlp2",
                    help="linear: the reference's default nn.Linear(20, 1) + cross-entropy, fp32 (not the headline)")
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--batch", type=int, default=32, help="per-GPU batch")
    ap.add_argument("--dataset-size", type=int, default=2048)
    ap.add_argument("--graph-steps", type=int, default=32)
    ap.add_argument("--own-tiles", type=int, default=0)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--no-amp", action="store_true", help="--impl torch: fp32 like the reference code")
    ap.add_argument("--allreduce-world1", type=int, default=1)
    ap.add_argument("--json-out", type=str, default="")
    return ap.parse_args()


def setup_dist(args: argparse.Namespace) -> Tuple[int, int, "torch.device"]:
    import torch
    import torch.distributed as dist

    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from distributed_training_amd.parallel.ipc import device_index, dist_backend, shared_gpu

    if ws != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={ws}")
    # one rank per GPU (RCCL); DTA_SHARED_GPU=1 rehearses N ranks on fewer GPUs
    # (gloo control plane + IPC data plane; the numbers are then not a scaling result)
    dev = torch.device("cuda", device_index(local))
    torch.cuda.set_device(dev)
    if ws > 1:
        backend = dist_backend(True)
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))
    args.shared_gpu = shared_gpu() and ws > 1
    return rank, ws, dev


def build(args: argparse.Namespace, dev: "torch.device", ws: int) -> Tuple[Any, "torch.nn.Module", Any]:
    import torch

    from distributed_training_amd.data.datasets import DeviceDataLoader, MyTrainDataset
    from distributed_training_amd.models.mlp import MLP
    from distributed_training_amd.parallel.sampler import DistributedSampler

    torch.manual_seed(0)
    ds = MyTrainDataset(args.dataset_size, 20, 1, seed=0)
    model = MLP(20, args.hidden, 1, activation="relu").to(dev)
    rank = int(os.environ.get("RANK", "0"))
    loader = DeviceDataLoader(ds, args.batch, sampler=DistributedSampler(ds, num_replicas=ws, rank=rank), device=dev)
    return ds, model, loader


def bench_comm(dev: "torch.device") -> Any:
    """The step's communicator (``make_comm``: native RCCL at N > 1).  A native communicator that cannot come up
    on every rank (librccl not loadable, init refused) falls back to torch.distributed's own process group --
    RCCL through c10d -- so the run still yields its number; the JSON's ``comm`` says which one ran."""
    import torch.distributed as dist

    from distributed_training_amd.parallel.comm import TorchComm, make_comm

    try:
        return make_comm(dev)
    except Exception as e:  # noqa: BLE001 - load / init failures are raised on every rank alike
        if not dist.is_initialized() or dist.get_world_size() == 1:
            raise
        print(f"[bench] native communicator unavailable ({e}); torch.distributed used", file=sys.stderr)
        return TorchComm(device=dev)


def run_fused(args: argparse.Namespace, dev: "torch.device", ws: int) -> "Runner":
    import torch

    from distributed_training_amd.engine.fused_mlp import FusedMLPProgram, fused_eligible
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    ds, model, loader = build(args, dev, ws)
    comm = bench_comm(dev)
    ddp = DistributedDataParallel(model, comm=comm, device=dev)
    opt = FusedSGD(ddp.parameters(), lr=args.lr)
    why = fused_eligible(model, opt, loader, "mse", dev)
    if why:
        raise SystemExit(f"fused path not applicable: {why}")
    prog = FusedMLPProgram(model, opt, loader, comm, loss="mse", graph_steps=args.graph_steps,
                           own_tiles=args.own_tiles or None, allreduce_world1=bool(args.allreduce_world1))

    def step_fn(n: int) -> None:
        prog.run_steps(n)

    def finish() -> float:
        prog.store_to_module()
        return float(prog.last_losses(1)[0].item()) if prog.launched else float("nan")

    # which DDP step form ran (persistent loop + in-kernel exchange, or per-step
    # kernel + all-reduce), and the per-form calibration times when ranks > 1
    form = ("persistent" + (f"/{prog.xmode}" if ws > 1 else "")) if prog.persistent else "per-step"
    finish.info = {"step_form": form,
                   "calibration_ms": getattr(prog, "exchange_times_ms", None)}
    return step_fn, finish, comm


def run_fused_linear(args: argparse.Namespace, dev: "torch.device", ws: int) -> "Runner":
    """The reference's default workload (src/distributed_trainer.py:160-165, 199-200):
    nn.Linear(20, 1), F.cross_entropy on float targets, fp32, SGD, DDP -- on the fused
    Linear step program (csrc/linear_step.hip)."""
    import torch

    from distributed_training_amd.data.datasets import DeviceDataLoader, MyTrainDataset
    from distributed_training_amd.engine.fused_linear import FusedLinearProgram, linear_eligible
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.sampler import DistributedSampler

    torch.manual_seed(0)
    ds = MyTrainDataset(args.dataset_size, 20, 1, seed=0)
    model = torch.nn.Linear(20, 1).to(dev)
    rank = int(os.environ.get("RANK", "0"))
    loader = DeviceDataLoader(ds, args.batch, sampler=DistributedSampler(ds, num_replicas=ws, rank=rank), device=dev)
    comm = bench_comm(dev)
    ddp = DistributedDataParallel(model, comm=comm, device=dev)
    opt = FusedSGD(ddp.parameters(), lr=args.lr)
    why = linear_eligible(model, opt, loader, "cross_entropy", dev)
    if why:
        raise SystemExit(f"fused Linear path not applicable: {why}")
    prog = FusedLinearProgram(model, opt, loader, comm, loss="cross_entropy")

    def step_fn(n: int) -> None:
        prog.run_steps(n)

    def finish() -> float:
        prog.store_to_module()
        return float(prog.last_losses(1)[0].item()) if prog.launched else float("nan")

    finish.info = {"step_form": "persistent" if ws == 1 else "per-step graph"}
    return step_fn, finish, comm


def run_generic(args: argparse.Namespace, dev: "torch.device", ws: int) -> "Runner":
    import torch
    import torch.nn.functional as F

    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    ds, model, loader = build(args, dev, ws)
    comm = bench_comm(dev)
    ddp = DistributedDataParallel(model, comm=comm, device=dev)
    opt = FusedSGD(ddp.parameters(), lr=args.lr)
    state = {"it": None, "epoch": 0, "loss": None}

    def next_batch() -> Tuple["torch.Tensor", "torch.Tensor"]:
        while True:
            if state["it"] is None:
                loader.sampler.set_epoch(state["epoch"])
                state["it"] = iter(loader)
            try:
                return next(state["it"])
            except StopIteration:
                state["it"] = None
                state["epoch"] += 1

    def step_fn(n: int) -> None:
        for _ in range(n):
            x, y = next_batch()
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = ddp(x)
            loss = F.mse_loss(out.float(), y)
            loss.backward()
            opt.step()
            state["loss"] = loss

    def finish() -> float:
        return float(state["loss"].item()) if state["loss"] is not None else float("nan")

    return step_fn, finish, comm


def run_torch(args: argparse.Namespace, dev: "torch.device", ws: int) -> "Runner":
    """Stock PyTorch-ROCm with the reference's loop (src/distributed_trainer.py:160-183)."""
    import torch
    import torch.nn.functional as F
    from torch.nn.parallel import DistributedDataParallel as DDP
    from torch.utils.data import DataLoader
    from torch.utils.data.distributed import DistributedSampler

    from distributed_training_amd.data.datasets import MyTrainDataset

    torch.manual_seed(0)
    ds = MyTrainDataset(args.dataset_size, 20, 1, seed=0)
    model = torch.nn.Sequential(torch.nn.Linear(20, args.hidden), torch.nn.ReLU(),
                                torch.nn.Linear(args.hidden, 1)).to(dev)
    if ws > 1:
        model = DDP(model, device_ids=[dev.index])
    opt = torch.optim.SGD(model.parameters(), lr=args.lr)
    sampler = DistributedSampler(ds, num_replicas=ws, rank=int(os.environ.get("RANK", "0")))
    loader = DataLoader(ds, batch_size=args.batch, pin_memory=True, shuffle=False, sampler=sampler)
    state = {"it": None, "epoch": 0, "loss": None}

    def next_batch() -> Tuple["torch.Tensor", "torch.Tensor"]:
        while True:
            if state["it"] is None:
                sampler.set_epoch(state["epoch"])
                state["it"] = iter(loader)
            try:
                return next(state["it"])
            except StopIteration:
                state["it"] = None
                state["epoch"] += 1

    def step_fn(n: int) -> None:
        for _ in range(n):
            x, y = next_batch()
            x = x.to(dev)
            y = y.to(dev)
            opt.zero_grad()
            if args.no_amp:
                out = model(x)
            else:
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = model(x)
            loss = F.mse_loss(out.float(), y)
            loss.backward()
            opt.step()
            state["loss"] = loss

    def finish() -> float:
        return float(state["loss"].item()) if state["loss"] is not None else float("nan")

    return step_fn, finish, None


def main() -> None:
    args = parse()
    import torch
    import torch.distributed as dist

    rank, ws, dev = setup_dist(args)
    runner = {"fused": run_fused, "generic": run_generic, "torch": run_torch}[args.impl]
    if args.model == "linear":
        if args.impl != "fused":
            raise SystemExit("--model linear: only --impl fused")
        runner = run_fused_linear
    step_fn, finish, comm = runner(args, dev, ws)

    def dbarrier() -> None:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[dev.index])
        else:
            dist.barrier()

    def barrier() -> None:
        torch.cuda.synchronize(dev)
        if ws > 1:  # (one rank: the synchronize is the whole bracket; a second one is host time in the timed region)
            dbarrier()
            torch.cuda.synchronize(dev)

    # Closing bracket at ws > 1: the communicator's own barrier when it has one -- a
    # device all-reduce of one element on its stream, ordered after this rank's steps,
    # then a synchronize (one-shot IPC push over xGMI on a node, RCCL otherwise): a
    # real barrier (no rank returns before every rank has finished its steps) without
    # torch.distributed.barrier's host-side launch and bookkeeping in the timed region.
    fast = getattr(comm, "barrier", None) if ws > 1 and comm is not None else None

    def end_barrier() -> None:
        if fast is None:
            barrier()
            return
        torch.cuda.synchronize(dev)
        fast()

    step_fn(args.warmup)
    barrier()
    t0 = time.perf_counter()
    step_fn(args.steps)
    th = time.perf_counter()
    end_barrier()
    t1 = time.perf_counter()
    if fast is not None:
        if hasattr(comm, "poll_errors"):
            comm.poll_errors()  # a timed-out peer wait in the closing barrier raises here
        dbarrier()
    if os.environ.get("DTA_BENCH_TRACE"):
        print(f"[bench] host call {1e6 * (th - t0):.1f} us, wait {1e6 * (t1 - th):.1f} us", file=sys.stderr)
    elapsed = t1 - t0
    if ws > 1:
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    last_loss = finish()
    samples = args.batch * ws * args.steps
    value = samples / elapsed
    base = None
    bpath = ROOT / "bench_baseline.json"
    if bpath.exists():
        try:
            b = json.loads(bpath.read_text())
            b1 = b.get("torch_samples_per_s_1gpu")
            if b1:
                base = float(b1) * ws  # baseline assumed to scale perfectly (conservative for us)
        except (ValueError, OSError):
            base = None
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / base, 3) if base and args.model == "mlp2" else None,
        "dtype": "bf16" if args.model == "mlp2" else "fp32",
        "data": "synthetic (reference MyTrainDataset: 2048 x (rand(20), rand(1)), DistributedSampler order)",
        "config": {"model": f"mlp2 Linear(20,{args.hidden})-ReLU-Linear({args.hidden},1)" if args.model == "mlp2"
                   else "linear nn.Linear(20,1) (reference default)",
                   "global_batch": args.batch * ws, "seq_len": None, "parallelism": f"dp{ws}",
                   "per_gpu_batch": args.batch, "optimizer": "SGD(lr=1e-3)",
                   "loss": "mse" if args.model == "mlp2" else "cross_entropy", "impl": args.impl},
        "final_loss": last_loss,
    }
    if getattr(args, "shared_gpu", False):
        out["shared_gpu"] = f"{ws} ranks on {torch.cuda.device_count()} GPU(s): correctness rehearsal, not a scaling number"
    out.update(getattr(finish, "info", {}))
    if comm is not None and ws > 1:
        out["comm"] = getattr(comm, "name", type(comm).__name__)
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            Path(args.json_out).write_text(line + "\n")
    if ws > 1:
        dbarrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
