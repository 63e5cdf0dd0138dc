"""Training engine.

Reference: ``TrainingConfig`` (src/distributed_trainer.py:29-39) and ``Trainer``
(:108-192) -- same constructor, same ``train(max_epochs)`` loop, same log
lines:

    "[CUDA0] Running with 8 processes total"
    "[CUDA0] Epoch 3 | Batchsize: 32 | Steps: 8"
    "Loading snapshot" / "Epoch 4 | Training snapshot saved at snapshot.pt"

Engine differences (all behaviour-preserving unless noted):

* the model is wrapped by the native DDP/FSDP engines (``parallel/``);
* torch optimizers over GPU parameters are swapped for the fused HIP
  optimizers with identical hyper-parameters (``fused_optimizer``);
* batches come from the device-resident loader (no per-step H2D copy, no
  extra batch fetched just to log its size -- SURVEY.md Q6);
* for the 2-layer MLP (and the reference default, one nn.Linear) + DDP + SGD
  configuration the whole step runs as the
  fused gfx950 kernel + RCCL all-reduce, hipGraph-captured
  (:mod:`.fused_mlp`);
* checkpoint save is entered by every rank (rank 0 writes) -- required for
  FSDP's collective full-state gather;
* the loss is configurable (``cross_entropy`` = reference default, which is
  identically 0 for a 1-wide output -- SURVEY.md Q1; ``mse``).
"""
from __future__ import annotations

import logging
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Callable, Dict, Optional

import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader

from ..parallel.env import DistributedEnvironment
from ..parallel.sampler import DistributedSampler as DtaSampler
from ..parallel.strategy import DDPStrategy, DistributedStrategy, FSDPStrategy, default_comm
from ..utils import profiling as prof
from .checkpoint import ModelCheckpoint

logger = logging.getLogger("distributed_training_amd.trainer")


@dataclass
class TrainingConfig:
    """Configuration for training parameters (reference fields first)."""

    max_epochs: int
    save_every: int
    batch_size: int
    learning_rate: float
    snapshot_path: Path
    device: str = "auto"
    parallel_strategy: str = "ddp"
    # ---- extensions (defaults keep reference behaviour) ----
    loss: str = "cross_entropy"
    fused_step: bool = True          # fused MLP kernel path when eligible
    fused_optimizer: bool = True     # swap torch optimizers for the HIP ones
    graph_steps: int = 32            # steps per hipGraph replay (fused path)
    bucket_cap_mb: Any = "auto"      # MiB, or "auto": sized for xGMI (parallel/flat.py xgmi_bucket_caps)
    first_bucket_mb: Any = None      # MiB, or None / "auto" (with a numeric cap: 1 MiB like torch)
    mixed_precision: Optional[str] = None   # None / "bf16"
    fsdp_wrap: Optional[Any] = None          # wrap policy for FSDP
    log_throughput: bool = False
    grad_clip: Optional[float] = None
    save_optimizer: bool = False
    desync_check_every: int = 0
    fault_injection: Optional[Dict[str, int]] = None
    cpu_offload: bool = False        # FSDP: fp32 shards, gradients and optimizer on the host
    reduce_dtype: Optional[str] = None  # FSDP gradient reduce-scatter dtype: None = compute dtype, "fp32"
    fsdp_sharding: str = "full"      # FSDP: "full" (FULL_SHARD) or "hybrid" (HSDP: shard per node, replicate)
    hybrid_shard_size: Optional[int] = None  # HSDP shard group size (default: LOCAL_WORLD_SIZE)
    optimizer_in_backward: bool = False  # DDP on GPU: fused update per bucket inside the backward (no grad_clip)
    step_graph: bool = False         # DDP on GPU: whole step replayed as one hipGraph (engine/step_graph.py)
    extra: Dict[str, Any] = field(default_factory=dict)


LOSSES: Dict[str, Callable] = {
    "cross_entropy": F.cross_entropy,
    "mse": F.mse_loss,
}


def lm_loss(logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    """Token cross-entropy; the fused gfx950 kernel on GPU (ops/lm.py)."""
    from ..ops.lm import cross_entropy

    return cross_entropy(logits.reshape(-1, logits.shape[-1]), targets.reshape(-1))


class Trainer:
    """Manages the training process in a distributed environment."""

    def __init__(self, model: torch.nn.Module, train_data: Any, optimizer: torch.optim.Optimizer,
                 config: TrainingConfig, env: DistributedEnvironment) -> None:
        self.env = env
        self.config = config
        self.epochs_run = 0
        self.optimizer = optimizer
        self.train_data = train_data
        from ..data.datasets import DeviceDataLoader

        if isinstance(train_data, DeviceDataLoader):
            train_data.to(env.torch_device if hasattr(env, "torch_device") else torch.device(env.device))
        self._loss_fn = LOSSES.get(config.loss, None) if config.loss != "lm" else lm_loss
        if self._loss_fn is None:
            raise ValueError(f"unknown loss {config.loss!r}")
        self.model = self._setup_model(model)
        self.checkpoint = ModelCheckpoint(Path(config.snapshot_path), env, self._strategy,
                                          save_optimizer=config.save_optimizer)
        self._fused = None
        self._maybe_build_fused()
        if self._fused is None and config.optimizer_in_backward and not config.grad_clip \
                and hasattr(self.model, "overlap_optimizer"):
            # bit-identical to backward + step(); the update of late buckets overlaps the early backward
            if self.model.overlap_optimizer(self.optimizer):
                logger.debug("optimizer stepped per DDP bucket inside the backward")
        self.last_epoch_stats: Dict[str, float] = {}
        logger.info(
            f"[{str(self.env.device).upper()}{self.env.global_rank}] "
            f"Running with {self.env.world_size} processes total"
        )

    # ------------------------------------------------------------------ setup
    @property
    def device(self) -> torch.device:
        return self.env.torch_device if hasattr(self.env, "torch_device") else torch.device(self.env.device)

    def _make_strategy(self) -> DistributedStrategy:
        c = self.config
        if c.parallel_strategy.lower() == "fsdp":
            return FSDPStrategy(self.env.is_gpu, wrap_policy=c.fsdp_wrap, mixed_precision=c.mixed_precision,
                                cpu_offload=c.cpu_offload, reduce_dtype=c.reduce_dtype, sharding=c.fsdp_sharding,
                                hybrid_shard_size=c.hybrid_shard_size)
        return DDPStrategy(self.env.local_rank, self.env.is_gpu, bucket_cap_mb=c.bucket_cap_mb,
                           first_bucket_mb=c.first_bucket_mb, mixed_precision=c.mixed_precision)

    def _setup_model(self, model: torch.nn.Module) -> torch.nn.Module:
        device = self.env.torch_device.index if self.env.is_gpu else self.env.device
        self._strategy = self._make_strategy()
        from ..models.init import init_buffers_, is_meta, materialize_

        if is_meta(model):
            # built on the meta device (app.load_train_objs, LM configs): never initialised on the host.
            # FSDP materialises unit by unit into its shards; DDP allocates and initialises on the device
            if isinstance(self._strategy, FSDPStrategy):
                init_buffers_(model, self.device)
            else:
                materialize_(model, self.device)
        else:
            model = model.to(self.device)
        self.checkpoint = ModelCheckpoint(Path(self.config.snapshot_path), self.env, self._strategy)
        original_params = [p for g in self.optimizer.param_groups for p in g["params"]]
        model = self._strategy.prepare_model(model, self.device)
        self._rebind_optimizer(model, original_params)
        model, self.epochs_run = self.checkpoint.load(model, device, self.optimizer)
        return model

    def _rebind_optimizer(self, model: torch.nn.Module, original_params: Any) -> None:
        """FSDP replaces the parameters by shards: rebuild the optimizer over
        them (same class and hyper-parameters).  Torch optimizers over GPU
        parameters become the fused HIP optimizers."""
        from ..ops.optim import FusedAdamW, FusedSGD, same_kind_optimizer

        new_params = [p for p in model.parameters() if p.requires_grad]
        same = {id(p) for p in original_params} == {id(p) for p in new_params}
        fused = isinstance(self.optimizer, (FusedSGD, FusedAdamW))
        want_fused = self.config.fused_optimizer and self.env.is_gpu and all(p.is_cuda for p in new_params)
        if same and (fused or not want_fused):
            return
        if want_fused or not same:
            opt = same_kind_optimizer(self.optimizer, new_params)
            if not want_fused and not same:
                opt = type(self.optimizer)(new_params, **{k: v for k, v in self.optimizer.param_groups[0].items()
                                                          if k != "params"})
            self.optimizer = opt

    def _maybe_build_fused(self) -> None:
        if not (self.config.fused_step and self.env.is_gpu and isinstance(self._strategy, DDPStrategy)):
            return
        from ..data.datasets import DeviceDataLoader
        from .fused_mlp import FusedMLPProgram, fused_eligible

        module = self.model.module
        loader = self.train_data
        if isinstance(loader, DeviceDataLoader):
            loader.to(self.device)
        why = fused_eligible(module, self.optimizer, loader, self.config.loss, self.device)
        if why is None:
            self._fused = FusedMLPProgram(module, self.optimizer, loader, default_comm(self.device),
                                          loss=self.config.loss, graph_steps=self.config.graph_steps)
            logger.debug("fused MLP step program enabled")
            return
        # the reference's default model (one nn.Linear, CE, fp32, SGD)
        from .fused_linear import FusedLinearProgram, linear_eligible

        why_lin = linear_eligible(module, self.optimizer, loader, self.config.loss, self.device)
        if why_lin is None:
            self._fused = FusedLinearProgram(module, self.optimizer, loader, default_comm(self.device),
                                             loss=self.config.loss)
            logger.debug("fused Linear step program enabled")
        else:
            logger.debug(f"fused step programs not used: {why}; {why_lin}")

    # ------------------------------------------------------------------ loop
    def _graph_eligible(self, source: torch.Tensor, targets: torch.Tensor) -> bool:
        from ..ops.optim import FusedAdamW, FusedSGD
        from .step_graph import capture_policy

        c = self.config
        # only the fused optimizers keep their step count on the device (torch's AdamW keeps it on the
        # host and cannot be captured)
        if not (c.step_graph and self.env.is_gpu and source.is_cuda and not c.grad_clip
                and isinstance(self.optimizer, (FusedSGD, FusedAdamW))
                and not c.desync_check_every and getattr(self, "_graphed", None) is not False):
            return False
        if getattr(self, "_policy", None) is None:
            self._policy = capture_policy(self.model)  # (the one policy bench_lm.py applies too)
            if not self._policy[0]:
                logger.info(f"step graph not used: {self._policy[1]}")
        return self._policy[0]

    def _run_batch(self, source: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        if self._graph_eligible(source, targets):
            g = getattr(self, "_graphed", None)
            if g is None:
                from .step_graph import GraphedStep

                # one eager step on this batch (the warm-up), then the capture; a failed capture
                # (agreed on by every rank) leaves the eager step for the rest of the run
                g = GraphedStep(self._run_batch_eager, [source.clone(), targets.clone()], warmup=1,
                                engine=self.model)
                self._graphed = g if g.ok else False
                if g.ok:
                    logger.info("step graph: the whole training step is replayed as one hipGraph")
                return g.warmup_losses[-1]
            if all(s.shape == x.shape and s.dtype == x.dtype for s, x in zip(g.static, (source, targets))):
                return g(source, targets)
            # a batch of another shape (an epoch's short last batch): the eager step
        return self._run_batch_eager(source, targets)

    def _run_batch_eager(self, source: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        # roctx ranges (DTA_ROCTX=1): step phases on the rocprofv3 --marker-trace timeline
        self.optimizer.zero_grad()
        with prof.range_("forward"):
            if self.config.loss == "lm":  # transformer LMs fuse the head and the loss (models/gpt2.py, llama.py)
                loss = self.model(source, targets)
            else:
                output = self.model(source)
                loss = self._loss_fn(output, targets)
        with prof.range_("backward"):
            loss.backward()
        if self.config.grad_clip:
            with prof.range_("clip_grad_norm"):
                if hasattr(self.model, "clip_grad_norm_"):  # native engines: global norm over the flat (sharded) grads
                    self.model.clip_grad_norm_(self.config.grad_clip)
                else:
                    torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.config.grad_clip)
        with prof.range_("optimizer"):
            self.optimizer.step()
        return loss

    def _batch_size_for_log(self) -> int:
        sampler = getattr(self.train_data, "sampler", None)
        n = len(sampler) if sampler is not None else self.config.batch_size
        return min(self.config.batch_size, n)

    def _run_epoch(self, epoch: int) -> None:
        b_sz = self._batch_size_for_log()
        logger.info(
            f"[{str(self.env.device).upper()}{self.env.global_rank}] "
            f"Epoch {epoch} | Batchsize: {b_sz} | "
            f"Steps: {len(self.train_data)}"
        )
        sampler = self.train_data.sampler
        assert isinstance(sampler, (DtaSampler, torch.utils.data.distributed.DistributedSampler))
        t0 = time.perf_counter()
        loss_sum: Optional[torch.Tensor] = None  # this rank's epoch loss, summed on the device (no per-step sync)
        if self._fused is not None:
            steps = self._fused.run_epoch(epoch)
        else:
            sampler.set_epoch(epoch)
            steps = 0
            dev = self.device
            for source, targets in self.train_data:
                source = source.to(dev, non_blocking=True)
                targets = targets.to(dev, non_blocking=True)
                loss = self._run_batch(source, targets)
                if self.config.log_throughput and loss is not None:
                    # accumulate into a buffer of our own: a replayed step graph returns its static loss
                    # tensor (overwritten by the next replay), and .float() of an fp32 loss is no copy
                    if loss_sum is None:
                        loss_sum = torch.zeros((), dtype=torch.float32, device=loss.device)
                    loss_sum += loss.detach().float()
                steps += 1
                self._maybe_inject_fault(epoch, steps)
        if self.config.log_throughput or self.config.desync_check_every:
            if self.env.is_gpu:
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            samples = len(sampler) * self.env.world_size
            self.last_epoch_stats = {"epoch": epoch, "steps": steps, "seconds": dt, "samples_per_s": samples / dt}
            if self.config.log_throughput:
                msg = f"Epoch {epoch} | {steps} steps | {dt * 1e3:.2f} ms | {samples / dt:,.0f} samples/s"
                if loss_sum is not None and steps:
                    self.last_epoch_stats["loss"] = float(loss_sum.item()) / steps
                    msg += f" | loss {self.last_epoch_stats['loss']:.4f}"
                if steps:
                    self.last_epoch_stats["ms_per_step"] = dt * 1e3 / steps
                    msg += f" | {dt * 1e3 / steps:.2f} ms/step"
                seq = getattr(getattr(self.train_data, "dataset", None), "seq_len", None)
                if seq:  # token LMs: tokens/s over all ranks
                    self.last_epoch_stats["tokens_per_s"] = samples * int(seq) / dt
                    msg += f" | {samples * int(seq) / dt:,.0f} tokens/s"
                logger.info(msg)
        if self.config.desync_check_every and (epoch + 1) % self.config.desync_check_every == 0:
            from ..utils.desync import check_replicas_in_sync

            self._sync_fused_to_module()
            check_replicas_in_sync(self.model, self.env)

    def _maybe_inject_fault(self, epoch: int, step: int) -> None:
        fi = self.config.fault_injection
        if fi and fi.get("rank", -1) == self.env.global_rank and fi.get("epoch", -1) == epoch \
                and fi.get("step", 1) == step:
            from ..utils.fault import inject_fault

            inject_fault(fi)

    def _sync_fused_to_module(self) -> None:
        if self._fused is not None:
            self._fused.store_to_module()

    def train(self, max_epochs: int) -> None:
        for epoch in range(self.epochs_run, max_epochs):
            self._run_epoch(epoch)
            # (save_every <= 0: no snapshots -- an extension; the reference's modulo would divide by zero)
            if self.config.save_every > 0 and epoch % self.config.save_every == 0:
                self._sync_fused_to_module()
                self.checkpoint.save(self.model, epoch, self.optimizer)
        self._sync_fused_to_module()
