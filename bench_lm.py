#!/usr/bin/env python3
"""Transformer benchmarks for the GPT-2 small (DDP / FSDP) and Llama-3 8B
(FSDP) configurations of BASELINE.json: tokens/s (whole job), samples/s,
model-FLOPs utilisation against the 2.5 PF/s dense bf16 MFMA peak.

    python bench_lm.py --model gpt2 --strategy ddp --batch 8 --seq 1024
    python bench_lm.py --model gpt2 --strategy fsdp
    python bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --ckpt
    python bench_lm.py --model gpt2 --impl torch   # stock PyTorch-ROCm baseline (SDPA, torch DDP, AdamW)
    torchrun --nproc-per-node N bench_lm.py --gpus N ...

Synthetic tokens, random-init weights; every timed step is a full
forward + backward + gradient communication + AdamW update.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path
from typing import TYPE_CHECKING, Optional, Tuple, Union

if TYPE_CHECKING:
    import torch

    from distributed_training_amd.models.gpt2 import GPT2Config
    from distributed_training_amd.models.llama import LlamaConfig

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_BF16 = 2.5e15  # dense bf16 MFMA peak per MI355X


def parse() -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", default="gpt2", choices=["gpt2", "llama3_8b", "llama_1b", "llama_tiny"])
    ap.add_argument("--strategy", default="ddp", choices=["ddp", "fsdp"])
    ap.add_argument("--impl", default="native", choices=["native", "torch"])
    ap.add_argument("--batch", type=int, default=8, help="per-GPU micro-batch (sequences)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ckpt", action="store_true", help="activation checkpointing")
    ap.add_argument("--bucket-mb", default="auto", help="DDP bucket cap in MiB, or auto (xGMI-derived)")
    ap.add_argument("--layers", type=int, default=0, help="override n_layer (0 = config)")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--no-graph", action="store_true",
                    help="native DDP: launch the step's kernels eagerly instead of replaying the whole step as one "
                         "hipGraph (engine/step_graph.py)")
    ap.add_argument("--overlap-opt", action="store_true",
                    help="native DDP / FSDP: AdamW per bucket / unit inside the backward (overlap_optimizer of "
                         "DistributedDataParallel / FullyShardedDataParallel) instead of after it; bit-identical")
    ap.add_argument("--head-ce-chunk", type=int, default=0,
                    help="LM head + CE in row blocks of this many tokens, never holding the [T, V] logits "
                         "(ops/lm.py _ChunkedLinearCrossEntropy); 0 = one block")
    ap.add_argument("--tunableop", action="store_true",
                    help="let PyTorch's TunableOp pick the hipBLASLt/rocBLAS solution per GEMM shape (tuned in warmup)")
    return ap.parse_args()


def model_cfg(name: str, layers: int) -> Union["GPT2Config", "LlamaConfig"]:
    from distributed_training_amd.models.gpt2 import GPT2Config
    from distributed_training_amd.models.llama import LlamaConfig

    if name == "gpt2":
        c = GPT2Config()
    elif name == "llama3_8b":
        c = LlamaConfig()
    elif name == "llama_1b":
        c = LlamaConfig(n_layer=16, n_head=32, n_kv_head=8, n_embd=2048, ffn_hidden=8192, block_size=8192)
    else:
        c = LlamaConfig(n_layer=4, n_head=8, n_kv_head=2, n_embd=512, ffn_hidden=1536, vocab_size=32000,
                        block_size=4096)
    if layers:
        c.n_layer = layers
    return c


def main() -> None:
    args = parse()
    if args.tunableop:
        os.environ.setdefault("PYTORCH_TUNABLEOP_ENABLED", "1")
        os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "1")
        os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", f"/tmp/tunableop_{args.model}_%d.csv")
    import torch
    import torch.distributed as dist

    from distributed_training_amd.parallel.ipc import device_index, dist_backend

    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", device_index(local))  # DTA_SHARED_GPU=1: several ranks per GPU (rehearsal)
    local = dev.index
    torch.cuda.set_device(dev)
    if ws > 1:
        backend = dist_backend(True)
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))
    torch.manual_seed(0)
    cfg = model_cfg(args.model, args.layers)
    is_gpt = args.model == "gpt2"
    if is_gpt:
        from distributed_training_amd.models.gpt2 import GPT2 as M
    else:
        from distributed_training_amd.models.llama import Llama as M
    with torch.device("meta"):
        n_params = sum(p.numel() for p in M(cfg).parameters())
    with torch.device(dev):  # initialise straight on the GPU (8B params: no host round trip)
        model = M(cfg)
    if args.ckpt:
        model.enable_activation_checkpointing()
    V = cfg.vocab_size
    gen = torch.Generator(device=dev).manual_seed(1 + rank)
    data = torch.randint(0, V, (max(4, 64 // max(1, args.batch)) * args.batch, args.seq + 1), device=dev,
                         generator=gen)

    overlap_opt = False
    if args.impl == "native":
        from distributed_training_amd.ops import lm
        from distributed_training_amd.ops.optim import FusedAdamW

        lm.set_head_ce_chunk(args.head_ce_chunk)
        from distributed_training_amd.parallel.comm import make_comm

        comm = make_comm(dev, bulk=True)  # DDP / FSDP traffic: RCCL or the IPC push plane per message size
        model = model.to(dev)
        if args.strategy == "ddp":
            from distributed_training_amd.parallel.ddp import DistributedDataParallel

            wrapped = DistributedDataParallel(model, comm=comm, device=dev, param_dtype=torch.bfloat16,
                                              bucket_cap_mb=args.bucket_mb if args.bucket_mb == "auto" else float(args.bucket_mb))
        else:
            from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel, lm_wrap_policy

            # blocks + (Llama) the embedding and the output head as units of their own
            wrapped = FullyShardedDataParallel(model, comm=comm, device=dev, wrap_policy=lm_wrap_policy(model),
                                               param_dtype=torch.bfloat16)
        opt = FusedAdamW(wrapped.parameters(), lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1)
        overlap_opt = args.overlap_opt and wrapped.overlap_optimizer(opt)

        def loss_fn(logits: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
            return lm.cross_entropy(logits.reshape(-1, logits.shape[-1]), y.reshape(-1))
    else:
        import torch.nn.functional as F

        model = model.to(dev)
        # stock path: swap the framework ops for torch's (SDPA, F.layer_norm, ...)
        _patch_torch_ops()
        if args.strategy == "ddp":
            wrapped = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local]) if ws > 1 else model
        else:
            from torch.distributed.fsdp import FullyShardedDataParallel as TFSDP
            from torch.distributed.fsdp import MixedPrecision
            from torch.distributed.fsdp.wrap import ModuleWrapPolicy

            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29577")
                dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
            wrapped = TFSDP(model, auto_wrap_policy=ModuleWrapPolicy({M.block_class}), device_id=dev,
                            mixed_precision=MixedPrecision(param_dtype=torch.bfloat16, reduce_dtype=torch.bfloat16))
        opt = torch.optim.AdamW(wrapped.parameters(), lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1, fused=True)

        def loss_fn(logits: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
            return F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), y.reshape(-1))

    nb = data.shape[0] // args.batch
    state = {"i": 0, "loss": None}

    from distributed_training_amd.utils import profiling as prof

    def step() -> None:
        prof.push("step")
        i = state["i"] % nb
        state["i"] += 1
        xb = data[i * args.batch:(i + 1) * args.batch]
        opt.zero_grad(set_to_none=True)
        if args.impl == "torch" and args.strategy == "ddp":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = wrapped(xb[:, :-1])
            loss = loss_fn(logits, xb[:, 1:])
        elif args.impl == "torch":
            loss = loss_fn(wrapped(xb[:, :-1]), xb[:, 1:])
        else:  # LM head + loss fused inside the model
            with prof.range_("forward"):
                loss = wrapped(xb[:, :-1], xb[:, 1:])
        with prof.range_("backward"):
            loss.backward()
        with prof.range_("optimizer"):
            opt.step()
        state["loss"] = loss
        prof.pop()

    graphed = None
    policy = (False, "torch baseline")
    if args.impl == "native":
        # the Trainer's policy (engine/step_graph.py capture_policy): engine state capturable, and at
        # world size > 1 every collective on the IPC data plane (RCCL in a graph: DTA_GRAPH_RCCL=1)
        from distributed_training_amd.engine.step_graph import capture_policy

        policy = capture_policy(wrapped)
    if args.impl == "native" and policy[0] and not args.no_graph:
        # the whole step (zero_grad, forward, backward with the bucket hooks, AdamW) as ONE hipGraph;
        # its construction runs 3 eager warm-up steps and the capture (untimed, before the warm-up below)
        from distributed_training_amd.engine.step_graph import GraphedStep

        def gstep(xb: torch.Tensor) -> torch.Tensor:
            opt.zero_grad(set_to_none=True)
            loss = wrapped(xb[:, :-1], xb[:, 1:])
            loss.backward()
            opt.step()
            return loss

        graphed = GraphedStep(gstep, [data[:args.batch].clone()], warmup=3, engine=wrapped)
        if not graphed.ok:  # a step that cannot be captured (all ranks agreed) keeps the eager launches
            print(f"[bench_lm] step graph unavailable ({graphed.error}); eager step", file=sys.stderr)
            graphed = None

    if graphed is not None:
        def step() -> None:  # noqa: F811 - the graph replay replaces the eager step
            i = state["i"] % nb
            state["i"] += 1
            state["loss"] = graphed(data[i * args.batch:(i + 1) * args.batch])

    def dbarrier() -> None:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[local])
        else:
            dist.barrier()

    def barrier() -> None:
        torch.cuda.synchronize(dev)
        if ws > 1:
            dbarrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    c0 = time.process_time()
    for _ in range(args.steps):
        step()
    # host cost of the step: the wall time until the last step is ENQUEUED (no sync inside the step, so
    # this is below the GPU time unless the host is the bottleneck) and the CPU time of every thread
    # (autograd's device thread included) -- eager vs graphed (--no-graph) is this difference
    t_enq = time.perf_counter() - t0
    c_enq = time.process_time() - c0
    barrier()
    el = time.perf_counter() - t0
    peak_mem = torch.cuda.max_memory_allocated(dev)
    if ws > 1:
        t = torch.tensor([el], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if os.environ.get("DTA_SYNC_DEBUG"):
        # diagnostics: one more (untimed) step with torch's sync debug mode -- every host
        # synchronisation inside the step (a .item(), a read-back) prints a warning + stack
        torch.cuda.set_sync_debug_mode("warn")
        step()
        torch.cuda.set_sync_debug_mode(0)
        torch.cuda.synchronize(dev)
    if os.environ.get("DTA_PROFILE_OPS"):
        # diagnostics: one more (untimed) step under torch.profiler on EVERY rank (the
        # step's collectives must match across ranks); rank 0 prints the table
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as tprof:
            step()
            torch.cuda.synchronize(dev)
        if rank == 0:
            print(tprof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=70),
                  file=sys.stderr)
    tokens = args.batch * args.seq * ws * args.steps
    flops_tok = 6 * (n_params - (cfg.block_size * cfg.n_embd if is_gpt else 0)) + 12 * cfg.n_layer * cfg.n_embd * args.seq
    tps = tokens / el
    mfu = tps * flops_tok / (PEAK_BF16 * ws)
    out = {"metric": f"tokens/s ({args.model} {args.strategy} bf16)", "value": round(tps, 1), "unit": "tokens/s",
           "n_gpus": ws, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
           "higher_is_better": True, "scaling": "weak", "dtype": "bf16", "data": "synthetic tokens",
           "samples_per_s": round(args.batch * ws * args.steps / el, 2), "mfu": round(mfu, 4),
           "params_M": round(n_params / 1e6, 1), "peak_mem_GB": round(peak_mem / 1e9, 2),
           "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 3),
           "host_cpu_ms_per_step": round(c_enq / args.steps * 1e3, 3),
           "final_loss": float(state["loss"].item()),
           "fsdp_units": (len(wrapped.units) if args.impl == "native" and args.strategy == "fsdp" else None),
           "comm": ("none: one rank (DDP skips the all-reduce, FSDP runs NO_SHARD)" if ws == 1 else
                    type(getattr(wrapped, "comm", None)).__name__ if args.impl == "native" else "torch"),
           "config": {"model": args.model, "layers": cfg.n_layer, "global_batch": args.batch * ws,
                      "seq_len": args.seq, "parallelism": f"{args.strategy}{ws}", "impl": args.impl, "tunableop": args.tunableop,
                      "activation_checkpointing": args.ckpt}}
    if args.impl == "native":
        from distributed_training_amd.ops import lm as _lm

        # which implementation each projection GEMM shape runs (measured per shape, DTA_GEMM=auto)
        out["optimizer_in_backward"] = bool(overlap_opt)
        out["step_graph"] = graphed is not None
        out["capture_policy"] = policy[1]
        if args.strategy == "ddp":
            out["bucket_caps"] = {"first_MiB": round(wrapped.bucket_bytes[0] / 2 ** 20, 2),
                                  "cap_MiB": round(wrapped.bucket_bytes[1] / 2 ** 20, 2),
                                  "buckets": len(wrapped.buckets), "source": wrapped.bucket_caps_source}
        out["head_ce_chunk"] = _lm.HEAD_CE_CHUNK
        routes = getattr(getattr(wrapped, "comm", None), "routes", None)
        if routes is not None:
            out["comm_routes"] = routes()
            out["comm_classes_at_wrap"] = getattr(wrapped.comm, "prepared_log", [])
        out["gemm_calls"] = {"dta": _lm.GEMM_STATS["dta"], "hipblaslt": _lm.GEMM_STATS["torch"]}
        out["gemm_impl"] = {f"{k[0]} {k[1]}x{k[2]}x{k[3]}": ("hipblaslt" if not v else
                                                             f"k64/t{v - _lm.K64}" if v >= _lm.K64 else f"r2/t{v}")
                            for k, v in sorted(_lm._GEMM_CHOICE.items())}
        src = list(_lm.GEMM_PICK_SOURCE.values())
        out["gemm_pick_source"] = {s_: src.count(s_) for s_ in sorted(set(src))}  # tracked table vs in-run timing
    if rank == 0:
        print(json.dumps(out), flush=True)
        if args.json_out:
            Path(args.json_out).write_text(json.dumps(out) + "\n")
    if dist.is_initialized():
        dbarrier()
        dist.destroy_process_group()


def _patch_torch_ops() -> None:
    """Route the models' op calls to stock PyTorch (for the baseline)."""
    import torch
    import torch.nn.functional as F

    from distributed_training_amd.ops import lm

    def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
                  scale: Optional[float] = None) -> torch.Tensor:
        H, Hkv = q.shape[2], k.shape[2]
        qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
        return F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal, scale=scale,
                                              enable_gqa=H != Hkv).transpose(1, 2)

    def attention_packed(qkv: torch.Tensor, n_head: int, n_kv_head: int, causal: bool = True,
                         scale: Optional[float] = None,
                         rope: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
        q, k, v = lm._split_qkv(qkv, n_head, n_kv_head)
        if rope is not None:
            q, k = lm.rope_reference(q, *rope), lm.rope_reference(k, *rope)
        return attention(q, k, v, causal, scale)

    def add_ln(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, b: torch.Tensor,
               eps: float = 1e-5) -> Tuple[torch.Tensor, torch.Tensor]:
        xn = x + res
        return xn, F.layer_norm(xn, (xn.shape[-1],), w, b, eps)

    def add_rms(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> Tuple[torch.Tensor, torch.Tensor]:
        xn = x + res
        return xn, F.rms_norm(xn, (xn.shape[-1],), w, eps)

    def linear_ce(x: torch.Tensor, w: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
        logits = F.linear(x, w)
        return F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), target.reshape(-1),
                               ignore_index=ignore_index)

    lm.attention = attention
    lm.attention_packed = attention_packed
    lm.layer_norm = lambda x, w, b, eps=1e-5: F.layer_norm(x, (x.shape[-1],), w, b, eps)
    lm.rms_norm = lambda x, w, eps=1e-5: F.rms_norm(x, (x.shape[-1],), w, eps)
    lm.add_layer_norm = add_ln
    lm.add_rms_norm = add_rms
    lm.linear = F.linear
    lm.linear_cross_entropy = linear_ce
    lm.gelu = lambda x: F.gelu(x, approximate="tanh")
    lm.embedding = F.embedding
    lm.swiglu = lambda ab: F.silu(ab.chunk(2, -1)[0]) * ab.chunk(2, -1)[1]
    lm.apply_rope = lm.rope_reference


if __name__ == "__main__":
    main()
