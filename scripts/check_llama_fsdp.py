"""Debug: Llama tiny loss trajectories -- plain vs DDP vs FSDP (+/- activation checkpointing)."""
import torch

from distributed_training_amd.models.llama import Block, Llama, LlamaConfig
from distributed_training_amd.ops import lm
from distributed_training_amd.ops.optim import FusedAdamW
from distributed_training_amd.parallel.comm import RcclComm
from distributed_training_amd.parallel.ddp import DistributedDataParallel
from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

dev = torch.device("cuda", 0)
comm = RcclComm(0, 1, dev)
cfg = LlamaConfig(n_layer=2, n_head=4, n_kv_head=2, n_embd=256, ffn_hidden=512, vocab_size=1024, block_size=256)
x = torch.randint(0, 1024, (2, 129), device=dev, generator=torch.Generator(device=dev).manual_seed(0))


def run(kind, ckpt):
    torch.manual_seed(0)
    m = Llama(cfg).to(dev)
    if ckpt:
        m.enable_activation_checkpointing()
    if kind == "ddp":
        w = DistributedDataParallel(m, comm=comm, device=dev, param_dtype=torch.bfloat16)
    elif kind == "fsdp":
        w = FullyShardedDataParallel(m, comm=comm, device=dev, wrap_policy={Block}, param_dtype=torch.bfloat16)
    else:
        w = FullyShardedDataParallel(m, comm=comm, device=dev, wrap_policy=None, param_dtype=torch.bfloat16)
    opt = FusedAdamW(w.parameters(), lr=3e-3, weight_decay=0.0)
    out = []
    for _ in range(40):
        opt.zero_grad()
        logits = w(x[:, :-1])
        loss = lm.cross_entropy(logits.reshape(-1, logits.shape[-1]), x[:, 1:].reshape(-1))
        loss.backward()
        opt.step()
        out.append(round(loss.item(), 3))
    return out


for kind in ("ddp", "fsdp", "fsdp1"):
    for ck in (False, True):
        print(kind, ck, run(kind, ck)[::4])
