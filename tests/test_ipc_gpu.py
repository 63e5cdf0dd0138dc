"""IPC direct-push collectives (csrc/ipc_coll.hip) and the multi-rank DDP / FSDP
GPU engines on top of them, with several processes sharing the box's single
GPU (DTA_SHARED_GPU=1).  Same kernels, comm stream, record_stream, storage
resize_ and prefetch code as on a real 8-GPU node; only the link differs.

References: every collective against exact expectations built from all ranks'
inputs (gathered over gloo), reduced in rank order in fp32 and rounded once;
the engines against the same model trained by ONE rank on the global batch."""
import os

import pytest
import torch

from dist_utils import run_gloo

pytestmark = pytest.mark.gpu


def _shared():
    os.environ["DTA_SHARED_GPU"] = "1"
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


def _gather_cpu(x):
    """All ranks' copies of x as fp32 CPU tensors (exact for fp32 / bf16 inputs; gloo has no bf16)."""
    import torch.distributed as dist

    c = x.detach().float().cpu().contiguous()
    parts = [torch.empty_like(c) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, c)
    return parts


def _coll_worker(rank, ws, slot_mb):
    from distributed_training_amd.parallel.ipc import IpcComm

    dev = _shared()
    comm = IpcComm(rank, ws, dev, slot_mb=slot_mb)
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    # all-reduce: sizes around vector / chunk / segment boundaries, both dtypes, every op
    for dt in (torch.float32, torch.bfloat16):
        for n in (1, 7, 8 * ws + 3, 4097, 70001, 300007):
            for op in ("sum", "avg", "max", "min"):
                x = torch.randn(n, generator=g).to(dt).to(dev)
                parts = _gather_cpu(x)
                acc = parts[0].clone()
                for p in parts[1:]:  # rank order, fp32, like the kernel
                    acc = acc + p if op in ("sum", "avg") else (torch.maximum(acc, p) if op == "max"
                                                                else torch.minimum(acc, p))
                if op == "avg":
                    acc = acc * (1.0 / ws)
                want = acc.to(dt)
                comm.all_reduce(x, op)
                torch.cuda.synchronize()
                assert torch.equal(x.cpu(), want), (dt, n, op, (x.cpu().float() - want.float()).abs().max())
    # reduce-scatter / all-gather: aligned and unaligned chunk sizes, async + wait
    for dt in (torch.float32, torch.bfloat16):
        for m in (5, 64, 1000, 40000):
            inp = torch.randn(ws * m, generator=g).to(dt).to(dev)
            parts = _gather_cpu(inp)
            full = sum(parts[1:], parts[0].clone()) * (1.0 / ws)
            out = torch.empty(m, dtype=dt, device=dev)
            w = comm.reduce_scatter_into(out, inp, op="avg", async_op=True)
            w.wait()
            torch.cuda.synchronize()
            assert torch.equal(out.cpu(), full[rank * m:(rank + 1) * m].to(dt)), (dt, m)
            shard = torch.randn(m, generator=g).to(dt).to(dev)
            gathered = torch.empty(ws * m, dtype=dt, device=dev)
            comm.all_gather_into(gathered, shard)
            torch.cuda.synchronize()
            assert torch.equal(gathered.float().cpu(), torch.cat(_gather_cpu(shard))), (dt, m)
    # broadcast: even / odd byte counts, every root
    for root in range(ws):
        for n in (3, 1001, 200003):
            b = torch.full((n,), float(rank * 10 + 1), device=dev)
            comm.broadcast(b, src=root)
            torch.cuda.synchronize()
            assert torch.equal(b, torch.full_like(b, float(root * 10 + 1))), (root, n)
        c = torch.full((7,), rank + 3, dtype=torch.uint8, device=dev)  # 7 bytes: control-plane path
        comm.broadcast(c, src=root)
        assert int(c[0]) == root + 3
    # many back-to-back async ops with compute in between (parity reuse, stream ordering)
    xs = [torch.full((11280,), float(rank + i), device=dev) for i in range(40)]
    works = []
    for x in xs:
        x.mul_(2.0)
        works.append(comm.all_reduce(x, "sum", async_op=True))
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    for i, x in enumerate(xs):
        assert torch.equal(x, torch.full_like(x, float(sum(2 * (r + i) for r in range(ws))))), i
    # hipGraph capture of the inline all-reduce (device epochs advance on replay)
    buf = torch.zeros(5000, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            for _ in range(3):
                buf.add_(1.0)
                comm.all_reduce_inline(buf, "sum", stream=s)
    torch.cuda.current_stream().wait_stream(s)
    for rep in range(2):
        buf.fill_(float(rank))
        graph.replay()
        torch.cuda.synchronize()
        b = [float(r) for r in range(ws)]
        for _ in range(3):
            b = [sum(v + 1.0 for v in b)] * ws
        assert torch.equal(buf, torch.full_like(buf, b[0])), rep
    comm.poll_errors()
    comm.destroy()


@pytest.mark.parametrize("ws", [2, 4])
def test_ipc_collectives_shared_gpu(ws):
    run_gloo(_coll_worker, ws, 0.25)  # 256 KiB slots: multi-segment messages


def _bf16_8rank_worker(rank, ws):
    """bf16 all-reduce at 8 ranks: ONE rounding of the exact fp32 rank-order sum."""
    from distributed_training_amd.parallel.ipc import IpcComm

    dev = _shared()
    comm = IpcComm(rank, ws, dev)
    g = torch.Generator(device="cpu").manual_seed(7 + rank)
    x = torch.randn(1 << 18, generator=g).to(torch.bfloat16).to(dev)
    parts = [p.double() for p in _gather_cpu(x)]  # exact bf16 values
    exact = sum(parts)                      # fp64 reference of the bf16 inputs
    comm.all_reduce(x, "sum")
    torch.cuda.synchronize()
    got = x.cpu().double()
    # one rounding to bf16 (8 significant bits) of a sum accumulated in fp32
    rel = ((got - exact).abs() / exact.abs().clamp_min(1e-3)).max().item()
    assert rel <= 2 ** -8 + 1e-6, rel
    allx = _gather_cpu(x)
    assert all(torch.equal(allx[0], a) for a in allx), "ranks disagree"
    comm.destroy()


def test_ipc_bf16_allreduce_error_8_ranks():
    run_gloo(_bf16_8rank_worker, 8)


def _timeout_worker(rank, ws):
    import torch.distributed as dist

    from distributed_training_amd.parallel.ipc import IpcComm

    dev = _shared()
    comm = IpcComm(rank, ws, dev, timeout_s=1.0)
    if rank == 0:  # the peer never joins: bounded wait, sticky error seen by the host poll
        x = torch.ones(1000, device=dev)
        comm.all_reduce(x)
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="timed out"):
            comm.poll_errors()
    dist.barrier()
    comm.destroy()


def test_ipc_timeout_raises():
    run_gloo(_timeout_worker, 2)


def _ddp_stall_worker(rank, ws):
    """A rank that stops taking part: the DDP engine of the others raises at its next
    step instead of training on partial gradient sums (no hang: bounded waits)."""
    import torch.distributed as dist
    import torch.nn.functional as F

    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.ipc import IpcComm

    dev = _shared()
    comm = IpcComm(rank, ws, dev, timeout_s=1.0)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 1)).to(dev)
    ddp = DistributedDataParallel(net, comm=comm, device=dev)
    x, y = torch.randn(8, 16, device=dev), torch.randn(8, 1, device=dev)
    F.mse_loss(ddp(x), y).backward()  # both ranks: a normal step
    torch.cuda.synchronize()
    if rank == 0:
        F.mse_loss(ddp(x), y).backward()  # the peer is gone: this exchange times out
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="timed out"):
            F.mse_loss(ddp(x), y).backward()
    dist.barrier()
    comm.destroy()


def test_ddp_raises_when_a_peer_stalls():
    run_gloo(_ddp_stall_worker, 2)


# ---------------------------------------------------------------- engines
def _tiny_gpt2():
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    return GPT2(GPT2Config(n_layer=2, n_head=2, n_embd=128, vocab_size=512, block_size=64))


def _train(model_wrapped, opt, batches, steps):
    losses = []
    for it in range(steps):
        x = batches[it]
        opt.zero_grad(set_to_none=True)
        loss = model_wrapped(x[:, :-1], x[:, 1:])
        loss.backward()
        opt.step()
        losses.append(float(loss.item()))
    return losses


def _engine_worker(rank, ws, strategy, overlap_opt=False):
    import torch.distributed as dist

    from distributed_training_amd.models.gpt2 import GPT2
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel
    from distributed_training_amd.parallel.ipc import IpcComm

    dev = _shared()
    B, T, steps = 2, 64, 3
    g = torch.Generator(device="cpu").manual_seed(5)
    glob = [torch.randint(0, 512, (ws * B, T + 1), generator=g).to(dev) for _ in range(steps)]
    # reference: one rank, the global batch, same bf16 engine with no communication
    ref = _tiny_gpt2().to(dev)
    ref_w = DistributedDataParallel(ref, comm=IpcComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
    ref_opt = FusedSGD(ref_w.parameters(), lr=0.05, momentum=0.9)
    init_sd = {k[len("module."):]: v.float().cpu().clone() for k, v in ref_w.state_dict().items()}
    ref_losses = _train(ref_w, ref_opt, glob, steps)
    ref_sd = {k[len("module."):]: v.float().cpu() for k, v in ref_w.state_dict().items()}

    comm = IpcComm(rank, ws, dev)
    model = _tiny_gpt2().to(dev)
    if rank == 1:  # a different init on one rank: the wrap-time broadcast must fix it
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.5)
    if strategy == "ddp":
        w = DistributedDataParallel(model, comm=comm, device=dev, param_dtype=torch.bfloat16,
                                    bucket_cap_mb=0.25, first_bucket_mb=0.05)  # several buckets: overlap path
        assert len(w.buckets) >= 3
    else:
        w = FullyShardedDataParallel(model, comm=comm, device=dev, wrap_policy={GPT2.block_class},
                                     param_dtype=torch.bfloat16)
        assert len(w.units) == 3
    opt = FusedSGD(w.parameters(), lr=0.05, momentum=0.9)
    if overlap_opt:  # the SGD update per bucket on a side stream, after that bucket's all-reduce
        assert w.overlap_optimizer(opt)
    local = [x[rank * B:(rank + 1) * B] for x in glob]
    losses = _train(w, opt, local, steps)
    comm.poll_errors()
    # mean of the per-rank losses == the reference's global-batch loss (before any update diverges)
    l0 = torch.tensor([losses[0]])
    dist.all_reduce(l0)
    assert abs(l0.item() / ws - ref_losses[0]) < 2e-2 * abs(ref_losses[0]), (l0.item() / ws, ref_losses[0])
    sd = w.full_state_dict(rank0_only=False) if strategy == "fsdp" else {
        k[len("module."):]: v for k, v in w.state_dict().items()}
    assert set(sd) == set(ref_sd), (sorted(set(sd) ^ set(ref_sd)))
    for k, v in sd.items():
        a, b = v.float().cpu(), ref_sd[k]
        moved = (b - init_sd[k]).abs().max().item()
        # bf16 compute + bf16 gradient reduction across ranks vs one rank on the global batch:
        # the SGD trajectories agree to a small fraction of how far the weights moved
        assert (a - b).abs().max().item() <= 0.05 * moved + 1e-5, (k, (a - b).abs().max().item(), moved)
    # replicas are bit-identical across ranks (DDP: every parameter; FSDP: the gathered state)
    parts = _gather_cpu(torch.cat([v.float().reshape(-1).cpu() for v in sd.values()]))
    assert all(torch.equal(parts[0], p) for p in parts), "replicas diverged"
    comm.destroy()


def _engine_fp32_worker(rank, ws, strategy):
    """Tight check of the multi-rank data path: fp32 native DDP / FSDP (IPC collectives, several
    buckets / units) on each rank's slice vs stock PyTorch fp32 training ONE process on the global
    batch (torch.optim.SGD with momentum).  In fp32 the only differences are summation order, so
    every weight must agree to ~1e-5 relative -- a comm bug that perturbs gradients by even 0.1 %
    fails here (the bf16 LM test above cannot resolve that)."""
    import copy

    import torch.nn as nn
    import torch.nn.functional as F

    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel
    from distributed_training_amd.parallel.ipc import IpcComm

    class Block(nn.Module):
        def __init__(self, d):
            super().__init__()
            self.l1, self.l2 = nn.Linear(d, 4 * d), nn.Linear(4 * d, d)

        def forward(self, x):
            return x + self.l2(torch.tanh(self.l1(x)))

    dev = _shared()
    torch.manual_seed(0)
    base = nn.Sequential(nn.Linear(32, 128), *[Block(128) for _ in range(3)], nn.Linear(128, 8)).to(dev)
    ref = copy.deepcopy(base)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    comm = IpcComm(rank, ws, dev)
    if strategy == "ddp":
        w = DistributedDataParallel(copy.deepcopy(base), comm=comm, device=dev, bucket_cap_mb=0.1,
                                    first_bucket_mb=0.02)
        assert len(w.buckets) >= 3
    else:
        w = FullyShardedDataParallel(copy.deepcopy(base), comm=comm, device=dev, wrap_policy={Block})
        assert len(w.units) == 4
    opt = FusedSGD(w.parameters(), lr=0.05, momentum=0.9)
    B = 16
    g = torch.Generator(device="cpu").manual_seed(9)
    for _ in range(4):
        X = torch.randn(ws * B, 32, generator=g).to(dev)
        Y = torch.randn(ws * B, 8, generator=g).to(dev)
        ref_opt.zero_grad()
        F.mse_loss(ref(X), Y).backward()
        ref_opt.step()
        opt.zero_grad()
        F.mse_loss(w(X[rank * B:(rank + 1) * B]), Y[rank * B:(rank + 1) * B]).backward()
        opt.step()
    torch.cuda.synchronize()
    comm.poll_errors()
    sd = w.full_state_dict(rank0_only=False) if strategy == "fsdp" else {
        k[len("module."):]: v for k, v in w.state_dict().items()}
    for k, v in ref.state_dict().items():
        torch.testing.assert_close(sd[k].float().cpu(), v.float().cpu(), rtol=2e-5, atol=2e-6)
    comm.destroy()


def _fsdp_llama_units_worker(rank, ws):
    """Llama-shaped FSDP with lm_wrap_policy on the GPU (IPC collectives): the embedding and the
    output head are units of their own (root: the final norm only), the embedding is never
    re-gathered for backward, no unit is left gathered after a step, and training matches the
    same engine on one rank with the global batch."""
    import torch.distributed as dist

    from distributed_training_amd.models.llama import Llama, LlamaConfig
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel, lm_wrap_policy
    from distributed_training_amd.parallel.ipc import IpcComm

    dev = _shared()
    cfg = LlamaConfig(n_layer=2, n_head=4, n_kv_head=2, n_embd=256, ffn_hidden=512, vocab_size=1024, block_size=128)
    B, T, steps = 2, 64, 3
    g = torch.Generator(device="cpu").manual_seed(21)
    glob = [torch.randint(0, 1024, (ws * B, T + 1), generator=g).to(dev) for _ in range(steps)]

    def run(comm, batches):
        torch.manual_seed(0)
        model = Llama(cfg).to(dev)
        w = FullyShardedDataParallel(model, comm=comm, device=dev, wrap_policy=lm_wrap_policy(model),
                                     param_dtype=torch.bfloat16)
        opt = FusedSGD(w.parameters(), lr=0.05, momentum=0.9)
        init = {k: v.float().cpu() for k, v in w.full_state_dict(rank0_only=False).items()}
        losses = []
        for xb in batches:
            opt.zero_grad()
            loss = w(xb[:, :-1], xb[:, 1:])
            loss.backward()
            opt.step()
            losses.append(float(loss.item()))
            assert comm.world_size == 1 or not any(u.gathered for u in w.units)
        return w, losses, init

    ref, ref_losses, init_sd = run(IpcComm(0, 1, dev, tag="llama_ref"), glob)
    ref_sd = {k: v.float().cpu() for k, v in ref.full_state_dict(rank0_only=False).items()}
    comm = IpcComm(rank, ws, dev, tag="llama")
    w, losses, _ = run(comm, [x[rank * B:(rank + 1) * B] for x in glob])
    names = [[n for _, _, n, _ in u.entries] for u in w.units]
    assert names[0] == ["tok_embeddings.weight"] and names[-2] == ["output.weight"] and names[-1] == ["norm.weight"]
    assert not w.units[0].bwd_needs_params
    l0 = torch.tensor([losses[0]])
    dist.all_reduce(l0)
    assert abs(l0.item() / ws - ref_losses[0]) < 1e-2 * abs(ref_losses[0])
    sd = w.full_state_dict(rank0_only=False)
    for k, v in sd.items():
        a, b = v.float().cpu(), ref_sd[k]
        moved = (b - init_sd[k]).abs().max().item()
        # bf16 compute + bf16 reduce-scatter vs one rank on the global batch (see _engine_worker)
        assert (a - b).abs().max().item() <= 0.05 * moved + 1e-5, (k, (a - b).abs().max().item(), moved)
    comm.destroy()


@pytest.mark.parametrize("ws", [2, 4])
def test_fsdp_llama_embedding_head_units_shared_gpu(ws):
    run_gloo(_fsdp_llama_units_worker, ws)


@pytest.mark.parametrize("ws", [2, 4, 8])
@pytest.mark.parametrize("strategy", ["ddp", "fsdp"])
def test_engines_fp32_multi_rank_vs_torch_global_batch(strategy, ws):
    run_gloo(_engine_fp32_worker, ws, strategy)


@pytest.mark.parametrize("ws", [2, 4, 8])
@pytest.mark.parametrize("strategy", ["ddp", "fsdp"])
def test_engines_multi_rank_shared_gpu(strategy, ws):
    run_gloo(_engine_worker, ws, strategy)


@pytest.mark.parametrize("ws", [2, 4])
def test_ddp_optimizer_in_backward_multi_rank_shared_gpu(ws):
    """DDP with the optimizer stepped per bucket inside the backward (overlap_optimizer):
    same trajectory as the one-rank reference, replicas bit-identical."""
    run_gloo(_engine_worker, ws, "ddp", True)


def _offload_worker(rank, ws, opt_name):
    from distributed_training_amd.parallel.comm import make_comm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    dev = _shared() if ws > 1 else torch.device("cuda", 0)
    comm = make_comm(dev) if ws > 1 else None

    def build():
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                                torch.nn.Linear(256, 8)).to(dev)
        return m

    g = torch.Generator().manual_seed(7 + rank)
    batches = [(torch.randn(16, 64, generator=g).to(dev), torch.randn(16, 8, generator=g).to(dev)) for _ in range(4)]
    finals = []
    for offload in (False, True):
        m = build()
        kw = {"comm": comm} if comm is not None else {}
        f = FullyShardedDataParallel(m, device=dev, wrap_policy={torch.nn.Linear}, cpu_offload=offload, **kw)
        assert all(p.device.type == ("cpu" if offload else "cuda") for p in f.parameters())
        opt = (torch.optim.SGD(f.parameters(), lr=0.05, momentum=0.9) if opt_name == "sgd"
               else torch.optim.AdamW(f.parameters(), lr=1e-2))
        for x, y in batches:
            opt.zero_grad(set_to_none=True)
            torch.nn.functional.mse_loss(f(x), y).backward()
            opt.step()
        sd = f.full_state_dict(rank0_only=False, offload_to_cpu=True)
        finals.append(torch.cat([v.reshape(-1).float() for v in sd.values()]))
    torch.testing.assert_close(finals[1], finals[0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("ws,opt_name", [(1, "sgd"), (1, "adamw"), (2, "adamw")])
def test_fsdp_cpu_offload_matches_device_shards(ws, opt_name):
    """FSDP with the fp32 shards, gradients and a torch optimizer in pinned host memory
    (the reference's CPUOffload(offload_params=True)) trains exactly like device shards."""
    if ws == 1:
        _offload_worker(0, 1, opt_name)
    else:
        run_gloo(_offload_worker, ws, opt_name)


def _routed_worker(rank, ws):
    """RoutedComm on the GPU: two IPC data planes of different configuration stand in for RCCL
    and the push plane (RCCL refuses two ranks on one GPU).  The calibration table is the same
    on every rank; with each route forced, every op is exact; routing follows the size classes."""
    import hashlib

    import torch.distributed as dist

    from distributed_training_amd.parallel.ipc import IpcComm
    from distributed_training_amd.parallel.routed import MiB, RoutedComm

    dev = _shared()
    prim = IpcComm(rank, ws, dev, tag="prim", slot_mb=1)
    fast = IpcComm(rank, ws, dev, tag="fast", slot_mb=8)
    rc = RoutedComm(prim, fast, sizes=(MiB, 4 * MiB), iters=2)
    sig = hashlib.sha256(repr(sorted(rc.routes().items())).encode()).digest()
    sigs = [None] * ws
    dist.all_gather_object(sigs, sig)
    assert all(s == sig for s in sigs), "ranks disagree on the route table"
    g = torch.Generator(device="cpu").manual_seed(7 + rank)
    for route in ("primary", "fast"):
        rc.table = {k: [route, route] for k in rc.table}
        before = rc.counts[route]
        for dt in (torch.float32, torch.bfloat16):
            for n in (1000, 600000):  # both size classes
                x = torch.randn(n, generator=g).to(dt).to(dev)
                parts = _gather_cpu(x)
                want = parts[0].clone()
                for p in parts[1:]:
                    want = want + p
                rc.all_reduce(x, "sum")
                torch.cuda.synchronize()
                assert torch.equal(x.cpu(), want.to(dt)), (route, dt, n)
                m = n // ws
                out = torch.empty(ws * m, dtype=dt, device=dev)
                rc.all_gather_into(out, torch.full((m,), float(rank + 1), dtype=dt, device=dev))
                o = torch.empty(m, dtype=dt, device=dev)
                rc.reduce_scatter_into(o, torch.ones(ws * m, dtype=dt, device=dev), "sum")
                torch.cuda.synchronize()
                assert torch.equal(out.cpu(), torch.arange(1, ws + 1).repeat_interleave(m).to(dt))
                assert torch.equal(o.cpu(), torch.full((m,), float(ws)).to(dt))
        assert rc.counts[route] == before + 12
    # the FSDP unit sizes are prepared at wrap (parallel/routed.py prepare): a 512 MiB all-gather and
    # reduce-scatter get a class calibrated on both planes before any step; then each route is forced and
    # checked exactly at that size, and no further class appears
    big = 256 << 20  # 256 Mi bf16 elements = 512 MiB
    added = rc.prepare([("all_gather", torch.bfloat16, 2 * big), ("reduce_scatter", torch.bfloat16, 2 * big)])
    assert added == [512 * MiB] and rc.sizes[-1] == 512 * MiB, rc.sizes
    n_classes = len(rc.sizes)
    for route in ("primary", "fast"):
        rc.table = {k: [route] * len(rc.sizes) for k in rc.table}
        y = torch.empty(big, dtype=torch.bfloat16, device=dev)
        rc.all_gather_into(y, torch.full((big // ws,), float(rank + 1), dtype=torch.bfloat16, device=dev))
        o = torch.empty(big // ws, dtype=torch.bfloat16, device=dev)
        rc.reduce_scatter_into(o, torch.ones(big, dtype=torch.bfloat16, device=dev), "sum")
        torch.cuda.synchronize()
        want = torch.arange(1, ws + 1, dtype=torch.bfloat16, device=dev).repeat_interleave(big // ws)
        assert torch.equal(y, want), route
        assert bool((o == float(ws)).all()), route
        del want
    assert len(rc.sizes) == n_classes
    del y, o
    rc.poll_errors()
    rc.destroy()


@pytest.mark.parametrize("ws", [2, 4])
def test_routed_comm_shared_gpu(ws):
    run_gloo(_routed_worker, ws)


def _graph_multirank_worker(rank, ws):
    """The whole DDP step (GPT-2 with several buckets, deferred grouped weight gradients, the
    bucket all-reduces on the IPC comm stream, fused AdamW) captured ONCE per rank as a hipGraph
    and replayed: losses and fp32 master weights bit-identical to the eager steps on the same
    batches on every rank, and identical across ranks (the replayed collectives really ran)."""
    import torch.distributed as dist

    from distributed_training_amd.engine.step_graph import GraphedStep
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops import lm
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.ipc import IpcComm

    dev = _shared()
    g = torch.Generator(device="cpu").manual_seed(40 + rank)  # different batches per rank
    data = [torch.randint(0, 1024, (2, 129), generator=g).to(dev) for _ in range(5)]
    seq = [data[0]] * 3 + data[1:]  # GraphedStep's 3 warm-up steps train on the static batch
    out = []
    for graphed in (False, True):
        torch.manual_seed(0)
        model = GPT2(GPT2Config(n_layer=2, n_head=4, n_embd=256, vocab_size=1024, block_size=256)).to(dev)
        comm = IpcComm(rank, ws, dev, tag=f"graph{int(graphed)}")
        ddp = DistributedDataParallel(model, comm=comm, device=dev, param_dtype=torch.bfloat16,
                                      bucket_cap_mb=0.5, first_bucket_mb=0.25)
        assert len(ddp.buckets) >= 4
        opt = FusedAdamW(ddp.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1)
        before = lm.GEMM_STATS["deferred_wgrad"]

        def step(xb):
            opt.zero_grad(set_to_none=True)
            loss = ddp(xb[:, :-1], xb[:, 1:])
            loss.backward()
            opt.step()
            return loss

        losses = []
        if graphed:
            gs = GraphedStep(step, [data[0].clone()], warmup=3, engine=ddp)
            assert gs.ok, gs.error
            for xb in seq[3:]:
                losses.append(gs(xb).float().clone())
        else:
            for xb in seq:
                losses.append(step(xb).float().clone())
            losses = losses[3:]
            assert lm.GEMM_STATS["deferred_wgrad"] > before  # the grouped deferred path is exercised
        torch.cuda.synchronize()
        comm.poll_errors()
        out.append((torch.stack(losses).cpu(), ddp.flat.master.clone()))
    assert torch.equal(out[0][0], out[1][0]), (rank, out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1]), rank
    # replicas identical across ranks (gradients were averaged by the replayed collectives)
    parts = _gather_cpu(out[1][1])
    assert all(torch.equal(p, parts[0]) for p in parts[1:])
    assert not torch.equal(out[1][1], out[0][1] * 0)  # (sanity: trained weights)
    dist.barrier()


@pytest.mark.parametrize("ws", [2, 4])
def test_step_graph_multirank_matches_eager(ws):
    run_gloo(_graph_multirank_worker, ws)


def _fsdp_overlap_bitwise_worker(rank, ws):
    """FSDP with AdamW stepped unit by unit inside the backward (overlap_optimizer) vs backward +
    step(), both at this world size over the IPC collectives: identical losses and shards."""
    from distributed_training_amd.models.gpt2 import GPT2
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel
    from distributed_training_amd.parallel.ipc import IpcComm

    dev = _shared()
    B, T, steps = 2, 64, 3
    g = torch.Generator(device="cpu").manual_seed(8)
    local = [torch.randint(0, 512, (ws * B, T + 1), generator=g)[rank * B:(rank + 1) * B].to(dev)
             for _ in range(steps)]
    comm = IpcComm(rank, ws, dev)
    finals = []
    for overlap in (False, True):
        w = FullyShardedDataParallel(_tiny_gpt2().to(dev), comm=comm, device=dev, wrap_policy={GPT2.block_class},
                                     param_dtype=torch.bfloat16)
        opt = FusedAdamW(w.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1)
        if overlap:
            assert w.overlap_optimizer(opt)
        losses = _train(w, opt, local, steps)
        comm.poll_errors()
        torch.cuda.synchronize()
        finals.append((losses, w.shards.master.clone(), w.shards.compute.clone()))
    assert finals[0][0] == finals[1][0]
    assert torch.equal(finals[0][1], finals[1][1]) and torch.equal(finals[0][2], finals[1][2])
    comm.destroy()


@pytest.mark.parametrize("ws", [2, 4])
def test_fsdp_optimizer_in_backward_multi_rank_shared_gpu(ws):
    """FSDP overlap_optimizer across ranks: each unit's shard updated on a side stream after its
    reduce-scatter, bit-identical to the plain step; and the same trajectory as the one-rank
    global-batch reference (_engine_worker)."""
    run_gloo(_fsdp_overlap_bitwise_worker, ws)
    run_gloo(_engine_worker, ws, "fsdp", True)


def _hsdp_worker(rank, ws, shard_size):
    """HYBRID sharding on the shared GPU (IPC communicators per shard / replica group): the same
    trajectory as the one-rank reference on the global batch, replicas identical across groups."""
    import torch.distributed as dist

    from distributed_training_amd.models.gpt2 import GPT2
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.comm import make_hybrid_comms
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel
    from distributed_training_amd.parallel.ipc import IpcComm

    dev = _shared()
    B, T, steps = 2, 64, 3
    g = torch.Generator(device="cpu").manual_seed(15)
    glob = [torch.randint(0, 512, (ws * B, T + 1), generator=g).to(dev) for _ in range(steps)]
    ref = FullyShardedDataParallel(_tiny_gpt2().to(dev), comm=IpcComm(0, 1, dev, tag="hsdp_ref"), device=dev,
                                   wrap_policy={GPT2.block_class}, param_dtype=torch.bfloat16)
    init_sd = {k: v.float().cpu().clone() for k, v in ref.full_state_dict(rank0_only=False).items()}
    _train(ref, FusedSGD(ref.parameters(), lr=0.05, momentum=0.9), glob, steps)
    ref_sd = {k: v.float().cpu() for k, v in ref.full_state_dict(rank0_only=False).items()}
    shard, rep = make_hybrid_comms(dev, shard_size)
    w = FullyShardedDataParallel(_tiny_gpt2().to(dev), comm=shard, device=dev, wrap_policy={GPT2.block_class},
                                 param_dtype=torch.bfloat16, replicate_comm=rep)
    assert w.rep is not None and w.world_size == shard_size
    _train(w, FusedSGD(w.parameters(), lr=0.05, momentum=0.9), [x[rank * B:(rank + 1) * B] for x in glob], steps)
    shard.poll_errors()
    rep.poll_errors()
    sd = {k: v.float().cpu() for k, v in w.full_state_dict(rank0_only=False).items()}
    for k, v in sd.items():
        moved = (ref_sd[k] - init_sd[k]).abs().max().item()
        assert (v - ref_sd[k]).abs().max().item() <= 0.05 * moved + 1e-5, k
    parts = _gather_cpu(torch.cat([v.reshape(-1) for v in sd.values()]))
    assert all(torch.equal(parts[0], p) for p in parts), "replicas diverged"
    dist.barrier()
    shard.destroy()
    rep.destroy()


@pytest.mark.parametrize("ws,shard_size", [(2, 1), (4, 2), (8, 4)])  # (2, 1): one rank per shard group
def test_hybrid_shard_shared_gpu(ws, shard_size):
    run_gloo(_hsdp_worker, ws, shard_size)


def _fsdp_graph_multirank_worker(rank, ws, arch):
    """FULL_SHARD at world size > 1 in a capture-safe form -- every unit gathers
    into a FIXED buffer (parallel/fsdp.py _GatherRing) instead of allocating and freeing its storage --
    so the whole step (per-unit IPC all-gathers with prefetch, reduce-scatters, deferred grouped weight
    gradients, fused AdamW) is captured ONCE per rank and replayed.  Three runs on the same batches:
    eager with the allocate-and-free storage (gather_ring=0), eager with the ring, and the replayed
    graph: losses and fp32 master shards bit-identical across all three, replicas consistent across
    ranks, and the capture policy (engine/step_graph.py) says yes for the IPC data plane."""
    import torch.distributed as dist

    from distributed_training_amd.engine.step_graph import GraphedStep, capture_policy
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.models.llama import Llama, LlamaConfig
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel, lm_wrap_policy
    from distributed_training_amd.parallel.ipc import IpcComm

    dev = _shared()
    g = torch.Generator(device="cpu").manual_seed(60 + rank)  # different batches per rank
    data = [torch.randint(0, 1024, (2, 129), generator=g).to(dev) for _ in range(5)]
    seq = [data[0]] * 3 + data[1:]  # GraphedStep's 3 warm-up steps train on the static batch

    def build():
        torch.manual_seed(0)
        if arch == "gpt2":
            return GPT2(GPT2Config(n_layer=3, n_head=4, n_embd=256, vocab_size=1024, block_size=256)).to(dev)
        return Llama(LlamaConfig(n_layer=3, n_head=4, n_kv_head=2, n_embd=256, ffn_hidden=512, vocab_size=1024,
                                 block_size=256)).to(dev)

    out = []
    # one communicator for the three runs (an IPC buffer freed and re-allocated in one process can come back
    # at the same address, whose dmabuf export the driver then refuses)
    comm = IpcComm(rank, ws, dev, tag=f"fsdpg_{arch}")
    for mode in ("resize", "ring", "graph"):
        model = build()
        w = FullyShardedDataParallel(model, comm=comm, device=dev, wrap_policy=lm_wrap_policy(model),
                                     param_dtype=torch.bfloat16, gather_ring=0 if mode == "resize" else 3)
        assert (w._ring is None) == (mode == "resize")
        ok, why = capture_policy(w)
        assert ok == (mode != "resize"), why
        opt = FusedAdamW(w.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1)

        def step(xb):
            opt.zero_grad(set_to_none=True)
            loss = w(xb[:, :-1], xb[:, 1:])
            loss.backward()
            opt.step()
            return loss

        losses = []
        if mode == "graph":
            gs = GraphedStep(step, [data[0].clone()], warmup=3, engine=w)
            assert gs.ok, gs.error
            for xb in seq[3:]:
                losses.append(gs(xb).float().clone())
        else:
            for xb in seq:
                losses.append(step(xb).float().clone())
                assert not any(u.gathered for u in w.units)
            losses = losses[3:]
        torch.cuda.synchronize()
        comm.poll_errors()
        out.append((torch.stack(losses).cpu(), w.shards.master.clone()))
        if mode == "graph":
            full = torch.cat([v.float().reshape(-1).cpu() for v in w.full_state_dict(rank0_only=False).values()])
    comm.destroy()
    for k in (1, 2):
        assert torch.equal(out[0][0], out[k][0]), (rank, k, out[0][0], out[k][0])
        assert torch.equal(out[0][1], out[k][1]), (rank, k)
    parts = _gather_cpu(full)  # the gathered model is the same on every rank
    assert all(torch.equal(p, parts[0]) for p in parts[1:])
    dist.barrier()


@pytest.mark.parametrize("ws", [2, 4])
@pytest.mark.parametrize("arch", ["gpt2", "llama"])
def test_fsdp_step_graph_multirank_matches_eager(arch, ws):
    run_gloo(_fsdp_graph_multirank_worker, ws, arch)
