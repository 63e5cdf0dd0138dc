"""Native DDP / FSDP engines vs torch references, multi-process gloo (CPU)."""
import copy
import os

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from tests.dist_utils import run_gloo


class Block(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.l1 = nn.Linear(d, 2 * d)
        self.l2 = nn.Linear(2 * d, d)

    def forward(self, x):
        return x + self.l2(torch.relu(self.l1(x)))


class Net(nn.Module):
    def __init__(self, unused=False):
        super().__init__()
        self.inp = nn.Linear(20, 16)
        self.blocks = nn.ModuleList([Block(16) for _ in range(3)])
        self.out = nn.Linear(16, 1)
        self.unused = nn.Linear(3, 3) if unused else None
        self.register_buffer("scale", torch.ones(1))

    def forward(self, x):
        x = self.inp(x)
        for b in self.blocks:
            x = b(x)
        return self.out(x) * self.scale


def _ddp_parity(rank, ws, bucket_mb, unused, accum):
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    base = Net(unused)
    m_ref, m_new = copy.deepcopy(base), copy.deepcopy(base)
    if rank == 1:  # different init on rank 1: the init broadcast must fix it
        with torch.no_grad():
            for p in m_new.parameters():
                p.add_(1.0)
    ref = nn.parallel.DistributedDataParallel(m_ref, find_unused_parameters=unused)
    new = DistributedDataParallel(m_new, TorchComm(), bucket_cap_mb=bucket_mb, first_bucket_mb=bucket_mb / 4)
    assert len(new.buckets) >= (2 if bucket_mb < 0.01 else 1)
    o1 = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    o2 = FusedSGD(new.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(100 + rank)
    for it in range(4):
        o1.zero_grad()
        o2.zero_grad(set_to_none=it % 2 == 0)  # both the steal + batched-copy and the in-place-accumulate paths
        for micro in range(accum):
            x = torch.randn(8, 20, generator=g)
            y = torch.randn(8, 1, generator=g)
            last = micro == accum - 1
            ctx1 = ref.no_sync() if not last else _null()
            ctx2 = new.no_sync() if not last else _null()
            with ctx1:
                F.mse_loss(ref(x), y).backward()
            with ctx2:
                F.mse_loss(new(x), y).backward()
        o1.step()
        o2.step()
    s1, s2 = ref.state_dict(), new.state_dict()
    assert list(s1.keys()) == list(s2.keys())
    assert all(k.startswith("module.") for k in s2)
    for k in s1:
        torch.testing.assert_close(s2[k], s1[k], rtol=1e-5, atol=1e-6, msg=k)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


@pytest.mark.parametrize("bucket_mb,unused,accum", [(25.0, False, 1), (0.004, False, 1), (0.004, True, 1),
                                                    (0.004, False, 2)])
def test_native_ddp_matches_torch_ddp(bucket_mb, unused, accum):
    run_gloo(_ddp_parity, 2, bucket_mb, unused, accum)


def _fsdp_parity(rank, ws, wrap, opt_name, accum=False):
    from distributed_training_amd.ops.optim import FusedAdamW, FusedSGD
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    torch.manual_seed(0)
    ref = Net()
    m = copy.deepcopy(ref)
    fs = FullyShardedDataParallel(m, TorchComm(), torch.device("cpu"), wrap_policy={Block} if wrap else None)
    assert len(fs.units) == (4 if wrap else 1)
    for u in fs.units:
        assert u.total % (ws * 64) == 0 and u.shard_size * ws == u.total
        assert u.alias == (ws == 1)
    if opt_name == "adamw":
        o1 = torch.optim.AdamW(ref.parameters(), lr=1e-2)
        o2 = FusedAdamW(fs.parameters(), lr=1e-2)
    else:
        o1 = torch.optim.SGD(ref.parameters(), lr=1e-1, momentum=0.9)
        o2 = FusedSGD(fs.parameters(), lr=1e-1, momentum=0.9)
    for it in range(4):
        g = torch.Generator().manual_seed(100 + it)
        X = torch.randn(8 * ws, 20, generator=g)
        Y = torch.randn(8 * ws, 1, generator=g)
        # accum: two micro-batches per step, alternating zero_grad(set_to_none) forms
        # (set_to_none writes the first micro-batch's gradient in place, later ones accumulate)
        none = it % 2 == 0 or not accum
        o1.zero_grad(set_to_none=none)
        o2.zero_grad(set_to_none=none)
        for mb in range(2 if accum else 1):
            lo, hi = (mb * 4, mb * 4 + 4) if accum else (0, 8)
            xs = torch.cat([X[r * 8 + lo:r * 8 + hi] for r in range(ws)])
            ys = torch.cat([Y[r * 8 + lo:r * 8 + hi] for r in range(ws)])
            F.mse_loss(ref(xs), ys).backward()
            F.mse_loss(fs(X[rank * 8 + lo:rank * 8 + hi]), Y[rank * 8 + lo:rank * 8 + hi]).backward()
        o1.step()
        o2.step()
    sd = fs.full_state_dict(rank0_only=False)
    rs = ref.state_dict()
    assert list(sd.keys()) == list(rs.keys())
    for k in rs:
        torch.testing.assert_close(sd[k], rs[k], rtol=1e-4, atol=1e-5, msg=k)
    # rank0_only: other ranks get nothing, and nobody hangs
    sd0 = fs.full_state_dict(rank0_only=True)
    assert (len(sd0) > 0) == (rank == 0)
    # load round trip into a fresh wrapper
    fs2 = FullyShardedDataParallel(Net(), TorchComm(), torch.device("cpu"), wrap_policy={Block} if wrap else None)
    fs2.load_state_dict(rs)
    for k, v in fs2.full_state_dict(rank0_only=False).items():
        torch.testing.assert_close(v, rs[k])
    # eval forward under no_grad works and matches
    with torch.no_grad():
        x = torch.randn(4, 20)
        torch.testing.assert_close(fs(x), ref(x), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("wrap,opt_name,accum", [(True, "adamw", False), (False, "sgd", False), (True, "sgd", False),
                                                (True, "sgd", True), (False, "adamw", True)])
def test_native_fsdp_matches_single_process(wrap, opt_name, accum):
    run_gloo(_fsdp_parity, 2, wrap, opt_name, accum)


def _fsdp_ws(rank, ws):
    _fsdp_parity(rank, ws, True, "adamw", False)


@pytest.mark.parametrize("wrap,opt_name,accum", [(True, "adamw", True), (False, "sgd", False)])
def test_native_fsdp_single_rank_aliases_shard(wrap, opt_name, accum):
    """World size 1: units point at the shard's compute copy instead of gathering
    a copy of it (NO_SHARD behaviour); training, accumulation, state dicts still match."""
    run_gloo(_fsdp_parity, 1, wrap, opt_name, accum)


@pytest.mark.parametrize("ws", [4, 8])
def test_native_fsdp_world(ws):
    """4 and 8 ranks (the 8-GPU node's rank count) over gloo: shard padding, gathers,
    reduce-scatters and the full state dict at every world size the bench runs."""
    run_gloo(_fsdp_ws, ws)


def _clip_parity(rank, ws, strategy):
    """Global-norm clipping: each rank's shard (FSDP) / replica (DDP) scaled by the
    coefficient of the WHOLE gradient, as torch's clip_grad_norm_ on one process."""
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    torch.manual_seed(0)
    ref = Net()
    m = copy.deepcopy(ref)
    if strategy == "fsdp":
        w = FullyShardedDataParallel(m, TorchComm(), torch.device("cpu"), wrap_policy={Block})
    else:
        w = DistributedDataParallel(m, TorchComm())
    g = torch.Generator().manual_seed(3)
    X, Y = torch.randn(8 * ws, 20, generator=g), torch.randn(8 * ws, 1, generator=g)
    F.mse_loss(ref(X), Y).backward()
    F.mse_loss(w(X[rank * 8:(rank + 1) * 8]), Y[rank * 8:(rank + 1) * 8]).backward()
    want = torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.05)
    got = w.clip_grad_norm_(0.05)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)
    assert float(want) > 0.05  # the clip is active
    o1 = torch.optim.SGD(ref.parameters(), lr=1.0)
    o2 = torch.optim.SGD(w.parameters(), lr=1.0)
    o1.step()
    o2.step()
    sd = w.full_state_dict(rank0_only=False) if strategy == "fsdp" else {
        k[len("module."):]: v for k, v in w.state_dict().items()}
    for k, v in ref.state_dict().items():
        torch.testing.assert_close(sd[k], v, rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.parametrize("strategy", ["fsdp", "ddp"])
def test_clip_grad_norm_global(strategy):
    run_gloo(_clip_parity, 2, strategy)


def _comm_ops(rank, ws):
    from distributed_training_amd.parallel.comm import TorchComm

    c = TorchComm()
    t = torch.full((6,), float(rank + 1))
    c.all_reduce(t, op="avg")
    assert torch.allclose(t, torch.full((6,), (ws + 1) / 2))
    out = torch.empty(ws * 3)
    c.all_gather_into(out, torch.full((3,), float(rank)))
    assert torch.equal(out, torch.arange(ws).repeat_interleave(3).float())
    rs = torch.empty(3)
    c.reduce_scatter_into(rs, torch.ones(ws * 3), op="avg")
    assert torch.allclose(rs, torch.ones(3))
    b = torch.full((2,), float(rank))
    w = c.broadcast(b, src=1, async_op=True)
    w.wait()
    assert torch.equal(b, torch.ones(2))
    c.barrier()


def test_torch_comm_collectives():
    run_gloo(_comm_ops, 3)


class CkptNet(Net):
    def forward(self, x):
        from torch.utils.checkpoint import checkpoint

        x = self.inp(x)
        for b in self.blocks:
            x = checkpoint(b, x, use_reentrant=False)
        return self.out(x) * self.scale


def _fsdp_ckpt(rank, ws):
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    torch.manual_seed(0)
    ref = CkptNet()
    m = copy.deepcopy(ref)
    fs = FullyShardedDataParallel(m, TorchComm(), torch.device("cpu"), wrap_policy={Block})
    o1 = torch.optim.SGD(ref.parameters(), lr=0.1)
    o2 = FusedSGD(fs.parameters(), lr=0.1)
    for it in range(3):
        g = torch.Generator().manual_seed(7 + it)
        X, Y = torch.randn(8 * ws, 20, generator=g), torch.randn(8 * ws, 1, generator=g)
        o1.zero_grad()
        F.mse_loss(ref(X), Y).backward()
        o1.step()
        o2.zero_grad()
        F.mse_loss(fs(X[rank * 8:(rank + 1) * 8]), Y[rank * 8:(rank + 1) * 8]).backward()
        o2.step()
    for k, v in fs.full_state_dict(rank0_only=False).items():
        torch.testing.assert_close(v, ref.state_dict()[k], rtol=1e-4, atol=1e-5, msg=k)


def test_native_fsdp_with_activation_checkpointing():
    run_gloo(_fsdp_ckpt, 2)


def _fsdp_tied(rank, ws):
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    torch.manual_seed(0)
    cfg = GPT2Config(n_layer=2, n_head=2, n_embd=32, vocab_size=100, block_size=16)
    ref = GPT2(cfg)
    m = copy.deepcopy(ref)
    fs = FullyShardedDataParallel(m, TorchComm(), torch.device("cpu"), wrap_policy={GPT2.block_class})
    o1 = torch.optim.AdamW(ref.parameters(), lr=1e-2)
    o2 = FusedAdamW(fs.parameters(), lr=1e-2)
    g = torch.Generator().manual_seed(3)
    X = torch.randint(0, 100, (4 * ws, 17), generator=g)
    for it in range(3):
        o1.zero_grad()
        lo = ref(X[:, :-1])
        F.cross_entropy(lo.reshape(-1, lo.shape[-1]), X[:, 1:].reshape(-1)).backward()
        o1.step()
        o2.zero_grad()
        xs = X[rank * 4:(rank + 1) * 4]
        lo2 = fs(xs[:, :-1])
        F.cross_entropy(lo2.reshape(-1, lo2.shape[-1]), xs[:, 1:].reshape(-1)).backward()
        o2.step()
    sd = fs.full_state_dict(rank0_only=False)
    rs = ref.state_dict()
    assert set(sd) == set(rs) and "lm_head.weight" in sd
    for k in rs:
        torch.testing.assert_close(sd[k], rs[k], rtol=1e-4, atol=1e-5, msg=k)


def test_native_fsdp_tied_weights_gpt2():
    run_gloo(_fsdp_tied, 2)


def _resume_parity(rank, ws, strategy, opt_name, tmpdir):
    """Checkpoint with OPTIM_STATE mid-training, resume into fresh engine + optimizer:
    the continued run matches an uninterrupted one (momentum / Adam moments and
    step restored; FSDP's per-rank shards gathered and re-sharded)."""
    import torch.distributed as dist

    from distributed_training_amd.engine.checkpoint import ModelCheckpoint
    from distributed_training_amd.ops.optim import FusedAdamW, FusedSGD
    from distributed_training_amd.parallel.strategy import DDPStrategy, FSDPStrategy

    class Env:
        global_rank = rank

        @staticmethod
        def barrier():
            dist.barrier()

    def make():
        torch.manual_seed(0)
        strat = FSDPStrategy(False, wrap_policy={Block}) if strategy == "fsdp" else DDPStrategy(0, False)
        w = strat.prepare_model(Net(), torch.device("cpu"))
        o = FusedAdamW(w.parameters(), lr=1e-2) if opt_name == "adamw" else FusedSGD(w.parameters(), lr=0.1,
                                                                                        momentum=0.9)
        return strat, w, o

    def steps(w, o, its):
        for it in its:
            g = torch.Generator().manual_seed(200 + it)
            X, Y = torch.randn(8 * ws, 20, generator=g), torch.randn(8 * ws, 1, generator=g)
            o.zero_grad()
            F.mse_loss(w(X[rank * 8:(rank + 1) * 8]), Y[rank * 8:(rank + 1) * 8]).backward()
            o.step()

    def state(strat, w):
        return strat.model_state(w) if strategy == "fsdp" else w.state_dict()

    strat, w, o = make()
    steps(w, o, range(6))
    want = state(strat, w)
    strat, w, o = make()
    steps(w, o, range(3))
    ck = ModelCheckpoint(f"{tmpdir}/snap.pt", Env, strat, save_optimizer=True)
    ck.save(w, 3, o)
    strat2, w2, o2 = make()
    w2, ep = ck.load(w2, "cpu", o2)
    assert ep == 3
    steps(w2, o2, range(3, 6))
    got = state(strat2, w2)
    if rank == 0 or strategy == "ddp":
        for k in want:
            torch.testing.assert_close(got[k], want[k], rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.parametrize("strategy,opt_name", [("fsdp", "adamw"), ("fsdp", "sgd"), ("ddp", "adamw"),
                                               ("ddp", "sgd")])
def test_resume_restores_optimizer_state(strategy, opt_name, tmp_path):
    run_gloo(_resume_parity, 2, strategy, opt_name, str(tmp_path))


@pytest.mark.parametrize("cap, first, want_first", [(25, "auto", 1.0), (25, None, 1.0), (25, 2, 2.0),
                                                    ("auto", "auto", None)])
def test_ddp_bucket_caps_numeric_cap_with_auto_first(cap, first, want_first):
    """A numeric ``bucket_cap_mb`` with ``first_bucket_mb: auto`` (the shipped default of
    conf/train/default.yaml) keeps torch's 1 MiB first bucket instead of failing on float("auto")."""
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.ddp import MiB, DistributedDataParallel

    model = nn.Sequential(nn.Linear(20, 64), nn.ReLU(), nn.Linear(64, 1))
    ddp = DistributedDataParallel(model, comm=TorchComm(), bucket_cap_mb=cap, first_bucket_mb=first)
    first_b, cap_b = ddp.bucket_bytes
    if want_first is not None:
        assert first_b == int(want_first * MiB) and cap_b == int(float(cap) * MiB)


def test_forward_generation_two_forwards_one_backward():
    """Two forwards before one backward: a weight used once in each is NOT single-use for the
    coming backward (its gradient must not be deferred)."""
    from distributed_training_amd.ops import lm

    w = torch.zeros(4, requires_grad=True)
    lm.new_forward_generation()
    lm._count_use(w)
    assert lm._single_use(w)
    lm.new_forward_generation()  # second forward, first backward not run yet
    lm._count_use(w)
    assert not lm._single_use(w)
    lm.close_forward_generations()  # the backward finished
    lm.new_forward_generation()
    lm._count_use(w)
    assert lm._single_use(w)
    lm.new_forward_generation()  # a no-grad forward in between counts nothing and closes itself
    lm.close_forward_generations()
    lm.new_forward_generation()
    lm._count_use(w)
    assert lm._single_use(w)
    lm.abandon_step()


def _tiny_llama():
    from distributed_training_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(0)
    return Llama(LlamaConfig(n_layer=2, n_head=4, n_kv_head=2, n_embd=32, ffn_hidden=64, vocab_size=96,
                             block_size=16))


def _fsdp_llama_units(rank, ws, steps):
    """lm_wrap_policy: blocks, the embedding and the output head are units of their own (the
    root keeps only the final norm); training matches one process on the global batch."""
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel, lm_wrap_policy

    ref = _tiny_llama()
    model = _tiny_llama()
    fs = FullyShardedDataParallel(model, comm=TorchComm(), wrap_policy=lm_wrap_policy(model))
    names = [[n for _, _, n, _ in u.entries] for u in fs.units]
    assert names[0] == ["tok_embeddings.weight"] and names[-2] == ["output.weight"], names
    assert names[-1] == ["norm.weight"] and fs.units[-1].is_root
    assert len(fs.units) == 2 + 2 + 1
    assert not fs.units[0].bwd_needs_params and fs.units[-2].bwd_needs_params
    o_ref = FusedAdamW(ref.parameters(), lr=1e-2)
    o_fs = FusedAdamW(fs.parameters(), lr=1e-2)
    B, S = 2, 8
    for it in range(steps):
        g = torch.Generator().manual_seed(300 + it)
        X = torch.randint(0, 96, (B * ws, S + 1), generator=g)
        o_ref.zero_grad()
        ref(X[:, :-1], X[:, 1:]).backward()
        o_ref.step()
        o_fs.zero_grad()
        xb = X[rank * B:(rank + 1) * B]
        fs(xb[:, :-1], xb[:, 1:]).backward()
        o_fs.step()
        # after backward no unit is left gathered (the head kept for backward was freed)
        assert ws == 1 or not any(u.gathered for u in fs.units)
    sd = fs.full_state_dict(rank0_only=False)
    for k, v in ref.state_dict().items():
        if k in sd:
            torch.testing.assert_close(sd[k], v, rtol=2e-4, atol=2e-5, msg=k)


@pytest.mark.parametrize("ws", [2, 4])
def test_native_fsdp_llama_embedding_head_units(ws):
    run_gloo(_fsdp_llama_units, ws, 3)


def _routed_cpu(rank, ws):
    """RoutedComm mechanics over two gloo data planes: a calibrated table identical on every
    rank, messages routed by (op, dtype, size class), results exact on both routes."""
    import hashlib

    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.routed import MiB, RoutedComm

    rc = RoutedComm(TorchComm(), TorchComm(), sizes=(MiB // 16, MiB // 4), iters=2, lazy_max=0)
    sig = hashlib.sha256(repr(sorted(rc.routes().items())).encode()).digest()
    sigs = [None] * ws
    dist.all_gather_object(sigs, sig)
    assert all(s == sig for s in sigs), "ranks disagree on the route table"
    for table_route in ("primary", "fast"):
        rc.table = {k: [table_route] * 2 for k in rc.table}
        before = dict(rc.counts)
        for n in (1000, 50000):  # both size classes (4 KB, 200 KB of fp32)
            x = torch.arange(n, dtype=torch.float32) + rank
            rc.all_reduce(x, "sum")
            assert torch.equal(x, 2 * torch.arange(n, dtype=torch.float32) + sum(range(ws)))
            out = torch.empty(ws * n)
            rc.all_gather_into(out, torch.full((n,), float(rank)))
            assert torch.equal(out, torch.arange(ws).repeat_interleave(n).float())
            o = torch.empty(n)
            rc.reduce_scatter_into(o, torch.ones(ws * n), "sum")
            assert torch.equal(o, torch.full((n,), float(ws)))
        assert rc.counts[table_route] == before[table_route] + 6
    # max is never routed to the fast plane
    rc.table = {k: ["fast"] * 2 for k in rc.table}
    before = dict(rc.counts)
    y = torch.tensor([float(rank)])
    rc.all_reduce(y, "max")
    assert float(y) == ws - 1 and rc.counts == before


def test_routed_comm_cpu():
    run_gloo(_routed_cpu, 2)


def _routed_prepare_cpu(rank, ws):
    """The engines hand their message sizes to RoutedComm.prepare when they wrap the model: every
    message past the default classes gets a class calibrated THEN (the DDP buckets here), and the
    training steps that follow add none (no in-step calibration, verdict r4 item 6)."""
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.routed import MiB, RoutedComm

    rc = RoutedComm(TorchComm(), TorchComm(), sizes=(MiB // 64,), iters=1)
    added = rc.prepare([("all_reduce", torch.float32, 100_000), ("all_gather", torch.float32, 99_000),
                        ("reduce_scatter", torch.float32, 1000), ("broadcast", torch.float32, 10 ** 6)])
    assert added == [102_400] and rc.sizes == [MiB // 64, 102_400], rc.sizes  # one class, 4 KB multiple
    assert [e["when"] for e in rc.prepared_log] == ["at wrap"]
    assert set(rc.prepared_log[0]["routes"]) == {"all_gather float32", "all_reduce float32"}
    assert rc.prepare([("all_reduce", torch.float32, 100_000)]) == []  # already covered
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 512))
    ddp = DistributedDataParallel(net, comm=rc, bucket_cap_mb=0.3, first_bucket_mb=0.05)
    sizes = sorted((b.end - b.start) * 4 for b in ddp.buckets)
    assert sizes[-1] > MiB // 64  # a bucket past the default class: prepared at wrap
    n_classes = len(rc.sizes)
    assert n_classes > 2
    g = torch.Generator().manual_seed(rank)
    for _ in range(2):
        ddp.zero_grad()
        ddp(torch.randn(8, 64, generator=g)).square().mean().backward()
    assert len(rc.sizes) == n_classes, "a class was calibrated inside a training step"
    assert all(e["when"] == "at wrap" for e in rc.prepared_log)


def test_routed_prepare_at_wrap_cpu():
    run_gloo(_routed_prepare_cpu, 2)


def _routed_lazy_cpu(rank, ws):
    """A message larger than every size class adds a class of its own on first use (calibrated for every
    op / dtype on all ranks at the same point), kept sorted; the same table on every rank; a calibration
    failure on ONE rank (at one key) sends every rank to the primary plane without a hang."""
    import hashlib

    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.routed import MiB, RoutedComm

    rc = RoutedComm(TorchComm(), TorchComm(), sizes=(MiB // 16,), iters=1)
    x = torch.ones(100_000) * (rank + 1)  # 400 KB > 64 KB: a 512 KB class
    rc.all_reduce(x, "sum")
    assert torch.equal(x, torch.full((100_000,), float(sum(range(1, ws + 1)))))
    assert rc.sizes == [MiB // 16, MiB // 2] and all(len(v) == 2 for v in rc.table.values())
    sig = hashlib.sha256(repr(sorted(rc.routes().items())).encode()).digest()
    sigs = [None] * ws
    dist.all_gather_object(sigs, sig)
    assert all(s == sig for s in sigs)
    out = torch.empty(ws * 30_000)  # 120 KB * ws: inside the new class, no further calibration
    rc.all_gather_into(out, torch.full((30_000,), float(rank)))
    assert rc.sizes == [MiB // 16, MiB // 2]

    class Broken(TorchComm):
        # rank 1's data plane fails; rank 0's bounded peer wait (IpcComm: timeout_iters) then fails the
        # same collective -- emulated by raising on both ranks at that call
        def all_gather_into(self, out, inp, async_op=False):
            raise RuntimeError("injected data-plane failure" if rank == 1 else "peer wait timed out")

    rb = RoutedComm(TorchComm(), Broken(), sizes=(MiB // 16,), iters=1)
    assert rb.failed and all(r == "primary" for v in rb.table.values() for r in v)


def test_routed_comm_lazy_classes_cpu():
    run_gloo(_routed_lazy_cpu, 2)



def _fsdp_reduce_dtype_worker(rank, ws, out):
    """bf16 FSDP gradients after one backward, reduce-scattered in bf16 (the default: torch
    MixedPrecision(param_dtype=reduce_dtype=bf16)) and with reduce_dtype=fp32, against the fp64 mean of
    every rank's local bf16 gradients (each rank recomputes all ranks' local gradients with a plain bf16
    copy of the model)."""
    import torch.distributed as dist

    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    torch.manual_seed(0)
    base = Net()
    g = torch.Generator().manual_seed(11)
    B = 16
    X, Y = torch.randn(B * ws, 20, generator=g), torch.randn(B * ws, 1, generator=g)
    ref = {}
    for r in range(ws):
        m = copy.deepcopy(base).bfloat16()
        F.mse_loss(m(X[r * B:(r + 1) * B].bfloat16()).float(), Y[r * B:(r + 1) * B]).backward()
        for n, p in m.named_parameters():
            ref[n] = ref.get(n, 0) + p.grad.double() / ws
    errs = {}
    for rd in (None, torch.float32):
        fs = FullyShardedDataParallel(copy.deepcopy(base), TorchComm(), torch.device("cpu"), wrap_policy={Block},
                                      param_dtype=torch.bfloat16, reduce_dtype=rd)
        assert fs.shards.grad_dtype == (rd or torch.bfloat16)
        F.mse_loss(fs(X[rank * B:(rank + 1) * B].bfloat16()).float(), Y[rank * B:(rank + 1) * B]).backward()
        err = scale = 0.0
        for u in fs.units:
            full = torch.zeros(u.total, dtype=torch.float64)
            for (_, _, name, _), o, n in zip(u.entries, u.offsets, u.numels):
                full[o:o + n] = ref[name].reshape(-1)
            want = full[rank * u.shard_size:(rank + 1) * u.shard_size]
            got = fs.shards.grad_view(fs.shards.index_of(u.shard_param)).double()
            err = max(err, (got - want).abs().max().item())
            scale = max(scale, want.abs().max().item())
        t = torch.tensor([err, scale], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        errs["bf16" if rd is None else "fp32"] = t[0].item() / t[1].item()
    if rank == 0:
        out.put(errs)


@pytest.mark.parametrize("ws", [2, 8])
def test_fsdp_reduce_dtype_pins_bf16_reduction_error(ws):
    """FSDP reduce_dtype (torch MixedPrecision.reduce_dtype): with fp32 the reduce-scattered gradient is
    the fp64 mean of the ranks' bf16 gradients up to fp32 rounding; the default bf16 reduction's extra
    error (a rounding per partial sum: RCCL's ring rounds at every hop, gloo here) stays within a few
    bf16 ulps of the largest gradient at 8 ranks -- the bound this test pins."""
    import multiprocessing as mp

    q = mp.get_context("spawn").SimpleQueue()
    run_gloo(_fsdp_reduce_dtype_worker, ws, q)
    errs = q.get()
    print(f"ws={ws} max rel. gradient error vs the fp64 mean: {errs}")
    assert errs["fp32"] < 1e-6, errs
    assert errs["bf16"] < 2 ** -7, errs
    assert errs["fp32"] < errs["bf16"], errs


def _hsdp_worker(rank, ws, shard_size, opt_name):
    """HYBRID sharding over gloo: shard groups of ``shard_size`` ranks, replicas across them; every
    rank trains on its own micro-batch and the result matches one process on the global batch."""
    from distributed_training_amd.ops.optim import FusedAdamW, FusedSGD
    from distributed_training_amd.parallel.comm import make_hybrid_comms
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    torch.manual_seed(0)
    ref = Net()
    m = copy.deepcopy(ref)
    if rank % 2:  # replicas start from replica 0 (sync_module_states), whatever their own init
        with torch.no_grad():
            for p in m.parameters():
                p.add_(0.25)
        torch.manual_seed(0)
        m = copy.deepcopy(ref) if shard_size > 1 and rank % shard_size else m
    shard, rep = make_hybrid_comms(torch.device("cpu"), shard_size)
    assert shard.world_size == shard_size and rep.world_size == ws // shard_size
    fs = FullyShardedDataParallel(m, shard, torch.device("cpu"), wrap_policy={Block}, replicate_comm=rep)
    assert (fs.rep is None) == (ws // shard_size == 1)
    if opt_name == "adamw":
        o1, o2 = torch.optim.AdamW(ref.parameters(), lr=1e-2), FusedAdamW(fs.parameters(), lr=1e-2)
    else:
        o1 = torch.optim.SGD(ref.parameters(), lr=1e-1, momentum=0.9)
        o2 = FusedSGD(fs.parameters(), lr=1e-1, momentum=0.9)
    for it in range(3):
        g = torch.Generator().manual_seed(200 + it)
        X, Y = torch.randn(8 * ws, 20, generator=g), torch.randn(8 * ws, 1, generator=g)
        o1.zero_grad(set_to_none=True)
        o2.zero_grad(set_to_none=True)
        F.mse_loss(ref(X), Y).backward()
        F.mse_loss(fs(X[rank * 8:(rank + 1) * 8]), Y[rank * 8:(rank + 1) * 8]).backward()
        o1.step()
        o2.step()
    sd = fs.full_state_dict(rank0_only=False)
    for k, v in ref.state_dict().items():
        torch.testing.assert_close(sd[k], v, rtol=1e-4, atol=1e-5, msg=k)
    # rank0_only: only the global rank 0 keeps the state dict
    sd0 = fs.full_state_dict(rank0_only=True)
    assert (len(sd0) > 0) == (rank == 0)


@pytest.mark.parametrize("ws,shard_size,opt_name", [(4, 2, "adamw"), (4, 2, "sgd"), (8, 4, "adamw"), (4, 1, "sgd"),
                                                    (4, 4, "adamw")])
def test_hybrid_shard_matches_single_process(ws, shard_size, opt_name):
    """HSDP (torch HYBRID_SHARD): FSDP within shard groups (one node's GPUs: xGMI gathers and
    reduce-scatters), one gradient all-reduce across the replica groups (the inter-node fabric);
    also the degenerate sizes 1 (pure replication) and ws (plain FULL_SHARD)."""
    run_gloo(_hsdp_worker, ws, shard_size, opt_name)


def test_hybrid_shard_strategy_from_config():
    """train.fsdp_sharding=hybrid / hybrid_shard_size map onto the FSDP strategy."""
    from pathlib import Path

    from distributed_training_amd.app import training_config_from
    from distributed_training_amd.config import compose
    from distributed_training_amd.parallel.strategy import FSDPStrategy

    conf = Path(__file__).resolve().parent.parent / "conf"
    cfg = compose(conf, "config", ["train.parallel_strategy=fsdp", "+train.fsdp_sharding=hybrid",
                                   "+train.hybrid_shard_size=2"])
    tc = training_config_from(cfg)
    assert tc.fsdp_sharding == "hybrid" and int(tc.hybrid_shard_size) == 2
    st = FSDPStrategy(False, sharding=tc.fsdp_sharding, hybrid_shard_size=tc.hybrid_shard_size)
    assert st.sharding == "hybrid"
    with pytest.raises(ValueError):
        FSDPStrategy(False, sharding="hsdp2")


def test_capture_policy_routes():
    """ONE capture policy (engine/step_graph.py capture_policy) for the Trainer and
    bench_lm.py -- at world size > 1 the whole-step hipGraph is used only when every collective of the
    step routes to the IPC data plane (RCCL-in-graph replay is unverified on a multi-GPU node: opt-in
    DTA_GRAPH_RCCL=1); process-group calls never; one rank always (if the engine state allows)."""
    from types import SimpleNamespace

    from distributed_training_amd.engine.step_graph import capture_policy
    from distributed_training_amd.parallel.comm import RcclComm, TorchComm
    from distributed_training_amd.parallel.ipc import IpcComm
    from distributed_training_amd.parallel.routed import MiB, RoutedComm

    def stub(cls):
        c = cls.__new__(cls)
        c.rank, c.world_size, c.device = 0, 2, torch.device("cpu")
        return c

    rc = RoutedComm(stub(RcclComm), stub(IpcComm), sizes=(MiB, 16 * MiB), calibrate=False)
    msgs = [("all_reduce", torch.bfloat16, MiB // 4), ("all_reduce", torch.bfloat16, 6 * MiB)]
    eng = SimpleNamespace(graph_capturable=lambda: True, world_size=2, comm=rc, step_messages=lambda: msgs)
    rc.table[("all_reduce", torch.bfloat16)] = ["fast", "fast"]
    assert capture_policy(eng)[0]
    rc.table[("all_reduce", torch.bfloat16)] = ["fast", "primary"]  # the 6 MB bucket goes to RCCL
    ok, why = capture_policy(eng)
    assert not ok and "RCCL" in why
    os.environ["DTA_GRAPH_RCCL"] = "1"
    try:
        assert capture_policy(eng)[0]
    finally:
        del os.environ["DTA_GRAPH_RCCL"]
    eng.comm = TorchComm()  # gloo / torch process group: never captured
    assert not capture_policy(eng)[0]
    eng.world_size = 1
    assert capture_policy(eng)[0]
    eng.graph_capturable = lambda: False  # e.g. FSDP with CPU offload
    assert not capture_policy(eng)[0]


def _fsdp_ring_vs_resize(rank, ws):
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    finals = []
    for ring in (0, 3, 2):
        for raf in (True, False):
            torch.manual_seed(0)
            m = CkptNet() if raf else Net()
            fs = FullyShardedDataParallel(m, TorchComm(), torch.device("cpu"), wrap_policy={Block}, gather_ring=ring,
                                          reshard_after_forward=raf)
            assert (fs._ring is None) == (ring == 0) and len(fs.units) >= 3
            if ring:
                assert len(fs._ring.bufs) == ring and fs.graph_capturable()
            opt = FusedSGD(fs.parameters(), lr=0.1, momentum=0.9)
            for it in range(3):
                g = torch.Generator().manual_seed(11 + it)
                X, Y = torch.randn(8 * ws, 20, generator=g), torch.randn(8 * ws, 1, generator=g)
                opt.zero_grad()
                F.mse_loss(fs(X[rank * 8:(rank + 1) * 8]), Y[rank * 8:(rank + 1) * 8]).backward()
                opt.step()
                assert not any(u.gathered for u in fs.units if not u.is_root)
            finals.append((ring, raf, torch.cat([v.reshape(-1) for v in fs.full_state_dict(rank0_only=False).values()])))
    base = {raf: t for ring, raf, t in finals if ring == 0}
    for ring, raf, t in finals:
        assert torch.equal(t, base[raf]), (ring, raf)


def test_fsdp_gather_ring_matches_allocate_and_free():
    """parallel/fsdp.py _GatherRing (fixed gather buffers at world size > 1, 2 or 3 slots) trains bit-identically
    to the allocate-and-free unit storage, with prefetch, activation checkpointing (re-gathered units) and
    reshard_after_forward off (units evicted from a shared slot and re-gathered for backward)."""
    run_gloo(_fsdp_ring_vs_resize, 3)


def _bench_comm_fallback(rank, ws):
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import bench
    from distributed_training_amd.parallel import comm as comm_mod

    def refuse(*a, **k):
        raise RuntimeError("could not load librccl: test")

    orig = comm_mod.make_comm
    comm_mod.make_comm = refuse
    try:
        c = bench.bench_comm(torch.device("cpu"))
    finally:
        comm_mod.make_comm = orig
    assert c.name == "torch" and c.world_size == ws
    t = torch.full((3,), float(rank + 1))
    c.all_reduce(t, op="sum")
    assert t.tolist() == [float(sum(range(1, ws + 1)))] * 3


def test_bench_comm_falls_back_to_torch_distributed():
    """bench.py at N > 1: a native communicator that cannot come up on the ranks leaves the run on
    torch.distributed's process group instead of ending it (the JSON's ``comm`` names the one that ran)."""
    run_gloo(_bench_comm_fallback, 2)
