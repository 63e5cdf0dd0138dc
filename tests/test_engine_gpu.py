"""End-to-end GPU tests of the engines on one MI355X (RCCL world size 1)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _dev():
    return torch.device("cuda", 0)


def _setup(hidden=512, size=256, batch=32, momentum=0.0, graph_steps=4, persistent=None):
    from distributed_training_amd.data.datasets import DeviceDataLoader, MyTrainDataset
    from distributed_training_amd.engine.fused_mlp import FusedMLPProgram
    from distributed_training_amd.models.mlp import MLP
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.sampler import DistributedSampler

    dev = _dev()
    torch.manual_seed(0)
    ds = MyTrainDataset(size, 20, 1, seed=0)
    model = MLP(20, hidden, 1).to(dev)
    ref = MLP(20, hidden, 1).to(dev)
    ref.load_state_dict(model.state_dict())
    comm = RcclComm(0, 1, dev)
    ddp = DistributedDataParallel(model, comm=comm, device=dev)
    opt = FusedSGD(ddp.parameters(), lr=0.05, momentum=momentum)
    loader = DeviceDataLoader(ds, batch, sampler=DistributedSampler(ds, num_replicas=1, rank=0, seed=3), device=dev)
    prog = FusedMLPProgram(model, opt, loader, comm, loss="mse", graph_steps=graph_steps, persistent=persistent)
    return ds, model, ref, prog, loader


@pytest.mark.parametrize("momentum,size,batch,persistent", [(0.0, 256, 32, None), (0.9, 256, 32, None),
                                                             (0.0, 256, 32, False), (0.9, 200, 32, None),
                                                             (0.0, 96, 64, None)])
def test_fused_program_matches_torch_sgd(momentum, size, batch, persistent):
    """Fused program (persistent single-workgroup loop, or eager + hipGraph
    replays across epoch boundaries with partial last batches) vs a plain fp32
    torch training loop over the same batches."""
    ds, model, ref, prog, loader = _setup(size=size, batch=batch, momentum=momentum, persistent=persistent)
    assert prog.persistent == (persistent is None and size % batch == 0 and batch <= 32)
    opt_ref = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=momentum)
    n_epochs = 3
    ref_losses = []
    for ep in range(n_epochs):
        loader.sampler.set_epoch(ep)
        for x, y in loader:
            opt_ref.zero_grad()
            loss = F.mse_loss(ref(x), y)
            loss.backward()
            opt_ref.step()
            ref_losses.append(loss.item())
    for ep in range(n_epochs):
        prog.run_epoch(ep)
    prog.store_to_module()
    torch.cuda.synchronize()
    got = prog.last_losses(len(ref_losses)).cpu()
    exp = torch.tensor(ref_losses)
    assert got.shape == exp.shape
    torch.testing.assert_close(got, exp, rtol=3e-2, atol=2e-3)
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        err = (p - q).abs().max().item()
        assert err < 2e-2 * max(1.0, q.abs().max().item()), (n, err)


def test_fused_program_graph_used():
    ds, model, ref, prog, loader = _setup(size=2048, batch=32, graph_steps=8, persistent=False)
    prog.run_steps(100)
    torch.cuda.synchronize()
    assert 0 in prog._graphs or 1 in prog._graphs
    assert int(prog.cursor.item()) == 100
    assert torch.isfinite(prog.last_losses(100)).all()


def test_persistent_program_long_run():
    """Persistent launches of up to chunk_steps steps, crossing epochs and
    index-ring wrap-around, match the per-step program bit-for-bit in loss
    trajectory shape and end in the same place within bf16 tolerance."""
    _, model_a, _, pa, _ = _setup(size=2048, batch=32)
    _, model_b, _, pb, _ = _setup(size=2048, batch=32, persistent=False)
    assert pa.persistent and not pb.persistent
    pa.run_steps(2500)
    pb.run_steps(2500)
    pa.store_to_module()
    pb.store_to_module()
    torch.cuda.synchronize()
    assert int(pa.cursor.item()) == 2500 % pa.R
    la, lb = pa.last_losses(2500).cpu(), pb.last_losses(2500).cpu()
    assert torch.isfinite(la).all()
    # the FULL per-step loss sequence: a batch-order / index-ring / launch-boundary bug
    # shows as a different batch's loss at that step (the two programs only differ in
    # bf16 rounding order, which drifts slowly); early steps tightly, all steps loosely
    torch.testing.assert_close(la[:64], lb[:64], rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(la, lb, rtol=5e-2, atol=5e-3)
    # the per-step loss varies strongly between batches: the two sequences must move together
    da, db = la[1:] - la[:-1], lb[1:] - lb[:-1]
    corr = float((da * db).sum() / (da.norm() * db.norm()))
    assert corr > 0.98, corr
    for (n, p), (_, q) in zip(model_a.named_parameters(), model_b.named_parameters()):
        assert (p - q).abs().max().item() < 3e-2 * max(1.0, q.abs().max().item()), n


def test_trainer_end_to_end_gpu(tmp_path):
    """Reference-compatible Trainer on GPU (fused path), checkpoint + resume."""
    import os

    from distributed_training_amd.data.datasets import MyTrainDataset
    from distributed_training_amd.engine.trainer import Trainer, TrainingConfig
    from distributed_training_amd.models.mlp import MLP
    from distributed_training_amd.app import prepare_dataloader
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.env import DistributedEnvironment

    from dist_utils import setup_env_on_free_port

    os.environ.update({"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1"})
    env = setup_env_on_free_port(DistributedEnvironment("cuda"))
    try:
        torch.manual_seed(0)
        ds = MyTrainDataset(512, 20, 1, seed=0)
        model = MLP(20, 256, 1)
        opt = FusedSGD(model.parameters(), lr=1e-2)
        snap = tmp_path / "snap.pt"
        cfg = TrainingConfig(max_epochs=3, save_every=1, batch_size=32, learning_rate=1e-2, snapshot_path=snap,
                             loss="mse")
        tr = Trainer(model, prepare_dataloader(ds, 32), opt, cfg, env)
        assert tr._fused is not None
        tr.train(3)
        ck = torch.load(snap, weights_only=True)
        assert ck["EPOCHS_RUN"] == 2
        assert set(ck["MODEL_STATE"]) == {"module.fc1.weight", "module.fc1.bias", "module.fc2.weight",
                                          "module.fc2.bias"}
        for k, v in tr.model.state_dict().items():
            torch.testing.assert_close(ck["MODEL_STATE"][k].to(v.device), v)
    finally:
        env.teardown()


def test_trainer_step_graph_matches_eager(tmp_path):
    """train.step_graph=true (generic DDP path): the first batch runs eagerly and is captured,
    later full batches replay the graph, an epoch's short last batch runs eagerly -- the final
    weights equal the all-eager run's bit for bit."""
    import os

    from distributed_training_amd.app import prepare_dataloader
    from distributed_training_amd.data.datasets import MyTrainDataset
    from distributed_training_amd.engine.trainer import Trainer, TrainingConfig
    from distributed_training_amd.models.mlp import MLP
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.env import DistributedEnvironment

    from dist_utils import setup_env_on_free_port

    os.environ.update({"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1"})
    env = setup_env_on_free_port(DistributedEnvironment("cuda"))
    try:
        finals = []
        for graph in (False, True):
            torch.manual_seed(0)
            ds = MyTrainDataset(100, 20, 1, seed=0)  # 3 full batches + one of 4 per epoch
            model = MLP(20, 256, 1)
            opt = FusedSGD(model.parameters(), lr=1e-2, momentum=0.9)
            cfg = TrainingConfig(max_epochs=2, save_every=5, batch_size=32, learning_rate=1e-2,
                                 snapshot_path=tmp_path / f"s{int(graph)}.pt", loss="mse", fused_step=False,
                                 step_graph=graph)
            tr = Trainer(model, prepare_dataloader(ds, 32), opt, cfg, env)
            assert tr._fused is None
            tr.train(2)
            torch.cuda.synchronize()
            if graph:
                assert tr._graphed is not None and tr._graphed.replays == 5, tr._graphed.replays
            finals.append({k: v.detach().clone() for k, v in tr.model.state_dict().items()})
        for k in finals[0]:
            assert torch.equal(finals[0][k], finals[1][k]), k
    finally:
        env.teardown()


class _FakeComm:
    """A communicator stub for the GraphedStep host logic (poll / agreement)."""

    def __init__(self, peer_ok=True):
        self.world_size = 2
        self.device = _dev()
        self.peer_ok = peer_ok
        self.timed_out = False

    def all_reduce(self, t, op="sum", async_op=False):
        if op == "min" and not self.peer_ok:
            t.zero_()  # another rank reported a failed capture

    def poll_errors(self):
        if self.timed_out:
            raise RuntimeError("peer exchange timed out")


class _FakeEngine:
    def __init__(self, comm):
        self.comm = comm
        self.world_size = comm.world_size
        self.resets = 0

    def reset_iteration(self):
        self.resets += 1


def test_graphed_step_polls_comm_errors_after_replay():
    """the replay skips the DDP finalize's host-side error poll, so GraphedStep polls
    the communicator after every replay -- a timed-out peer exchange raises."""
    from distributed_training_amd.engine.step_graph import GraphedStep

    dev = _dev()
    w = torch.zeros(64, device=dev)
    x = torch.ones(64, device=dev)

    def step(xb):
        w.add_(xb)
        return w.sum()

    eng = _FakeEngine(_FakeComm())
    g = GraphedStep(step, [x.clone()], warmup=1, engine=eng)
    assert g.ok
    g(x)
    torch.cuda.synchronize()
    assert float(w[0]) == 2.0  # warm-up + one replay (the capture itself does not run)
    eng.comm.timed_out = True
    with pytest.raises(RuntimeError, match="timed out"):
        g(x)


@pytest.mark.parametrize("local_fail", [True, False])
def test_graphed_step_capture_failure_agreed(local_fail):
    """A capture that fails here (or on another rank: the MIN agreement) resets the engine's step
    state and disables the graph on every rank -- the caller runs the eager step."""
    from distributed_training_amd.engine.step_graph import GraphedStep

    dev = _dev()
    x = torch.ones(8, device=dev)

    def step(xb):
        if local_fail and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("op not capturable")
        return xb.sum()

    eng = _FakeEngine(_FakeComm(peer_ok=False))  # (local_fail=False: only the peer failed)
    g = GraphedStep(step, [x.clone()], warmup=1, engine=eng)
    assert not g.ok and g.error is not None
    assert eng.resets == (1 if local_fail else 0)
    with pytest.raises(RuntimeError, match="eager"):
        g(x)


@pytest.mark.parametrize("arch,strategy", [("gpt2", "ddp"), ("llama", "fsdp"), ("gpt2", "fsdp")])
def test_chunked_head_ce_under_engines(arch, strategy, monkeypatch):
    """The row-blocked LM head + CE (weight gradient formed in the forward, written straight into the
    engine's final gradient slice: DDP's flat buffer -- GPT-2's tied embedding rows added into it in
    place afterwards -- or the one-rank FSDP unit's flat-gradient slice) gives the same gradients and
    loss as the one-block head under the same engine, over two steps."""
    import copy

    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.models.llama import Llama, LlamaConfig
    from distributed_training_amd.ops import lm
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel, lm_wrap_policy

    dev = _dev()
    torch.manual_seed(3)
    if arch == "gpt2":
        base = GPT2(GPT2Config(n_layer=2, n_head=4, n_embd=256, vocab_size=1024, block_size=128))
    else:
        base = Llama(LlamaConfig(n_layer=2, n_head=4, n_kv_head=2, n_embd=256, ffn_hidden=512, vocab_size=1024,
                                 block_size=128))
    idx = torch.randint(0, 1024, (2, 2, 129), device=dev)
    results = []
    for chunk in (0, 64):
        monkeypatch.setattr(lm, "HEAD_CE_CHUNK", chunk)
        m = copy.deepcopy(base).to(dev)
        if strategy == "ddp":
            w = DistributedDataParallel(m, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
        else:
            w = FullyShardedDataParallel(m, device=dev, wrap_policy=lm_wrap_policy(m), param_dtype=torch.bfloat16)
        losses, grads = [], []
        for s in range(2):
            w.zero_grad(set_to_none=True)
            loss = w(idx[s, :, :-1], idx[s, :, 1:])
            loss.backward()
            torch.cuda.synchronize()
            losses.append(loss.item())
            grads.append([p.grad.float().clone() for p in w.parameters()])
        results.append((losses, grads))
    (l0, g0), (l1, g1) = results
    for a, b in zip(l0, l1):
        assert abs(a - b) < 1e-2 * abs(a)
    for s in range(2):
        for a, b in zip(g0[s], g1[s]):
            assert ((a - b).norm() / (a.norm() + 1e-12)).item() < 2e-2


@pytest.mark.parametrize("strategy", ["ddp", "fsdp"])
def test_deferred_norm_grads_bitwise(strategy, monkeypatch):
    """The norms' gamma / beta gradients finished by the batched column-sum launch at the flush
    (ops/lm.py _NORM_DEFER) are bit-identical to the per-norm launch (DTA_NORM_DEFER=0), under the engine
    whose flat-gradient slices make the deferral possible."""
    import copy

    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops import lm
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel, lm_wrap_policy

    dev = _dev()
    torch.manual_seed(4)
    base = GPT2(GPT2Config(n_layer=2, n_head=4, n_embd=256, vocab_size=1024, block_size=128))
    idx = torch.randint(0, 1024, (2, 129), device=dev)
    grads = []
    for defer in ("1", "0"):
        monkeypatch.setenv("DTA_NORM_DEFER", defer)
        n0 = lm.GEMM_STATS["deferred_norm"]
        m = copy.deepcopy(base).to(dev)
        if strategy == "ddp":
            w = DistributedDataParallel(m, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
        else:
            w = FullyShardedDataParallel(m, device=dev, wrap_policy=lm_wrap_policy(m), param_dtype=torch.bfloat16)
        w.zero_grad(set_to_none=True)
        w(idx[:, :-1], idx[:, 1:]).backward()
        torch.cuda.synchronize()
        assert not lm._NORM_DEFER  # flushed by the end of the backward
        assert (lm.GEMM_STATS["deferred_norm"] > n0) == (defer == "1")  # the deferred path did run
        grads.append([p.grad.clone() for p in w.parameters()])
    for a, b in zip(*grads):
        assert torch.equal(a, b)
