"""Fused step program of the reference's default model (csrc/linear_step.hip,
engine/fused_linear.py): one nn.Linear, soft-label cross-entropy or MSE, fp32,
SGD, DistributedSampler batch order.

References are plain fp32 PyTorch: the same model trained by the reference
loop (zero_grad -> forward -> loss -> backward -> SGD step) on the same
batches; with several ranks, the mean of the per-rank gradients (DDP)."""
import os
import types

import pytest
import torch
import torch.nn.functional as F

from dist_utils import run_gloo

pytestmark = pytest.mark.gpu


def _reference(model, X, T, batches, loss, sgd_kw):
    """batches: per step, a list of per-rank index tensors (DDP mean of their gradients)."""
    ref = torch.nn.Linear(model.in_features, model.out_features)
    ref.load_state_dict({k: v.detach().cpu().float() for k, v in model.state_dict().items()})
    opt = torch.optim.SGD(ref.parameters(), **sgd_kw)
    losses = []
    for per_rank in batches:
        grads = []
        for idx in per_rank:
            ref.zero_grad()
            out = ref(X[idx])
            lv = F.cross_entropy(out, T[idx]) if loss == "cross_entropy" else F.mse_loss(out, T[idx])
            lv.backward()
            grads.append([p.grad.clone() for p in ref.parameters()])
            losses.append(float(lv.detach()))
        for p, *gs in zip(ref.parameters(), *grads):
            p.grad = sum(gs) / len(gs)
        opt.step()
    ref.opt = opt
    return ref, losses


def _setup(out_dim, n, seed=0):
    from distributed_training_amd.data.datasets import MyTrainDataset

    ds = MyTrainDataset(n, 20, out_dim, seed=seed)
    return ds


@pytest.mark.parametrize("loss,out_dim,sgd_kw", [
    ("cross_entropy", 4, dict(lr=0.5)),
    ("cross_entropy", 5, dict(lr=0.2, momentum=0.9, weight_decay=1e-2)),
    ("mse", 3, dict(lr=0.1, momentum=0.8, nesterov=True)),
    ("mse", 1, dict(lr=0.05, momentum=0.5, dampening=0.1, maximize=False)),
])
def test_linear_program_matches_reference_loop(loss, out_dim, sgd_kw):
    from distributed_training_amd.data.datasets import DeviceDataLoader
    from distributed_training_amd.engine.fused_linear import FusedLinearProgram, linear_eligible
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.sampler import DistributedSampler

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ds = _setup(out_dim, 200)  # 200 / 32: last batch of each epoch is short (8)
    model = torch.nn.Linear(20, out_dim).to(dev)
    opt = FusedSGD(model.parameters(), **sgd_kw)
    sampler = DistributedSampler(ds, num_replicas=1, rank=0)
    loader = DeviceDataLoader(ds, 32, sampler=sampler, device=dev)
    assert linear_eligible(model, opt, loader, loss, dev) is None
    comm = types.SimpleNamespace(world_size=1, rank=0)
    init = torch.nn.Linear(20, out_dim)
    init.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
    prog = FusedLinearProgram(model, opt, loader, comm, loss=loss)
    batches = []
    for ep in range(3):
        prog.run_epoch(ep)
        sampler.set_epoch(ep)
        idx = sampler.epoch_indices()
        batches += [[idx[i:i + 32]] for i in range(0, len(idx), 32)]
    prog.store_to_module()
    torch.cuda.synchronize()
    ref, losses = _reference(init, ds.X, ds.Y, batches, loss, sgd_kw)
    got = prog.last_losses(len(losses)).cpu()
    torch.testing.assert_close(got, torch.tensor(losses), rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(model.weight.detach().cpu(), ref.weight.detach(), rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(model.bias.detach().cpu(), ref.bias.detach(), rtol=2e-5, atol=2e-6)
    if sgd_kw.get("momentum"):
        # the program's momentum reaches the optimizer state (checkpoint OPTIM_STATE) ...
        for p, q in zip(model.parameters(), ref.parameters()):
            torch.testing.assert_close(opt.state[p]["momentum_buffer"].cpu(), ref.opt.state[q]["momentum_buffer"],
                                       rtol=2e-5, atol=2e-6)
        # ... and a new program (a resumed run) continues it: one more epoch matches the reference's
        prog2 = FusedLinearProgram(model, opt, loader, comm, loss=loss)
        prog2.run_epoch(3)
        prog2.store_to_module()
        torch.cuda.synchronize()
        sampler.set_epoch(3)
        idx = sampler.epoch_indices()
        for i in range(0, len(idx), 32):
            ref.zero_grad()
            out = ref(ds.X[idx[i:i + 32]])
            t = ds.Y[idx[i:i + 32]]
            (F.cross_entropy(out, t) if loss == "cross_entropy" else F.mse_loss(out, t)).backward()
            ref.opt.step()
        torch.testing.assert_close(model.weight.detach().cpu(), ref.weight.detach(), rtol=5e-5, atol=5e-6)


def test_reference_default_is_a_noop_step():
    """Linear(20, 1) + CE on one logit (the reference default): loss 0, weights unchanged."""
    from distributed_training_amd.data.datasets import DeviceDataLoader
    from distributed_training_amd.engine.fused_linear import FusedLinearProgram
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.sampler import DistributedSampler

    dev = torch.device("cuda", 0)
    ds = _setup(1, 2048)
    model = torch.nn.Linear(20, 1).to(dev)
    w0 = model.weight.detach().clone()
    opt = FusedSGD(model.parameters(), lr=1e-3)
    loader = DeviceDataLoader(ds, 32, sampler=DistributedSampler(ds, num_replicas=1, rank=0), device=dev)
    prog = FusedLinearProgram(model, opt, loader, types.SimpleNamespace(world_size=1, rank=0), "cross_entropy")
    assert prog.run_epoch(0) == 64
    prog.store_to_module()
    torch.cuda.synchronize()
    assert torch.equal(model.weight.detach(), w0)
    assert torch.all(prog.last_losses(64) == 0)


def test_trainer_default_config_uses_fused_linear(tmp_path):
    """The reference's own entrypoint config (ws 1) picks the fused Linear program and keeps the
    checkpoint contract ({"MODEL_STATE": module.* keys, "EPOCHS_RUN"})."""
    from distributed_training_amd.app import load_train_objs, prepare_dataloader, training_config_from
    from distributed_training_amd.config import compose
    from distributed_training_amd.engine.fused_linear import FusedLinearProgram
    from distributed_training_amd.engine.trainer import Trainer
    from distributed_training_amd.parallel.env import DistributedEnvironment

    os.environ.update({"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1"})
    from dist_utils import setup_env_on_free_port

    snap = tmp_path / "snap.pt"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = compose(os.path.join(root, "conf"), "config",
                  ["train.total_epochs=3", f"train.snapshot_path={snap}", "train.loss=mse", "train.seed=0"],
                  runtime={"output_dir": str(tmp_path)})
    env = setup_env_on_free_port(DistributedEnvironment("cuda"))
    try:
        ds, model, opt = load_train_objs(cfg)
        tc = training_config_from(cfg, model)
        tr = Trainer(model, prepare_dataloader(ds, tc.batch_size), opt, tc, env)
        assert isinstance(tr._fused, FusedLinearProgram)
        w0 = tr.model.module.weight.detach().clone()
        tr.train(tc.max_epochs)
        assert not torch.equal(w0, tr.model.module.weight.detach())  # mse: gradients are non-zero
        ck = torch.load(snap, weights_only=True)
        assert set(ck["MODEL_STATE"]) == {"module.weight", "module.bias"} and ck["EPOCHS_RUN"] == 2
        torch.testing.assert_close(ck["MODEL_STATE"]["module.weight"].cpu(), tr.model.module.weight.detach().cpu())
    finally:
        env.teardown()


def _ddp_worker(rank, ws, loss, sgd_kw):
    import torch.distributed as dist

    from distributed_training_amd.data.datasets import DeviceDataLoader
    from distributed_training_amd.engine.fused_linear import FusedLinearProgram
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.comm import make_comm
    from distributed_training_amd.parallel.sampler import DistributedSampler

    os.environ["DTA_SHARED_GPU"] = "1"
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ds = _setup(3, 256 * ws + 40)
    torch.manual_seed(0)
    model = torch.nn.Linear(20, 3).to(dev)
    init = torch.nn.Linear(20, 3)
    init.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
    opt = FusedSGD(model.parameters(), **sgd_kw)
    samplers = [DistributedSampler(ds, num_replicas=ws, rank=r) for r in range(ws)]
    loader = DeviceDataLoader(ds, 32, sampler=samplers[rank], device=dev)
    comm = make_comm(dev)
    prog = FusedLinearProgram(model, opt, loader, comm, loss=loss)
    batches = []
    for ep in range(3):  # epoch 0 eager, epochs 1-2 replay the captured graph
        prog.run_epoch(ep)
        per = []
        for s in samplers:
            s.set_epoch(ep)
            per.append(s.epoch_indices())
        S = len(loader)
        batches += [[p[i * 32:(i + 1) * 32] for p in per] for i in range(S)]
    prog.store_to_module()
    torch.cuda.synchronize()
    final = torch.cat([model.weight.detach().reshape(-1), model.bias.detach()]).cpu()
    parts = [torch.empty_like(final) for _ in range(ws)]
    dist.all_gather(parts, final)
    for p in parts[1:]:
        assert torch.equal(p, parts[0]), "replicas diverged"
    ref, _ = _reference(init, ds.X, ds.Y, batches, loss, sgd_kw)
    want = torch.cat([ref.weight.detach().reshape(-1), ref.bias.detach()])
    torch.testing.assert_close(final, want, rtol=3e-5, atol=3e-6)


@pytest.mark.parametrize("ws", [2, 4])
def test_linear_program_ddp_shared_gpu(ws):
    run_gloo(_ddp_worker, ws, "cross_entropy", dict(lr=0.3, momentum=0.9))
