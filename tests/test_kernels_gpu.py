"""Numerics of the hand-written gfx950 kernels vs plain PyTorch fp32 references.

Run on an MI355X: ``pytest -m gpu tests/test_kernels_gpu.py``.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    from distributed_training_amd.ops import native

    return native()


def dev():
    return torch.device("cuda", 0)


@pytest.mark.parametrize("momentum,nesterov,wd,damp", [(0.0, False, 0.0, 0.0), (0.9, False, 1e-2, 0.0),
                                                        (0.9, True, 0.0, 0.0), (0.5, False, 0.0, 0.1)])
@pytest.mark.parametrize("n", [1, 7, 4096, 100003])
def test_flat_sgd_matches_torch(C, n, momentum, nesterov, wd, damp):
    torch.manual_seed(0)
    p0 = torch.randn(n, device=dev())
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.SGD([ref], lr=0.1, momentum=momentum, nesterov=nesterov, weight_decay=wd, dampening=damp)
    p = p0.clone()
    mom = torch.zeros(n, device=dev()) if momentum else None
    pb = torch.empty(n, device=dev(), dtype=torch.bfloat16)
    for it in range(3):
        g = torch.randn(n, device=dev())
        ref.grad = g.clone()
        opt.step()
        C.flat_sgd(p, p, g, mom, pb, 0.1, momentum, damp, wd, 1.0, nesterov, False, it == 0, -1)
    torch.cuda.synchronize()
    torch.testing.assert_close(p, ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(pb.float(), p.bfloat16().float())


@pytest.mark.parametrize("amsgrad", [False, True])
@pytest.mark.parametrize("n", [5, 65536 + 3])
def test_flat_adamw_matches_torch(C, n, amsgrad):
    torch.manual_seed(1)
    p0 = torch.randn(n, device=dev())
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([ref], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, amsgrad=amsgrad)
    p = p0.clone()
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    vmax = torch.zeros_like(p) if amsgrad else None
    step = torch.zeros(1, device=dev())
    for _ in range(4):
        g = torch.randn(n, device=dev())
        ref.grad = g.clone()
        opt.step()
        C.flat_adam(p, g, m, v, vmax, None, step, 1e-2, 0.9, 0.95, 1e-8, 0.1, 1.0, True, False, amsgrad, True, -1)
    torch.cuda.synchronize()
    assert step.item() == 4.0
    torch.testing.assert_close(p, ref.detach(), rtol=1e-5, atol=1e-6)


def test_mt_scale_copy(C):
    torch.manual_seed(2)
    srcs = [torch.randn(s, device=dev()) for s in (1, 17, 16384, 16385, 300000)] * 10
    dsts = [torch.empty_like(s) for s in srcs]
    C.mt_scale_copy(srcs, dsts, 0.25, -1)
    for s, d in zip(srcs, dsts):
        torch.testing.assert_close(d, s * 0.25)
    dbf = [torch.empty(s.numel(), device=dev(), dtype=torch.bfloat16) for s in srcs]
    C.mt_scale_copy(srcs, dbf, 1.0, -1)
    for s, d in zip(srcs, dbf):
        torch.testing.assert_close(d.float(), s.bfloat16().float())


def test_sumsq_and_clip(C):
    x = torch.randn(1_000_003, device=dev())
    out = torch.zeros(1, device=dev())
    C.flat_sumsq(x, out, -1)
    torch.testing.assert_close(out[0], (x * x).sum(), rtol=1e-4, atol=1e-3)
    ref = x.clone()
    torch.nn.utils.clip_grad_norm_([torch.nn.Parameter(torch.zeros_like(ref))], 1.0)  # API smoke
    norm = ref.norm()
    C.flat_clip(x, out, 1.0, -1)
    torch.testing.assert_close(x, ref * (1.0 / (norm + 1e-6)), rtol=1e-4, atol=1e-6)


def _mlp_case(in_dim, hidden, out_dim, batch, n=256, seed=0):
    from distributed_training_amd.ops import mlp_fused as mf

    g = torch.Generator().manual_seed(seed)
    lay = mf.make_layout(in_dim, hidden, out_dim)
    X = torch.rand(n, in_dim, generator=g).to(dev())
    T = torch.rand(n, out_dim, generator=g).to(dev())
    flat = torch.zeros(lay.total)
    v = lay.views(flat)
    v["fc1.weight"].copy_(torch.randn(hidden, in_dim, generator=g) * (1 / in_dim ** 0.5))
    v["fc1.bias"].copy_(torch.randn(hidden, generator=g) * 0.1)
    v["fc2.weight"].copy_(torch.randn(out_dim, hidden, generator=g) * (1 / hidden ** 0.5))
    v["fc2.bias"].copy_(torch.randn(out_dim, generator=g) * 0.1)
    idx = torch.randperm(n, generator=g)[: 4 * 128].int()
    return lay, X, T, flat.to(dev()), idx


@pytest.mark.parametrize("in_dim,hidden,out_dim,batch,act,loss,own", [
    (20, 512, 1, 32, "relu", "mse", 4),
    (20, 512, 1, 32, "relu", "cross_entropy", 4),
    (20, 256, 4, 32, "gelu", "cross_entropy", 2),
    (31, 128, 8, 64, "silu", "mse", 1),
    (7, 1024, 2, 100, "relu", "mse", 8),
    (20, 64, 1, 5, "relu", "mse", 1),
])
def test_mlp2_fused_step_no_update(C, in_dim, hidden, out_dim, batch, act, loss, own):
    from distributed_training_amd.ops import mlp_fused as mf

    lay, X, T, flat, idx = _mlp_case(in_dim, hidden, out_dim, batch)
    stride = 128
    ring = torch.zeros(4, stride, dtype=torch.int32)
    ring.view(-1)[: idx.numel()] = idx
    ring = ring.to(dev())
    cursor = torch.tensor([1], dtype=torch.int32, device=dev())
    stage = mf.make_stage(dev())
    loss_ring = torch.zeros(8, device=dev())
    scale = 0.5
    params_cpu = {k: v.cpu() for k, v in lay.views(flat).items()}
    # step A gathers its own batch (ring row 1) and stages row 2; step B reads the staged batch
    for step, (parity, gather_self, row) in enumerate(((0, True, 1), (1, False, 2))):
        p_out = torch.full_like(flat, float("nan"))
        g_prev = torch.zeros_like(flat)
        g_out = torch.zeros_like(flat)
        mf.fused_step(X, T, ring, cursor, stage, loss_ring, flat, p_out, g_prev, g_out, None, None, lay, batch,
                      own, act, loss, False, scale, {"lr": 0.1}, 1.0, False, parity=parity,
                      gather_self=gather_self)
        torch.cuda.synchronize()
        if gather_self:
            assert cursor.item() == 1  # the host advances it after a self-gathering step
            cursor.add_(1)
        else:
            assert cursor.item() == 3
        nxt = ring[row + 1 if row + 1 < 4 else 0, :batch].long()
        torch.testing.assert_close(stage[0][1 - parity, :batch, :in_dim].float(), X[nxt].bfloat16().float())
        for k, v in lay.views(p_out).items():  # owners copied every parameter through unchanged
            torch.testing.assert_close(v, lay.views(flat)[k], msg=k)
        step_idx = ring[row, :batch].cpu()
        ref_loss, ref_g = mf.reference_step(X.cpu(), T.cpu(), step_idx, params_cpu, act, loss, emulate_bf16=True)
        torch.testing.assert_close(loss_ring[step].cpu(), ref_loss, rtol=1e-3, atol=1e-5)
        assert int(stage[2].item()) == step + 1
        got = lay.views(g_out)
        for k in ref_g:
            exp = ref_g[k] * scale
            tol = 3e-2 * exp.abs().max().item() + 1e-6
            err = (got[k].cpu() - exp).abs().max().item()
            assert err <= tol, f"{k}: max err {err} > {tol}"


def test_mlp2_fused_step_sgd_update_pingpong(C):
    """apply_update=1 must equal torch SGD(momentum) applied to g_prev, and the
    updated weights must be what the forward used."""
    from distributed_training_amd.ops import mlp_fused as mf

    in_dim, hidden, out_dim, batch = 20, 512, 1, 32
    lay, X, T, flat, idx = _mlp_case(in_dim, hidden, out_dim, batch, seed=3)
    ring = idx[:128].view(1, 128).contiguous().to(dev())
    cursor = torch.zeros(1, dtype=torch.int32, device=dev())
    stage = mf.make_stage(dev())
    loss_ring = torch.zeros(4, device=dev())
    g_prev = torch.randn_like(flat) * 0.01
    mom_in = torch.randn_like(flat) * 0.01
    mom_out = torch.zeros_like(flat)
    p_out = torch.zeros_like(flat)
    g_out = torch.zeros_like(flat)
    sgd = {"lr": 0.05, "momentum": 0.9, "weight_decay": 1e-3, "nesterov": True}
    mf.fused_step(X, T, ring, cursor, stage, loss_ring, flat, p_out, g_prev, g_out, mom_in, mom_out, lay, batch, 4,
                  "relu", "mse", True, 1.0, sgd, 1.0, False, parity=0, gather_self=True)
    torch.cuda.synchronize()
    buf = mom_in.clone()
    exp_p = mf.apply_sgd_reference(flat, g_prev, buf, sgd, first_step=False)
    for k, v in lay.views(p_out).items():
        torch.testing.assert_close(v, lay.views(exp_p)[k], rtol=1e-5, atol=1e-6, msg=k)
        torch.testing.assert_close(lay.views(mom_out)[k], lay.views(buf)[k], rtol=1e-5, atol=1e-6)
    ref_loss, ref_g = mf.reference_step(X.cpu(), T.cpu(), ring[0, :batch].cpu(),
                                        {k: v.cpu() for k, v in lay.views(exp_p).items()}, "relu", "mse",
                                        emulate_bf16=True)
    torch.testing.assert_close(loss_ring[0].cpu(), ref_loss, rtol=1e-3, atol=1e-5)
    for k in ref_g:
        exp = ref_g[k]
        err = (lay.views(g_out)[k].cpu() - exp).abs().max().item()
        assert err <= 3e-2 * exp.abs().max().item() + 1e-6, k


def test_rccl_world1_collectives(C):
    from distributed_training_amd.ops import ensure_rccl

    ensure_rccl()
    uid = C.rccl_unique_id()
    comm = C.RcclComm(uid, 1, 0, 0)
    x = torch.arange(1000, dtype=torch.float32, device=dev())
    y = x.clone()
    comm.all_reduce(y, "sum", -1)
    comm.all_reduce(y, "avg", -1)
    out = torch.empty(1000, device=dev())
    comm.all_gather(out, x, -1)
    rs = torch.empty(1000, device=dev())
    comm.reduce_scatter(rs, x, "sum", -1)
    bf = x.bfloat16()
    comm.broadcast(bf, 0, -1)
    a2a = torch.empty_like(x)
    comm.all_to_all(a2a, x, -1)
    torch.cuda.synchronize()
    torch.testing.assert_close(y, x)
    torch.testing.assert_close(out, x)
    torch.testing.assert_close(rs, x)
    torch.testing.assert_close(a2a, x)
    comm.destroy()
    with pytest.raises(RuntimeError, match="aborted"):  # a destroyed handle is never touched again
        comm.all_reduce(y, "sum", -1)


_ABORT_RACE = r"""
import sys, threading, time
import torch
from distributed_training_amd.parallel.comm import RcclComm

dev = torch.device("cuda", 0)
comm = RcclComm(0, 1, dev, timeout_s=0.3)   # watchdog armed at one rank (explicit timeout)
t = torch.ones(1 << 16, device=dev)
seen, calls = [], [0]

def spam():
    try:
        while True:   # the training thread: collectives enqueued back to back
            comm.all_reduce(t, "sum", async_op=True)
            calls[0] += 1
    except RuntimeError as e:
        seen.append(str(e))

class Never:      # an injected collective that never completes
    def query(self):
        return False

th = threading.Thread(target=spam)
th.start()
time.sleep(0.05)
comm.watchdog.track(Never(), "injected never-completing collective")
th.join(timeout=20)
assert not th.is_alive(), "enqueue thread never observed the abort"
assert seen and ("aborted" in seen[0] or "not complete" in seen[0]), seen
assert comm.aborted and comm._comm.aborted
torch.cuda.synchronize()
comm.destroy()
print("OK", calls[0], seen[0][:80])
"""


def test_rccl_watchdog_abort_races_enqueue(tmp_path):
    """the watchdog thread aborts the communicator while another thread enqueues
    all_reduce in a tight loop -- the loop raises RuntimeError within the deadline and the process
    exits 0 (no use of a freed handle, no segfault).  Run in a child process so a crash is a failed
    exit status, not a dead test runner."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _ABORT_RACE], cwd=root, capture_output=True, text=True, timeout=100,
                       env=dict(os.environ, DTA_COMM_TIMEOUT_EXIT="1"))
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "OK" in r.stdout
