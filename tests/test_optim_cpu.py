"""Fused optimizers (CPU math path + FlatParamGroup bookkeeping) vs torch.optim."""
import pytest
import torch

from distributed_training_amd.ops.optim import FusedAdamW, FusedSGD, same_kind_optimizer


@pytest.mark.parametrize("kw", [dict(), dict(momentum=0.9), dict(momentum=0.9, nesterov=True, weight_decay=1e-2),
                                dict(momentum=0.5, dampening=0.1), dict(maximize=True, weight_decay=0.1)])
def test_sgd_matches_torch(kw):
    torch.manual_seed(0)
    p0 = [torch.randn(5, 3), torch.randn(7)]
    a = [torch.nn.Parameter(t.clone()) for t in p0]
    b = [torch.nn.Parameter(t.clone()) for t in p0]
    o1 = torch.optim.SGD(a, lr=0.1, **kw)
    o2 = FusedSGD(b, lr=0.1, **kw)
    for _ in range(4):
        gs = [torch.randn_like(t) for t in p0]
        for p, g in zip(a, gs):
            p.grad = g.clone()
        for p, g in zip(b, gs):
            p.grad = g.clone()
        o1.step()
        o2.step()
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y)


@pytest.mark.parametrize("adamw,ams", [(True, False), (True, True), (False, False)])
def test_adam_matches_torch(adamw, ams):
    torch.manual_seed(1)
    p0 = [torch.randn(4, 4), torch.randn(3)]
    a = [torch.nn.Parameter(t.clone()) for t in p0]
    b = [torch.nn.Parameter(t.clone()) for t in p0]
    cls = torch.optim.AdamW if adamw else torch.optim.Adam
    o1 = cls(a, lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1, amsgrad=ams)
    o2 = FusedAdamW(b, lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1, amsgrad=ams, adamw=adamw)
    for _ in range(5):
        gs = [torch.randn_like(t) for t in p0]
        for p, g in zip(a, gs):
            p.grad = g.clone()
        for p, g in zip(b, gs):
            p.grad = g.clone()
        o1.step()
        o2.step()
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_same_kind_optimizer_and_zero_grad_flat():
    from distributed_training_amd.parallel.flat import FlatParamGroup

    m = torch.nn.Linear(4, 2)
    opt = torch.optim.SGD(m.parameters(), lr=0.3, momentum=0.5)
    new = same_kind_optimizer(opt, list(m.parameters()))
    assert isinstance(new, FusedSGD) and new.param_groups[0]["lr"] == 0.3
    fg = FlatParamGroup(list(m.parameters()), torch.device("cpu"))
    assert fg.total % 16 == 0
    for i, p in enumerate(fg.params):
        assert p.data_ptr() == fg.param_view(i).data_ptr() and p.grad.data_ptr() == fg.grad_view(i).data_ptr()
    m(torch.randn(3, 4)).sum().backward()
    assert fg.grad.abs().sum() > 0  # autograd accumulated straight into the flat buffer
    new.zero_grad()
    assert fg.grad.abs().sum() == 0 and all(fg.grad_is_view(i) for i in range(len(fg.params)))
    b = fg.make_buckets(range(len(fg.params)), cap_bytes=16, first_cap_bytes=8)
    assert b[0].start == 0 and b[-1].end <= fg.total and sum(len(x.param_ids) for x in b) == 2
