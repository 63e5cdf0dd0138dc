"""The fused-kernel host helpers (layout, limits, fp32 reference) on CPU."""
import torch

from distributed_training_amd.models.mlp import MLP, build_mlp
from distributed_training_amd.ops import mlp_fused as mf


def test_layout_alignment_and_views():
    lay = mf.make_layout(20, 512, 1)
    # 16-byte aligned regions (float4 access); b1 and W2 four LDS banks apart
    assert lay.o_w1 == 0 and all(o % 4 == 0 for o in lay.offsets) and lay.total % 16 == 0
    assert (lay.o_w2 - lay.o_b1) % 32 == 4
    flat = torch.arange(lay.total, dtype=torch.float32)
    v = lay.views(flat)
    assert v["fc1.weight"].shape == (512, 20) and v["fc2.weight"].shape == (1, 512)
    assert v["fc1.bias"][0].item() == lay.o_b1


def test_supported_limits():
    assert mf.supported(20, 512, 1, 32)
    assert mf.supported(20, 1024, 1, 32)
    assert not mf.supported(32, 512, 1, 32)      # needs a spare ones-column (in <= 31)
    assert not mf.supported(20, 500, 1, 32)      # hidden % 32
    assert not mf.supported(20, 512, 9, 32)      # out <= 8
    assert not mf.supported(20, 512, 1, 129)     # batch <= 128
    assert not mf.supported(20, 8192, 1, 32)     # LDS image
    assert mf.lds_bytes(20, 512, 1, 32, momentum=True) > mf.lds_bytes(20, 512, 1, 32)


def test_reference_step_matches_module_autograd():
    torch.manual_seed(0)
    m = MLP(20, 64, 3, activation="gelu")
    lay = mf.make_layout(20, 64, 3)
    X, T = torch.rand(50, 20), torch.rand(50, 3)
    idx = torch.randperm(50)[:16]
    params = {k: v.detach() for k, v in m.named_parameters()}
    for loss in ("mse", "cross_entropy"):
        lv, g = mf.reference_step(X, T, idx, params, "gelu", loss)
        m.zero_grad()
        out = m(X[idx])
        l2 = mf.loss_fn(out, T[idx], loss)
        l2.backward()
        torch.testing.assert_close(lv, l2.detach())
        for k, p in m.named_parameters():
            torch.testing.assert_close(g[k], p.grad)


def test_reference_cross_entropy_quirk():
    """Reference: F.cross_entropy on a 1-wide output is identically 0."""
    torch.manual_seed(0)
    lin = build_mlp({"input_size": 20, "output_size": 1})
    assert isinstance(lin, torch.nn.Linear)
    out = lin(torch.rand(32, 20))
    loss = torch.nn.functional.cross_entropy(out, torch.rand(32, 1))
    loss.backward()
    assert loss.item() == 0.0 and lin.weight.grad.abs().sum().item() == 0.0
