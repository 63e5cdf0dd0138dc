"""gfx950 transformer kernels (flash attention, norms, activations, RoPE,
fused cross-entropy) vs fp32 PyTorch references, forward and backward."""
import math

import pytest
import torch
import torch.nn.functional as F

from distributed_training_amd.ops import lm

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("B,S,H,Hkv,D,causal", [(2, 256, 4, 4, 64, True), (1, 200, 4, 2, 128, True),
                                                 (2, 128, 2, 2, 64, False), (1, 333, 8, 1, 64, True),
                                                 (1, 1024, 2, 2, 128, True), (1, 320, 4, 2, 128, False),
                                                 (1, 600, 4, 2, 64, False)])
@pytest.mark.parametrize("fwd_waves", ["4", "8"])
@pytest.mark.parametrize("bwd_ilv", ["1", "0"])
def test_flash_attention_fwd_bwd(B, S, H, Hkv, D, causal, fwd_waves, bwd_ilv, monkeypatch):
    monkeypatch.setenv("DTA_ATTN_FWD_WAVES", fwd_waves)  # both forward workgroup shapes
    monkeypatch.setenv("DTA_ATTN_BWD_ILV", bwd_ilv)  # backward softmax interleaved with the MFMAs (D 128 default) or not
    torch.manual_seed(0)
    q = torch.randn(B, S, H, D, device=DEV).bfloat16().requires_grad_()
    k = torch.randn(B, S, Hkv, D, device=DEV).bfloat16().requires_grad_()
    v = torch.randn(B, S, Hkv, D, device=DEV).bfloat16().requires_grad_()
    do = torch.randn(B, S, H, D, device=DEV).bfloat16()
    o = lm.attention(q, k, v, causal=causal)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = lm.attention_reference(qr, kr, vr, causal=causal)
    orf.backward(do.float())
    assert _rel(o, orf) < 1e-2
    assert _rel(q.grad, qr.grad) < 2e-2
    assert _rel(k.grad, kr.grad) < 2e-2
    assert _rel(v.grad, vr.grad) < 2e-2


def test_attention_strided_qkv_views():
    """q/k/v as strided views of one fused QKV projection (no copies)."""
    torch.manual_seed(1)
    B, S, H, D = 2, 64, 3, 64
    qkv = torch.randn(B, S, 3, H, D, device=DEV).bfloat16()
    o = lm.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal=True)
    ref = lm.attention_reference(qkv[:, :, 0].float(), qkv[:, :, 1].float(), qkv[:, :, 2].float(), causal=True)
    assert _rel(o, ref) < 1e-2


@pytest.mark.parametrize("C,N", [(768, 37), (4096, 37), (200 * 8, 37), (2048, 1537), (4096, 1537), (6144, 300),
                                 (8192, 769)])
@pytest.mark.parametrize("rms", [False, True])
def test_norms(C, N, rms):
    """LayerNorm / RMSNorm forward + backward vs fp32 autograd; C a multiple of 2048 takes the
    workgroup-per-row backward (several rows per workgroup once N > 768)."""
    torch.manual_seed(2)
    x = (torch.randn(N, C, device=DEV) * 3 + 1).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(C, device=DEV)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(C, device=DEV)).bfloat16().requires_grad_()
    dy = torch.randn(N, C, device=DEV).bfloat16()
    y = lm.rms_norm(x, w) if rms else lm.layer_norm(x, w, b)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    if rms:
        yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    else:
        yr = F.layer_norm(xr, (C,), wr, br, 1e-5)
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    if not rms:
        assert _rel(b.grad, br.grad) < 2e-2


def test_gelu_swiglu_rope():
    torch.manual_seed(3)
    x = torch.randn(64, 256, device=DEV).bfloat16().requires_grad_()
    y = lm.gelu(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    F.gelu(xr, approximate="tanh").backward(dy.float())
    assert _rel(y, F.gelu(x.detach().float(), approximate="tanh")) < 1e-2 and _rel(x.grad, xr.grad) < 1e-2

    ab = torch.randn(32, 2 * 192, device=DEV).bfloat16().requires_grad_()
    y = lm.swiglu(ab)
    dy = torch.randn_like(y)
    y.backward(dy)
    abr = ab.detach().float().requires_grad_()
    a, b = abr.chunk(2, -1)
    (F.silu(a) * b).backward(dy.float())
    assert _rel(ab.grad, abr.grad) < 1e-2

    B, S, Hh, D = 2, 50, 3, 128
    cos, sin = lm.rope_tables(64, D, 500000.0, DEV)
    xq = torch.randn(B, S, Hh, D, device=DEV).bfloat16().requires_grad_()
    yq = lm.apply_rope(xq, cos, sin)
    dy = torch.randn_like(yq)
    yq.backward(dy)
    xr = xq.detach().float().requires_grad_()
    lm.rope_reference(xr, cos, sin).backward(dy.float())
    assert _rel(yq, lm.rope_reference(xq.detach().float(), cos, sin)) < 1e-2
    assert _rel(xq.grad, xr.grad) < 1e-2


@pytest.mark.parametrize("V", [50304, 1001, 128256])
def test_fused_cross_entropy(V):
    torch.manual_seed(4)
    N = 96
    logits = (torch.randn(N, V, device=DEV) * 2).bfloat16().requires_grad_()
    t = torch.randint(0, V, (N,), device=DEV)
    t[5] = -100
    loss = lm.cross_entropy(logits, t)
    loss.backward()
    lr = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(lr, t, ignore_index=-100)
    ref.backward()
    torch.testing.assert_close(loss.float(), ref, rtol=2e-3, atol=2e-3)
    assert _rel(logits.grad, lr.grad) < 2e-2
    assert logits.grad[5].abs().sum().item() == 0.0


def test_gpt2_tiny_trains_on_gpu():
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    dev = torch.device(DEV, 0)
    m = GPT2(GPT2Config(n_layer=2, n_head=2, n_embd=128, vocab_size=1000, block_size=128)).to(dev)
    ddp = DistributedDataParallel(m, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
    opt = FusedAdamW(ddp.parameters(), lr=3e-3, weight_decay=0.0)
    x = torch.randint(0, 1000, (4, 128), device=dev)
    losses = []
    for _ in range(30):
        opt.zero_grad()
        logits = ddp(x[:, :-1])
        loss = lm.cross_entropy(logits.reshape(-1, logits.shape[-1]), x[:, 1:].reshape(-1))
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] * 0.5, losses


def test_ddp_linear_gradients_written_into_flat_buffer():
    """Native Linear and LayerNorm backwards write dW / db straight into the DDP
    engine's flat gradient slices (no bucket copy), a Linear used twice in one
    backward still gets the sum of both uses, and gradients match an un-wrapped copy."""
    import copy

    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = lm.Linear(128, 256)
            self.b = lm.Linear(256, 128)
            self.shared = lm.Linear(128, 128)
            self.ln = torch.nn.LayerNorm(128)

        def forward(self, x):
            x = lm.layer_norm(x, self.ln.weight, self.ln.bias)
            h = self.shared(self.b(lm.gelu(self.a(x))))
            return self.shared(h)  # second use of the same weight in this backward

    torch.manual_seed(3)
    dev = torch.device(DEV, 0)
    net = Net().to(dev).bfloat16()
    ref = copy.deepcopy(net)
    ddp = DistributedDataParallel(net, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
    copied = []
    orig = ddp._gather_into_bucket

    def spy(b, scale):
        copied.extend(ddp.flat.names[i] for i in ddp._pending[b])
        return orig(b, scale)

    ddp._gather_into_bucket = spy
    x = torch.randn(512, 128, device=dev).bfloat16()
    for it in range(2):
        ddp.zero_grad(set_to_none=True)
        copied.clear()
        ddp(x).float().square().mean().backward()
        assert not {"a.weight", "b.weight", "a.bias", "ln.weight", "ln.bias"} & set(copied), copied
        for name, p in ref.named_parameters():
            p.grad = None
        ref(x).float().square().mean().backward()
        for i, (name, p) in enumerate(net.named_parameters()):
            q = dict(ref.named_parameters())[name]
            assert _rel(p.grad, q.grad) < 2e-2, (it, name)
        assert all(ddp.flat.grad_is_view(i) for i in range(len(ddp.flat.params)))


@pytest.mark.parametrize("fused_add", [False, True])
def test_ddp_norm_weight_used_twice(fused_add):
    """A LayerNorm (gamma, beta) applied twice in one backward: the deferred column-sum path
    (ops/lm.py _NORM_DEFER) must not be taken for it -- the gradient is the sum of both uses,
    equal to an un-wrapped copy's."""
    import copy

    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = lm.Linear(256, 256)
            self.ln = torch.nn.LayerNorm(256)
            self.b = lm.Linear(256, 256)

        def forward(self, x):
            h = self.a(x)
            if fused_add:
                r, h = lm.add_layer_norm(h, x, self.ln.weight, self.ln.bias)
            else:
                h = lm.layer_norm(h, self.ln.weight, self.ln.bias)
            h = self.b(h)
            return lm.layer_norm(h, self.ln.weight, self.ln.bias)  # second use of gamma / beta

    torch.manual_seed(5)
    dev = torch.device(DEV, 0)
    net = Net().to(dev).bfloat16()
    with torch.no_grad():
        net.ln.weight.uniform_(0.5, 1.5)
        net.ln.bias.uniform_(-0.5, 0.5)
    ref = copy.deepcopy(net)
    ddp = DistributedDataParallel(net, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
    x = torch.randn(1024, 256, device=dev).bfloat16()
    for it in range(3):
        ddp.zero_grad(set_to_none=True)
        ddp(x).float().square().mean().backward()
        for p in ref.parameters():
            p.grad = None
        ref(x).float().square().mean().backward()
        refs = dict(ref.named_parameters())
        for name, p in net.named_parameters():
            assert _rel(p.grad, refs[name].grad) < 2e-2, (it, name)


def test_llama_tiny_fsdp_trains_on_gpu():
    from distributed_training_amd.models.llama import Block, Llama, LlamaConfig
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    torch.manual_seed(0)
    dev = torch.device(DEV, 0)
    cfg = LlamaConfig(n_layer=2, n_head=4, n_kv_head=2, n_embd=256, ffn_hidden=512, vocab_size=1024, block_size=256)
    m = Llama(cfg).to(dev)
    m.enable_activation_checkpointing()
    fs = FullyShardedDataParallel(m, comm=RcclComm(0, 1, dev), device=dev, wrap_policy={Block},
                                  param_dtype=torch.bfloat16)
    opt = FusedAdamW(fs.parameters(), lr=3e-3, weight_decay=0.0)
    x = torch.randint(0, 1024, (2, 129), device=dev)
    losses = []
    for _ in range(30):
        opt.zero_grad()
        logits = fs(x[:, :-1])
        loss = lm.cross_entropy(logits.reshape(-1, logits.shape[-1]), x[:, 1:].reshape(-1))
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] * 0.5, losses
    sd = fs.full_state_dict(rank0_only=False)
    assert "layers.0.attention.wqkv.weight" in sd and sd["output.weight"].dtype == torch.float32


@pytest.mark.parametrize("H,Hkv,D,rope", [(4, 4, 64, False), (4, 2, 128, True), (8, 1, 64, True)])
def test_packed_attention_with_rope(H, Hkv, D, rope):
    """Attention on the packed QKV projection output: packed dQKV gradient, RoPE applied in place in the
    forward and inverted on dQ / dK inside the backward kernels' epilogues."""
    torch.manual_seed(3)
    B, S = 2, 160
    qkv = (torch.randn(B, S, (H + 2 * Hkv) * D, device=DEV) * 0.5).bfloat16().requires_grad_()
    cos, sin = lm.rope_tables(S, D, 10000.0, device=DEV)
    do = torch.randn(B, S, H, D, device=DEV).bfloat16()
    o = lm.attention_packed(qkv, H, Hkv, causal=True, rope=(cos, sin) if rope else None)
    o.backward(do)
    ref_in = qkv.detach().float().requires_grad_()
    q, k, v = lm._split_qkv(ref_in, H, Hkv)
    if rope:
        q, k = lm.rope_reference(q, cos, sin), lm.rope_reference(k, cos, sin)
    orf = lm.attention_reference(q.float(), k.float(), v.float(), causal=True)
    orf.backward(do.float())
    assert _rel(o, orf) < 1e-2
    assert _rel(qkv.grad, ref_in.grad) < 2e-2
    if rope:  # in-place RoPE on an intermediate (the model's projection output): bit-identical
        leaf = qkv.detach().clone().requires_grad_()
        o2 = lm.attention_packed(leaf * 1, H, Hkv, causal=True, rope=(cos, sin), rope_inplace=True)
        o2.backward(do)
        assert torch.equal(o2, o) and torch.equal(leaf.grad, qkv.grad)


@pytest.mark.parametrize("N,C", [(300, 768), (1000, 4096)])
@pytest.mark.parametrize("rms", [False, True])
def test_add_norm_fused_residual(rms, N, C):
    torch.manual_seed(4)
    x = torch.randn(N, C, device=DEV).bfloat16().requires_grad_()
    r = torch.randn(N, C, device=DEV).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(C, device=DEV)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(C, device=DEV)).bfloat16().requires_grad_()
    gx = torch.randn(N, C, device=DEV).bfloat16()
    gy = torch.randn(N, C, device=DEV).bfloat16()
    if rms:
        xn, y = lm.add_rms_norm(x, r, w)
    else:
        xn, y = lm.add_layer_norm(x, r, w, b)
    (xn.float() * gx.float()).sum().add((y.float() * gy.float()).sum()).backward()
    xf, rf, wf, bf = (t.detach().float().requires_grad_() for t in (x, r, w, b))
    xs = (xf + rf).bfloat16().float()  # the kernel normalises the stored bf16 sum
    xs = xf + rf + (xs - (xf + rf)).detach()
    if rms:
        yr = xs * torch.rsqrt(xs.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    else:
        yr = F.layer_norm(xs, (C,), wf, bf, 1e-5)
    ((xf + rf) * gx.float()).sum().add((yr * gy.float()).sum()).backward()
    assert _rel(xn, xf + rf) < 1e-2 and _rel(y, yr) < 1e-2
    assert _rel(x.grad, xf.grad) < 2e-2 and _rel(r.grad, rf.grad) < 2e-2
    assert _rel(w.grad, wf.grad) < 2e-2
    if not rms:
        assert _rel(b.grad, bf.grad) < 2e-2


def test_linear_native_bias_grad():
    torch.manual_seed(5)
    x = torch.randn(4, 300, 768, device=DEV).bfloat16().requires_grad_()
    w = (0.05 * torch.randn(2304, 768, device=DEV)).bfloat16().requires_grad_()
    b = torch.randn(2304, device=DEV).bfloat16().requires_grad_()
    dy = torch.randn(4, 300, 2304, device=DEV).bfloat16()
    lm.linear(x, w, b).backward(dy)
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    F.linear(xf, wf, bf).backward(dy.float())
    assert _rel(b.grad, bf.grad) < 1e-2
    assert _rel(w.grad, wf.grad) < 1e-2 and _rel(x.grad, xf.grad) < 1e-2


@pytest.mark.parametrize("chunk", [0, 128])
@pytest.mark.parametrize("V", [50304, 1000])
def test_linear_cross_entropy_fused_head(V, chunk):
    """The head + CE against fp32 autograd: one block (the [T, V] logits) and row blocks of 128
    tokens (chunk=128: blocks of 128, 128 and 1 rows; both gradients formed in the forward)."""
    torch.manual_seed(6)
    N, C = 257, 256
    x = (0.5 * torch.randn(N, C, device=DEV)).bfloat16().requires_grad_()
    w = (0.1 * torch.randn(V, C, device=DEV)).bfloat16().requires_grad_()
    t = torch.randint(0, V, (N,), device=DEV)
    t[::7] = -100
    loss = lm.linear_cross_entropy(x, w, t, chunk=chunk)
    (loss * 3.0).backward()
    xf, wf = (z.detach().float().requires_grad_() for z in (x, w))
    lr = F.cross_entropy(xf @ wf.t(), t, ignore_index=-100)
    (lr * 3.0).backward()
    assert abs(loss.item() - lr.item()) < 2e-2 * abs(lr.item())
    assert _rel(x.grad, xf.grad) < 3e-2 and _rel(w.grad, wf.grad) < 3e-2


def test_chunked_head_ce_peak_memory():
    """Row blocks never hold the [T, V] logits: the op's peak allocation falls by about
    (T - chunk) x V x 2 B against the one-block form."""
    torch.manual_seed(8)
    T, C, V, chunk = 4096, 512, 50304, 1024
    x = (0.5 * torch.randn(T, C, device=DEV)).bfloat16().requires_grad_()
    w = (0.1 * torch.randn(V, C, device=DEV)).bfloat16().requires_grad_()
    t = torch.randint(0, V, (T,), device=DEV)
    peaks, grads = [], []
    for ch in (0, chunk):
        x.grad = w.grad = None
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        lm.linear_cross_entropy(x, w, t, chunk=ch).backward()
        torch.cuda.synchronize()
        peaks.append(torch.cuda.max_memory_allocated() - base)
        grads.append((x.grad.float(), w.grad.float()))
    saved = peaks[0] - peaks[1]
    assert saved > 0.8 * (T - chunk) * V * 2, (peaks, saved)
    assert _rel(grads[1][0], grads[0][0]) < 1e-2 and _rel(grads[1][1], grads[0][1]) < 1e-2


def test_chunked_head_ce_dw_drift_many_blocks():
    """the row-blocked head accumulates dW in bf16 (one rounding per block, hipBLASLt beta = 1) --
    pinned with an explicit tolerance at many blocks (T / chunk = 32) against an fp32 reference: within
    1e-2 norm-relative and within 4x the one-block form's own error (plus a floor).  A second backward
    through the same graph raises instead of returning no gradients."""
    torch.manual_seed(11)
    T, C, V, chunk = 8192, 256, 4096, 256
    x = (0.5 * torch.randn(T, C, device=DEV)).bfloat16().requires_grad_()
    w = (0.1 * torch.randn(V, C, device=DEV)).bfloat16().requires_grad_()
    t = torch.randint(0, V, (T,), device=DEV)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    torch.nn.functional.cross_entropy(xf @ wf.t(), t).backward()
    errs = []
    for ch in (0, chunk):
        x.grad = w.grad = None
        lm.linear_cross_entropy(x, w, t, chunk=ch).backward()
        errs.append((_rel(x.grad, xf.grad), _rel(w.grad, wf.grad)))
    (ex0, ew0), (ex1, ew1) = errs
    assert ex1 < 1e-2 and ew1 < 1e-2, errs
    assert ew1 <= 4 * ew0 + 2e-3, errs
    loss = lm.linear_cross_entropy(x, w, t, chunk=chunk)
    loss.backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="one backward per forward"):
        loss.backward()


def test_chunked_head_ce_no_grad_forward_writes_no_gradient():
    """An evaluation forward (torch.no_grad) of the row-blocked head + CE computes the loss only: the
    weight-gradient destination hook an engine attaches (``_dta_gdest_fwd``) is never asked for a slice
    -- ``needs_input_grad`` alone is still True under no_grad -- and the loss equals the one-block form's."""
    torch.manual_seed(9)
    T, C, V = 600, 256, 1000
    x = (0.5 * torch.randn(T, C, device=DEV)).bfloat16().requires_grad_()
    w = (0.1 * torch.randn(V, C, device=DEV)).bfloat16().requires_grad_()
    t = torch.randint(0, V, (T,), device=DEV)
    asked = []
    w._dta_gdest_fwd = lambda: asked.append(1)
    with torch.no_grad():
        loss = lm.linear_cross_entropy(x, w, t, chunk=128)
        ref = lm.linear_cross_entropy(x, w, t, chunk=0)
    assert not asked and not loss.requires_grad
    assert abs(loss.item() - ref.item()) < 1e-3 * abs(ref.item())
    del w._dta_gdest_fwd


def test_linear_cross_entropy_scale_in_epilogue(monkeypatch):
    """The hand-written head GEMMs (DTA_GEMM=dta) fold the loss-gradient scale grad / count, a device
    scalar, into their epilogues (gemm64 alpha_dev) -- no separate scaling pass -- and match fp32."""
    monkeypatch.setenv("DTA_GEMM", "dta")
    torch.manual_seed(7)
    N, C, V = 768, 384, 2048  # (shapes no other test times: the per-shape choice is memoised)
    x = (0.5 * torch.randn(N, C, device=DEV)).bfloat16().requires_grad_()
    w = (0.1 * torch.randn(V, C, device=DEV)).bfloat16().requires_grad_()
    t = torch.randint(0, V, (N,), device=DEV)
    t[::5] = -100
    calls = dict(lm.GEMM_STATS)
    loss = lm.linear_cross_entropy(x, w, t)
    (loss * 2.5).backward()
    assert lm.GEMM_STATS["dta"] - calls.get("dta", 0) == 3  # forward, input and weight gradients
    xf, wf = (z.detach().float().requires_grad_() for z in (x, w))
    lr = F.cross_entropy(xf @ wf.t(), t, ignore_index=-100)
    (lr * 2.5).backward()
    assert abs(loss.item() - lr.item()) < 2e-2 * abs(lr.item())
    assert _rel(x.grad, xf.grad) < 3e-2 and _rel(w.grad, wf.grad) < 3e-2


@pytest.mark.parametrize("head_chunk", [0, 64])
@pytest.mark.parametrize("arch", ["gpt2", "llama"])
def test_fused_model_matches_fp32_reference(arch, head_chunk, monkeypatch):
    """The whole fused GPU model (packed attention, fused residual norms, native
    bias grads, fused head+CE -- one block or row blocks of 64 tokens, GPT-2's tied
    head/embedding gradient summed) against the same weights run through the
    unfused CPU fp32 path."""
    import copy

    monkeypatch.setattr(lm, "HEAD_CE_CHUNK", head_chunk)

    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(7)
    if arch == "gpt2":
        m = GPT2(GPT2Config(n_layer=2, n_head=4, n_embd=256, vocab_size=1000, block_size=128))
    else:
        m = Llama(LlamaConfig(n_layer=2, n_head=4, n_kv_head=2, n_embd=256, ffn_hidden=512, vocab_size=1000,
                              block_size=128))
    ref = copy.deepcopy(m).float()
    g = m.to(DEV).bfloat16()
    idx = torch.randint(0, 1000, (2, 97))
    loss = g(idx[:, :-1].to(DEV), idx[:, 1:].to(DEV))
    loss.backward()
    lr = ref(idx[:, :-1], idx[:, 1:])
    lr.backward()
    assert abs(loss.item() - lr.item()) < 2e-2 * lr.item()
    for (n, p), (_, q) in zip(g.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad.to(DEV)) < 6e-2, n


@pytest.mark.parametrize("mode", ["dta", "torch"])
def test_swiglu_linear_fused_backward(mode, monkeypatch):
    """(silu(a) * b) W^T with the SwiGLU backward in the input-gradient GEMM's epilogue (DTA_GEMM=dta) or
    hipBLASLt + the SwiGLU-backward kernel (torch) vs fp32 PyTorch autograd."""
    import torch.nn.functional as F

    monkeypatch.setenv("DTA_GEMM", mode)
    monkeypatch.setattr(lm, "_GEMM_CHOICE", {})
    torch.manual_seed(12)
    F_ = 512
    ab = torch.randn(2, 256, 2 * F_, device=DEV).bfloat16().requires_grad_()
    w = (torch.randn(384, F_, device=DEV) * 0.05).bfloat16().requires_grad_()
    calls = dict(lm.GEMM_STATS)
    y = lm.swiglu_linear(ab, w)
    gy = torch.randn_like(y)
    (y.float() * gy.float()).sum().backward()
    if mode == "dta":
        assert lm.GEMM_STATS["dta"] - calls.get("dta", 0) >= 2  # forward and the fused input gradient
    abf, wf = (t.detach().float().requires_grad_() for t in (ab, w))
    a, b = abf.chunk(2, dim=-1)
    yf = F.linear(F.silu(a) * b, wf)
    (yf * gy.float()).sum().backward()
    assert _rel(y, yf) < 1e-2
    assert _rel(ab.grad, abf.grad) < 2e-2 and _rel(w.grad, wf.grad) < 2e-2


@pytest.mark.parametrize("mode", ["dta", "torch"])
def test_gelu_linear_fused_backward(mode, monkeypatch):
    """gelu(h) W^T + b with the GELU backward in the input-gradient GEMM's epilogue (DTA_GEMM=dta)
    or hipBLASLt + the GELU-backward kernel (torch) vs fp32 PyTorch."""
    import torch.nn.functional as F

    monkeypatch.setenv("DTA_GEMM", mode)
    monkeypatch.setattr(lm, "_GEMM_CHOICE", {})
    torch.manual_seed(11)
    h = torch.randn(4, 128, 256, device=DEV).bfloat16().requires_grad_()
    w = (torch.randn(384, 256, device=DEV) * 0.05).bfloat16().requires_grad_()
    b = (torch.randn(384, device=DEV) * 0.1).bfloat16().requires_grad_()
    y = lm.gelu_linear(h, w, b)
    gy = torch.randn_like(y)
    (y.float() * gy.float()).sum().backward()
    hf, wf, bf = (t.detach().float().requires_grad_() for t in (h, w, b))
    yf = F.linear(F.gelu(hf, approximate="tanh"), wf, bf)
    (yf * gy.float()).sum().backward()
    assert _rel(y, yf) < 1e-2
    for t, r in ((h, hf), (w, wf), (b, bf)):
        assert _rel(t.grad, r.grad) < 2e-2
    if mode == "dta":
        assert lm._GEMM_CHOICE.get(("dgelu", 512, 256, 384), 0) != 0


@pytest.mark.parametrize("mode", ["dta", "torch"])
def test_mlp_gelu_in_up_projection_epilogue(mode, monkeypatch):
    """GPT-2 MLP with the GELU in c_fc's epilogue (dual store of h and gelu(h), DTA_GEMM=dta: the
    64-deep GEMM; torch: hipBLASLt + the GELU kernel) and its backward folded into c_proj's
    input-gradient GEMM, vs fp32 PyTorch: output and every parameter / input gradient."""
    import torch.nn.functional as F

    monkeypatch.setenv("DTA_GEMM", mode)
    monkeypatch.setattr(lm, "_GEMM_CHOICE", {})
    torch.manual_seed(13)
    x = torch.randn(4, 128, 256, device=DEV).bfloat16().requires_grad_()
    w1 = (torch.randn(1024, 256, device=DEV) * 0.05).bfloat16().requires_grad_()
    b1 = (torch.randn(1024, device=DEV) * 0.1).bfloat16().requires_grad_()
    w2 = (torch.randn(256, 1024, device=DEV) * 0.05).bfloat16().requires_grad_()
    b2 = (torch.randn(256, device=DEV) * 0.1).bfloat16().requires_grad_()
    before = dict(lm.GEMM_STATS)
    h, a = lm.linear_gelu(x, w1, b1)
    assert not a.requires_grad
    y = lm.gelu_linear(h, w2, b2, a=a)
    gy = torch.randn_like(y)
    (y.float() * gy.float()).sum().backward()
    ref = [t.detach().float().requires_grad_() for t in (x, w1, b1, w2, b2)]
    yf = F.linear(F.gelu(F.linear(ref[0], ref[1], ref[2]), approximate="tanh"), ref[3], ref[4])
    (yf * gy.float()).sum().backward()
    assert _rel(y, yf) < 1e-2
    assert _rel(a, F.gelu(h.float(), approximate="tanh")) < 1e-2
    for t, r in zip((x, w1, b1, w2, b2), ref):
        assert _rel(t.grad, r.grad) < 2e-2
    if mode == "dta":
        assert lm._GEMM_CHOICE.get(("fwd_gelub", 512, 1024, 256), 0) >= lm.K64
        assert lm.GEMM_STATS["dta"] > before["dta"]


@pytest.mark.parametrize("threshold", ["0", "1", "200"])
def test_ddp_deferred_grouped_weight_gradients(threshold, monkeypatch):
    """Weight + bias gradients deferred and computed by grouped launches (DTA_WGRAD_GROUP tiles
    per flush; 1 = a flush per weight, 200 = one flush at the end of the backward) match an
    unwrapped copy; a weight used twice is never deferred."""
    import copy

    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    monkeypatch.setenv("DTA_WGRAD_GROUP", threshold)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = lm.Linear(256, 768)
            self.b = lm.Linear(768, 512)
            self.c = lm.Linear(512, 256)
            self.shared = lm.Linear(256, 256)

        def forward(self, x):
            h = lm.gelu_linear(self.a(x), self.b.weight, self.b.bias)
            return self.shared(self.shared(self.c(h)))

    torch.manual_seed(5)
    dev = torch.device(DEV, 0)
    net = Net().to(dev).bfloat16()
    ref = copy.deepcopy(net)
    ddp = DistributedDataParallel(net, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
    x = torch.randn(2, 512, 256, device=dev).bfloat16()
    for it in range(3):
        ddp.zero_grad(set_to_none=True)
        n0, g0 = lm.GEMM_STATS["deferred_wgrad"], lm.GEMM_STATS["group_launches"]
        ddp(x).float().square().mean().backward()
        deferred = lm.GEMM_STATS["deferred_wgrad"] - n0
        launches = lm.GEMM_STATS["group_launches"] - g0
        assert deferred == (0 if threshold == "0" else 3), deferred  # a, b, c; never `shared`
        assert launches == {"0": 0, "1": 3, "200": 1}[threshold], launches
        for p in ref.parameters():
            p.grad = None
        ref(x).float().square().mean().backward()
        rp = dict(ref.named_parameters())
        for name, p in net.named_parameters():
            assert _rel(p.grad, rp[name].grad) < 2e-2, (threshold, it, name)


def test_ddp_deferred_after_raised_backward(monkeypatch):
    """A backward that RAISES after deferring weight gradients: the next step starts a
    fresh generation -- the abandoned step's queue is dropped and the end-of-backward flush is queued
    again, so the next step's gradients match an unwrapped copy (no stale entries, no unwritten
    slices read by the optimizer)."""
    import copy

    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    monkeypatch.setenv("DTA_WGRAD_GROUP", "200")  # one flush at the end of the backward

    class Boom(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.clone()

        @staticmethod
        def backward(ctx, g):
            raise RuntimeError("injected backward failure")

    torch.manual_seed(9)
    dev = torch.device(DEV, 0)
    net = torch.nn.Sequential(*[lm.Linear(512, 512) for _ in range(3)]).to(dev).bfloat16()
    ref = copy.deepcopy(net)
    ddp = DistributedDataParallel(net, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
    x = torch.randn(2, 512, 512, device=dev).bfloat16()
    ddp.zero_grad(set_to_none=True)
    n0 = lm.GEMM_STATS["deferred_wgrad"]
    # the failure sits BELOW the first layer, so layers 2 and 3 have deferred their weight gradients
    with pytest.raises(RuntimeError, match="injected"):
        ddp(Boom.apply(x.clone().requires_grad_())).float().square().mean().backward()
    assert lm.GEMM_STATS["deferred_wgrad"] - n0 >= 1
    assert lm.wgrad_pending()  # the raised backward never flushed
    for it in range(2):
        ddp.zero_grad(set_to_none=True)
        x = torch.randn(2, 512, 512, device=dev).bfloat16()
        ddp(x).float().square().mean().backward()
        assert not lm.wgrad_pending()
        for p in ref.parameters():
            p.grad = None
        ref(x).float().square().mean().backward()
        rp = dict(ref.named_parameters())
        for name, p in net.named_parameters():
            assert _rel(p.grad, rp[name].grad) < 2e-2, (it, name)


@pytest.mark.parametrize("impl", [1, 2])
def test_gemm_wgrad_group_vs_fp32(impl):
    """The grouped weight-gradient launch (full token reduction, several problems' tiles in one
    launch) on problems of different shapes and K, strided operands, vs fp32 torch: csrc/gemm_k64.hip's
    (impl 1: 256 x 256 tiles, bias gradients on the MFMA pipe split over the waves sharing A rows) and
    csrc/gemm_w4.hip's (impl 2: edge tiles and K tails, no bias gradients -- refused)."""
    from distributed_training_amd.ops import native

    torch.manual_seed(12)
    shapes = [(1024, 512, 256), (2048, 256, 768), (512, 768, 512), (192, 256, 256),
              (8192, 768, 768)]  # (K, M, N)
    if impl == 2:  # W4: edge tiles and K tails too
        shapes += [(520, 264, 776), (136, 1000, 200)]
    A, B, Cs, D = [], [], [], []
    for K, M, N in shapes:
        wide = torch.randn(K, M + 64, device=DEV).bfloat16()
        A.append(wide[:, 32:32 + M])
        B.append(torch.randn(K, N, device=DEV).bfloat16())
        Cs.append(torch.empty(M, N, device=DEV, dtype=torch.bfloat16))
        D.append(torch.empty(M, device=DEV, dtype=torch.bfloat16))
    D[1] = None  # a problem without bias
    if impl == 2:  # W4: no bias gradients (refused), the products alone
        with pytest.raises(RuntimeError, match="no bias gradients"):
            native().gemm_wgrad_group(A, B, Cs, D, -1, impl)
        D = [None] * len(shapes)
    native().gemm_wgrad_group(A, B, Cs, D, -1, impl)
    for i in range(len(shapes)):
        assert _rel(Cs[i], A[i].float().t() @ B[i].float()) < 1e-2, i
        if D[i] is not None:
            assert _rel(D[i], A[i].float().sum(0)) < 1e-2, i


def test_ddp_deferred_flush_between_backward_and_bucket_launch(monkeypatch):
    """A grouped flush that falls between a deferred weight's backward and its bucket's launch
    (DTA_WGRAD_GROUP=8: every second 512 x 512 weight flushes; buckets span several layers):
    every gradient is adopted as its flat-buffer view (no AccumulateGrad clone of the not yet
    written slice) and matches an unwrapped copy on every iteration (a stale slice would carry
    the previous iteration's gradient)."""
    import copy

    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    monkeypatch.setenv("DTA_WGRAD_GROUP", "8")
    torch.manual_seed(6)
    dev = torch.device(DEV, 0)
    net = torch.nn.Sequential(*[lm.Linear(512, 512) for _ in range(6)]).to(dev).bfloat16()
    ref = copy.deepcopy(net)
    ddp = DistributedDataParallel(net, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16,
                                  bucket_cap_mb=1.5, first_bucket_mb=1.0)
    assert len(ddp.buckets) >= 2
    for it in range(3):
        x = torch.randn(2, 512, 512, device=dev).bfloat16()
        ddp.zero_grad(set_to_none=True)
        n0 = lm.GEMM_STATS["deferred_wgrad"]
        (ddp(x).float().square().mean() * (it + 1)).backward()
        assert lm.GEMM_STATS["deferred_wgrad"] - n0 == 6
        fl = ddp.flat
        assert all(fl.grad_is_view(i) for i in range(len(fl.params)))
        for p in ref.parameters():
            p.grad = None
        (ref(x).float().square().mean() * (it + 1)).backward()
        rp = dict(ref.named_parameters())
        for name, p in net.named_parameters():
            assert _rel(p.grad, rp[name].grad) < 2e-2, (it, name)


@pytest.mark.parametrize("opt_name,group", [("adamw", "200"), ("adamw", "8"), ("sgd", "0")])
def test_ddp_optimizer_in_backward_bit_identical(opt_name, group, monkeypatch):
    """DDP overlap_optimizer (the update of each bucket on a side stream inside the backward,
    after its deferred weight gradients are written) gives the same bits as backward + step()."""
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops.optim import FusedAdamW, FusedSGD
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    monkeypatch.setenv("DTA_WGRAD_GROUP", group)
    dev = torch.device(DEV, 0)
    g = torch.Generator(device="cpu").manual_seed(3)
    data = [torch.randint(0, 1024, (2, 257), generator=g).to(dev) for _ in range(4)]
    finals = []
    for overlap in (False, True):
        torch.manual_seed(0)
        model = GPT2(GPT2Config(n_layer=3, n_head=4, n_embd=256, vocab_size=1024, block_size=256)).to(dev)
        ddp = DistributedDataParallel(model, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16,
                                      bucket_cap_mb=1.0, first_bucket_mb=0.25)
        assert len(ddp.buckets) >= 3
        opt = (FusedAdamW(ddp.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1) if opt_name == "adamw"
               else FusedSGD(ddp.parameters(), lr=0.05, momentum=0.9))
        assert ddp.overlap_optimizer(opt) if overlap else True
        losses = []
        for x in data:
            opt.zero_grad(set_to_none=True)
            loss = ddp(x[:, :-1], x[:, 1:])
            loss.backward()
            opt.step()
            losses.append(loss.float())
        torch.cuda.synchronize()
        finals.append((torch.stack(losses).cpu(), ddp.flat.master.clone(), ddp.flat.compute.clone()))
    assert torch.equal(finals[0][0], finals[1][0])
    assert torch.equal(finals[0][1], finals[1][1])
    assert torch.equal(finals[0][2], finals[1][2])
    assert not torch.equal(finals[0][1], finals[0][1] * 0)


def test_embedding_backward_vs_fp32():
    """Sorted-run embedding backward (repeated ids, out-of-order) vs fp32 torch."""
    torch.manual_seed(13)
    V, C = 300, 256
    w = (torch.randn(V, C, device=DEV) * 0.02).bfloat16().requires_grad_()
    idx = torch.randint(0, 40, (4, 129), device=DEV)  # many repeats of each id
    idx[0, :5] = V - 1
    y = lm.embedding(idx, w)
    assert torch.equal(y, F.embedding(idx, w.detach()))
    dy = torch.randn(4, 129, C, device=DEV).bfloat16()
    y.backward(dy)
    ref = torch.zeros(V, C, device=DEV).index_add_(0, idx.reshape(-1), dy.reshape(-1, C).float())
    assert _rel(w.grad, ref) < 1e-2
    assert w.grad[40:V - 1].abs().max().item() == 0


@pytest.mark.parametrize("N", [1, 777, 8192, 70000])
def test_ce_mean_matches_torch(N):
    """The one-launch CE mean (csrc/lm_ops.hip ce_mean_kernel): sum(rows) / max(1, #valid) and the
    count, against the torch-op form; every target ignored -> count 1; repeat calls bit-identical."""
    from distributed_training_amd.ops import native

    torch.manual_seed(N)
    rows = torch.rand(N, device=DEV) * 10
    tgt = torch.randint(0, 50, (N,), device=DEV)
    tgt[::3] = -100
    loss, count = native().ce_mean(rows, tgt, -100)
    ref_c = (tgt != -100).sum().clamp_min(1).float()
    assert count.item() == ref_c.item()
    assert abs(loss.item() - (rows.double().sum() / ref_c.double()).item()) <= 1e-5 * max(1.0, loss.item())
    loss2, _ = native().ce_mean(rows, tgt, -100)
    assert torch.equal(loss, loss2)
    _, c0 = native().ce_mean(rows, torch.full_like(tgt, -100), -100)
    assert c0.item() == 1.0


@pytest.mark.parametrize("T,V", [(1, 7), (1000, 40), (8192, 50304), (12289, 50304), (16384, 65535)])
def test_sort_ids_matches_torch(T, V):
    """The single-workgroup id sort (csrc/sort_ids.hip) returns torch.sort(stable=True)'s ids and
    positions bit for bit (many repeats: the order inside each run is the stability check); an id
    outside [0, V) comes back as V."""
    from distributed_training_amd.ops import native

    g = torch.Generator(device="cpu").manual_seed(T)
    ids = torch.randint(0, V, (T,), generator=g).to(DEV)
    sid, perm = native().sort_ids(ids, V)
    ref_s, ref_p = torch.sort(ids, stable=True)
    assert torch.equal(sid, ref_s) and torch.equal(perm, ref_p)
    if T > 2:
        ids[1], ids[2] = -3, V + 5
        sid, perm = native().sort_ids(ids, V)
        assert torch.equal(sid[-2:], torch.full((2,), V, device=DEV))
        assert sorted(perm[-2:].tolist()) == [1, 2]


def test_add_position_vs_fp32():
    """x + w[:S] (learned positions as a view, no ids): forward exact, dx = dy, dw = dy summed over
    the batch in rows < S and zero past S, against fp32 torch."""
    torch.manual_seed(14)
    P, S, C = 96, 80, 256
    w = (torch.randn(P, C, device=DEV) * 0.02).bfloat16().requires_grad_()
    x = torch.randn(3, S, C, device=DEV).bfloat16().requires_grad_()
    y = lm.add_position(x, w)
    assert torch.equal(y, x.detach() + w.detach()[:S])
    dy = torch.randn(3, S, C, device=DEV).bfloat16()
    y.backward(dy)
    assert torch.equal(x.grad, dy)
    ref = dy.float().sum(0)
    assert _rel(w.grad[:S], ref) < 1e-2
    assert w.grad[S:].abs().max().item() == 0


def test_tied_embedding_gradient_accumulated_in_place():
    """GPT-2 under the DDP engine: the token rows are added into the tied head's gradient slice
    (no autograd sum); wte / wpe gradients match the same model without the engine."""
    import copy

    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    dev = torch.device(DEV, 0)
    model = GPT2(GPT2Config(n_layer=2, n_head=2, n_embd=128, vocab_size=512, block_size=128)).to(dev)
    ref = copy.deepcopy(model).bfloat16()
    ddp = DistributedDataParallel(model, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
    x = torch.randint(0, 64, (2, 129), device=dev)  # repeated tokens
    for _ in range(2):
        ddp.zero_grad(set_to_none=True)
        ddp(x[:, :-1], x[:, 1:]).backward()
        for p in ref.parameters():
            p.grad = None
        ref(x[:, :-1], x[:, 1:]).backward()
        fl = ddp.flat
        i = fl.names.index("wte.weight")
        assert fl.grad_is_view(i)
        assert _rel(model.wte.weight.grad, ref.wte.weight.grad) < 2e-2
        assert _rel(model.wpe.weight.grad, ref.wpe.weight.grad) < 2e-2


def test_tied_embedding_gradient_fsdp_one_rank():
    """Same under the FSDP engine (one rank): the token rows go into the root unit's piece of the
    tied weight in place; the SGD update of wte / wpe matches the unwrapped model's."""
    import copy

    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    torch.manual_seed(0)
    dev = torch.device(DEV, 0)
    model = GPT2(GPT2Config(n_layer=2, n_head=2, n_embd=128, vocab_size=512, block_size=128)).to(dev)
    ref = copy.deepcopy(model).bfloat16()
    w0 = {k: v.detach().float().clone() for k, v in model.state_dict().items()}
    f = FullyShardedDataParallel(model, comm=RcclComm(0, 1, dev), device=dev, wrap_policy={GPT2.block_class},
                                 param_dtype=torch.bfloat16)
    opt = FusedSGD(f.parameters(), lr=1.0)
    x = torch.randint(0, 64, (2, 129), device=dev)
    opt.zero_grad(set_to_none=True)
    f(x[:, :-1], x[:, 1:]).backward()
    opt.step()
    ref(x[:, :-1], x[:, 1:]).backward()
    sd = f.full_state_dict(rank0_only=False)
    for name in ("wte.weight", "wpe.weight"):
        upd = w0[name].cpu() - sd[name].float().cpu()
        assert _rel(upd, dict(ref.named_parameters())[name].grad.cpu()) < 3e-2, name


def test_graphed_ddp_step_matches_eager():
    """The whole GPT-2 DDP step (zero_grad, forward, backward with bucket hooks and deferred
    weight gradients, fused AdamW) captured as one hipGraph and replayed: same losses and
    the same parameters, bit for bit, as the eager steps on the same batches."""
    from distributed_training_amd.engine.step_graph import GraphedStep
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    dev = torch.device(DEV, 0)
    g = torch.Generator(device="cpu").manual_seed(4)
    data = [torch.randint(0, 1024, (2, 257), generator=g).to(dev) for _ in range(4)]
    seq = [data[0]] * 3 + data[1:]  # GraphedStep's 3 warm-up steps train on the static batch
    out = []
    for graphed in (False, True):
        torch.manual_seed(0)
        model = GPT2(GPT2Config(n_layer=2, n_head=4, n_embd=256, vocab_size=1024, block_size=256)).to(dev)
        ddp = DistributedDataParallel(model, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
        opt = FusedAdamW(ddp.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1)

        def step(xb):
            opt.zero_grad(set_to_none=True)
            loss = ddp(xb[:, :-1], xb[:, 1:])
            loss.backward()
            opt.step()
            return loss

        losses = []
        if graphed:
            gs = GraphedStep(step, [data[0].clone()], warmup=3)
            for xb in seq[3:]:
                losses.append(gs(xb).float().clone())
        else:
            for xb in seq:
                losses.append(step(xb).float().clone())
            losses = losses[3:]
        torch.cuda.synchronize()
        out.append((torch.stack(losses).cpu(), ddp.flat.master.clone()))
    assert torch.equal(out[0][0], out[1][0]), (out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


def test_fsdp_one_rank_step_graph_matches_eager():
    """FSDP at one rank (every unit aliases its shard) captured as one hipGraph: the same losses
    and fp32 master weights, bit for bit, as the eager steps on the same batches."""
    from distributed_training_amd.engine.step_graph import GraphedStep
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel, lm_wrap_policy

    dev = torch.device(DEV, 0)
    g = torch.Generator(device="cpu").manual_seed(6)
    data = [torch.randint(0, 1024, (2, 257), generator=g).to(dev) for _ in range(4)]
    seq = [data[0]] * 3 + data[1:]
    out = []
    for graphed in (False, True):
        torch.manual_seed(0)
        model = GPT2(GPT2Config(n_layer=2, n_head=4, n_embd=256, vocab_size=1024, block_size=256)).to(dev)
        w = FullyShardedDataParallel(model, comm=RcclComm(0, 1, dev), device=dev, wrap_policy=lm_wrap_policy(model),
                                     param_dtype=torch.bfloat16)
        assert w.graph_capturable()
        opt = FusedAdamW(w.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1)

        def step(xb):
            opt.zero_grad(set_to_none=True)
            loss = w(xb[:, :-1], xb[:, 1:])
            loss.backward()
            opt.step()
            return loss

        losses = []
        if graphed:
            gs = GraphedStep(step, [data[0].clone()], warmup=3, engine=w)
            assert gs.ok, gs.error
            for xb in seq[3:]:
                losses.append(gs(xb).float().clone())
        else:
            for xb in seq:
                losses.append(step(xb).float().clone())
            losses = losses[3:]
        torch.cuda.synchronize()
        out.append((torch.stack(losses).cpu(), w.shards.master.clone()))
    assert torch.equal(out[0][0], out[1][0]), (out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


def test_fsdp_weight_used_twice_first_claim():
    """FSDP unit whose FIRST gradient piece of the backward belongs to a weight used twice: the
    buffer creation of that first claim must not erase the claim (the second use would get the
    same piece and overwrite the first use's gradient)."""
    import copy

    from distributed_training_amd.ops.optim import FusedSGD
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = lm.Linear(256, 256)
            self.shared = lm.Linear(256, 256)

        def forward(self, x):
            return self.shared(self.shared(self.a(x)))

    torch.manual_seed(8)
    dev = torch.device(DEV, 0)
    net = Net().to(dev)
    ref = copy.deepcopy(net).bfloat16()
    w0 = {k: v.detach().float().cpu().clone() for k, v in net.state_dict().items()}
    f = FullyShardedDataParallel(net, comm=RcclComm(0, 1, dev), device=dev, param_dtype=torch.bfloat16)
    opt = FusedSGD(f.parameters(), lr=1.0)
    x = torch.randn(512, 256, device=dev).bfloat16()
    opt.zero_grad(set_to_none=True)
    f(x).float().square().mean().backward()
    opt.step()
    ref(x).float().square().mean().backward()
    sd = f.full_state_dict(rank0_only=False)
    rp = dict(ref.named_parameters())
    for name in rp:
        upd = w0[name] - sd[name].float().cpu()
        assert _rel(upd, rp[name].grad.float().cpu()) < 3e-2, name



@pytest.mark.parametrize("opt_name", ["adamw", "sgd"])
def test_fsdp_optimizer_in_backward_bit_identical(opt_name):
    """FSDP overlap_optimizer at one rank (each unit's shard, aliased by the unit, updated on a
    side stream right after the unit's backward; the Llama-style lm_wrap_policy units with the
    tied GPT-2 embedding) gives the same bits as backward + step()."""
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops.optim import FusedAdamW, FusedSGD
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel, lm_wrap_policy

    dev = torch.device(DEV, 0)
    g = torch.Generator(device="cpu").manual_seed(4)
    data = [torch.randint(0, 1024, (2, 257), generator=g).to(dev) for _ in range(4)]
    finals = []
    for overlap in (False, True):
        torch.manual_seed(0)
        model = GPT2(GPT2Config(n_layer=3, n_head=4, n_embd=256, vocab_size=1024, block_size=256)).to(dev)
        fs = FullyShardedDataParallel(model, comm=RcclComm(0, 1, dev), device=dev, wrap_policy=lm_wrap_policy(model),
                                      param_dtype=torch.bfloat16)
        assert len(fs.units) >= 4
        opt = (FusedAdamW(fs.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1) if opt_name == "adamw"
               else FusedSGD(fs.parameters(), lr=0.05, momentum=0.9))
        assert fs.overlap_optimizer(opt) if overlap else True
        losses = []
        for x in data:
            opt.zero_grad(set_to_none=True)
            loss = fs(x[:, :-1], x[:, 1:])
            loss.backward()
            opt.step()
            losses.append(loss.float())
        torch.cuda.synchronize()
        finals.append((torch.stack(losses).cpu(), fs.shards.master.clone(), fs.shards.compute.clone()))
    assert torch.equal(finals[0][0], finals[1][0])
    assert torch.equal(finals[0][1], finals[1][1])
    assert torch.equal(finals[0][2], finals[1][2])


def test_fsdp_step_graph_capture_failure_then_eager():
    """a step-graph capture that fails MID-BACKWARD under the FSDP engine (one rank,
    graph_capturable) resets the engine (FullyShardedDataParallel.reset_iteration) -- the eager steps
    that follow bind / write every gradient and train exactly like a run that never tried to capture."""
    from distributed_training_amd.engine.step_graph import GraphedStep
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel, lm_wrap_policy

    dev = torch.device(DEV, 0)
    g = torch.Generator(device="cpu").manual_seed(8)
    data = [torch.randint(0, 1024, (2, 129), generator=g).to(dev) for _ in range(3)]
    failing = [False]

    class Boom(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.view_as(x)

        @staticmethod
        def backward(ctx, gr):
            if failing[0]:
                raise RuntimeError("op not capturable")
            return gr

    finals = []
    for try_graph in (False, True):
        torch.manual_seed(0)
        model = GPT2(GPT2Config(n_layer=3, n_head=4, n_embd=256, vocab_size=1024, block_size=128)).to(dev)
        model.h[1].register_forward_hook(lambda m, a, out: (Boom.apply(out[0]), out[1]))
        fs = FullyShardedDataParallel(model, comm=RcclComm(0, 1, dev), device=dev, wrap_policy=lm_wrap_policy(model),
                                      param_dtype=torch.bfloat16)
        opt = FusedAdamW(fs.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1)

        def step(xb):
            failing[0] = torch.cuda.is_current_stream_capturing()
            opt.zero_grad(set_to_none=True)
            loss = fs(xb[:, :-1], xb[:, 1:])
            loss.backward()
            opt.step()
            return loss

        if try_graph:
            assert fs.graph_capturable()
            gs = GraphedStep(step, [data[0].clone()], warmup=1, engine=fs)  # one real step, then the capture
            assert not gs.ok and "not capturable" in str(gs.error)
            failing[0] = False
            assert not fs._cb_queued and not fs._pending_rs and not any(u.in_backward for u in fs.units)
            rest = data[1:]
        else:
            rest = data
        for x in rest:
            step(x)
        torch.cuda.synchronize()
        finals.append(fs.shards.master.clone())
    assert torch.equal(finals[0], finals[1])


@pytest.mark.parametrize("ckpt", [False, True])
def test_fsdp_deferred_grouped_weight_gradients(ckpt, monkeypatch):
    """Under the FSDP engine the single-use weights' gradients are deferred into grouped launches
    (ops/lm.py _DEFER) and written into the unit pieces before the unit's gradient is used: the same
    training trajectory as with deferral off (DTA_FSDP_WGRAD_DEFER=0: per-weight kernels), within
    bf16 rounding of the two reduction orders; with activation checkpointing too."""
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.comm import RcclComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel, lm_wrap_policy

    dev = torch.device(DEV, 0)
    g = torch.Generator(device="cpu").manual_seed(6)
    data = [torch.randint(0, 1024, (2, 257), generator=g).to(dev) for _ in range(3)]
    runs = []
    for defer in ("1", "0"):
        monkeypatch.setenv("DTA_FSDP_WGRAD_DEFER", defer)
        torch.manual_seed(0)
        model = GPT2(GPT2Config(n_layer=3, n_head=4, n_embd=256, vocab_size=1024, block_size=256)).to(dev)
        if ckpt:
            model.enable_activation_checkpointing()
        fs = FullyShardedDataParallel(model, comm=RcclComm(0, 1, dev), device=dev, wrap_policy=lm_wrap_policy(model),
                                      param_dtype=torch.bfloat16)
        assert fs._defer_wgrad == (defer == "1")
        opt = FusedAdamW(fs.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1)
        before = lm.GEMM_STATS["deferred_wgrad"]
        losses = []
        for x in data:
            opt.zero_grad(set_to_none=True)
            loss = fs(x[:, :-1], x[:, 1:])
            loss.backward()
            opt.step()
            losses.append(loss.float().item())
        torch.cuda.synchronize()
        runs.append((losses, fs.shards.master.clone(), lm.GEMM_STATS["deferred_wgrad"] - before))
    (l1, m1, d1), (l0, m0, d0) = runs
    assert d0 == 0 and (ckpt or d1 >= 3 * 4 * 3), (d1, d0)  # every block's four Linear weights, every step
    # (under activation checkpointing the recomputed forward counts each weight a second time: not
    # single-use, so nothing is deferred -- the per-weight path, the same trajectory)
    for a, b in zip(l1, l0):
        assert abs(a - b) < 2e-3 * abs(b), (l1, l0)
    assert _rel(m1, m0) < 1e-3
