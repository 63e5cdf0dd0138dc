"""General bf16 GEMM (csrc/gemm_bf16.hip) against an fp32 PyTorch reference of
the same op on the same bf16 inputs: the three operand layouts (forward NT,
input-gradient NN, weight-gradient TN), every tile shape, strided operands and
the fused epilogues (alpha, bias, GELU, residual, fp32 output)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

LAYOUTS = [(False, False), (False, True), (True, True), (True, False)]


def _ops(M, N, K, a_t, b_t, gen, scale=1.0):
    a = (torch.randn(K, M, generator=gen) if a_t else torch.randn(M, K, generator=gen)) * scale
    b = (torch.randn(K, N, generator=gen) if b_t else torch.randn(N, K, generator=gen)) * scale
    a, b = a.bfloat16().cuda(), b.bfloat16().cuda()
    A = a.float().t() if a_t else a.float()
    B = b.float() if b_t else b.float().t()
    return a, b, A @ B  # [M, N] fp32 reference


def _close(got, want, K):
    # bf16 output rounding (2^-8 relative) + fp32 accumulation-order noise
    tol = 4e-3 * want.abs().max().item() + 1e-3 * K ** 0.5
    err = (got.float() - want).abs().max().item()
    assert err <= tol, (err, tol)


@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
@pytest.mark.parametrize("tile,M,N,K", [(1, 512, 512, 256), (2, 512, 384, 96), (3, 384, 256, 1056),
                                        (0, 1024, 768, 768)])
def test_gemm_layouts_and_tiles(a_t, b_t, tile, M, N, K):
    from distributed_training_amd.ops import native

    gen = torch.Generator().manual_seed(M + N + K + 7 * a_t + 3 * b_t)
    a, b, want = _ops(M, N, K, a_t, b_t, gen)
    got = native().gemm(a, b, a_t, b_t, tile=tile)
    torch.cuda.synchronize()
    _close(got, want, K)


def test_gemm_asymmetric_exact():
    """Small integers: every product and partial sum is exact in fp32, so any
    transposition / fragment-order mistake shows as a mismatch."""
    from distributed_training_amd.ops import native

    gen = torch.Generator().manual_seed(3)
    for a_t, b_t in LAYOUTS:
        M, N, K = 256, 256, 64
        a = torch.randint(-3, 4, (K, M) if a_t else (M, K), generator=gen).float()
        b = torch.randint(-3, 4, (K, N) if b_t else (N, K), generator=gen).float()
        want = (a.t() if a_t else a) @ (b if b_t else b.t())
        got = native().gemm(a.bfloat16().cuda(), b.bfloat16().cuda(), a_t, b_t, out_f32=True)
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), want), (a_t, b_t)


def test_gemm_epilogues_and_strides():
    from distributed_training_amd.ops import native

    gen = torch.Generator().manual_seed(11)
    M, N, K = 512, 768, 320
    xs = torch.randn(M, K + 64, generator=gen).bfloat16().cuda()[:, 16:16 + K]  # row stride K+64
    w = torch.randn(N, K, generator=gen).bfloat16().cuda() * 0.1
    bias = torch.randn(N, generator=gen).bfloat16().cuda()
    res = torch.randn(M, N, generator=gen).bfloat16().cuda()
    ref = xs.float() @ w.float().t()
    # bias + GELU (fp32 epilogue, one rounding) -- the GPT-2 MLP up-projection
    got = native().gemm(xs, w, bias=bias, act=2)
    want = F.gelu(ref + bias.float(), approximate="tanh")
    _close(got, want, K)
    # alpha + bias + residual: round(round(alpha * xW^T + b) + res)
    got = native().gemm(xs, w, alpha=0.5, bias=bias, residual=res)
    want = ((0.5 * ref + bias.float()).bfloat16().float() + res.float())
    _close(got, want, K)
    # fp32 output into a strided destination
    out = torch.zeros(M, N + 32, device="cuda")
    native().gemm(xs, w, out=out[:, :N], out_f32=True)
    torch.cuda.synchronize()
    assert torch.all(out[:, N:] == 0)
    _close(out[:, :N], ref, K)


def test_gemm_rejects_uncovered_shapes():
    from distributed_training_amd.ops import native

    a = torch.zeros(100, 64, dtype=torch.bfloat16, device="cuda")
    b = torch.zeros(128, 64, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(RuntimeError):
        native().gemm(a, b)  # M = 100: no tile divides it
    with pytest.raises(RuntimeError):
        native().gemm(torch.zeros(128, 48, dtype=torch.bfloat16, device="cuda"),
                      torch.zeros(128, 48, dtype=torch.bfloat16, device="cuda"))  # K % 32


@pytest.mark.parametrize("mode", ["dta", "torch", "auto"])
@pytest.mark.parametrize("bias", [True, False])
def test_linear_through_gemm_dispatch(mode, bias, monkeypatch):
    """lm.linear forward + backward (dx, dW, db) through the GEMM dispatcher, each
    implementation forced, vs fp32 PyTorch on the same bf16 inputs."""
    from distributed_training_amd.ops import lm

    monkeypatch.setenv("DTA_GEMM", mode)
    monkeypatch.setattr(lm, "_GEMM_CHOICE", {})
    gen = torch.Generator().manual_seed(5)
    T, K, N = 1024, 512, 1536  # N x K output 12 x 4 tiles of 128: > split-K limit? no -> wgrad split-K
    x = torch.randn(T, K, generator=gen).bfloat16().cuda().requires_grad_(True)
    w = (torch.randn(N, K, generator=gen) * 0.05).bfloat16().cuda().requires_grad_(True)
    b = torch.randn(N, generator=gen).bfloat16().cuda().requires_grad_(True) if bias else None
    dy = torch.randn(T, N, generator=gen).bfloat16().cuda()
    before = dict(lm.GEMM_STATS)
    y = lm.linear(x, w, b)
    y.backward(dy)
    if mode == "dta":
        assert lm.GEMM_STATS["dta"] >= before["dta"] + 2  # forward and input gradient on the dta kernel
    if mode == "torch":
        assert lm.GEMM_STATS["dta"] == before["dta"]
    xf, wf = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    bf = b.detach().float().requires_grad_(True) if bias else None
    yf = F.linear(xf, wf, bf)
    yf.backward(dy.float())
    _close(y, yf.detach(), K)
    _close(x.grad, xf.grad, N)
    _close(w.grad, wf.grad, T)
    if bias:
        _close(b.grad, bf.grad, T)


def test_big_weight_gradient_uses_general_gemm(monkeypatch):
    """Weight gradients above the split-K kernel's tile limit go through the
    dispatcher (dta TN layout) -- Llama-size outputs."""
    from distributed_training_amd.ops import lm

    monkeypatch.setenv("DTA_GEMM", "dta")
    monkeypatch.setattr(lm, "_GEMM_CHOICE", {})
    gen = torch.Generator().manual_seed(9)
    T, K, N = 512, 2048, 4096  # 32 x 16 = 512 output tiles of 128
    x = torch.randn(T, K, generator=gen).bfloat16().cuda()
    dy = torch.randn(T, N, generator=gen).bfloat16().cuda()
    dw = lm._weight_grad(dy, x)
    _close(dw, dy.float().t() @ x.float(), T)
    assert ("wgrad", N, K, T) in lm._GEMM_CHOICE
