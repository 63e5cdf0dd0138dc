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
