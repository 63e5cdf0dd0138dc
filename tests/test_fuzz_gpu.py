"""T4: hypothesis shape fuzzing of the gfx950 kernels against
plain fp32 PyTorch references -- odd row counts, widths off the tuned sizes,
sequence lengths that are not tile multiples, GQA ratios, split-K splits that
do not divide K.  Few examples per kernel (each one is a GPU launch pair)."""
import pytest
import torch
import torch.nn.functional as F
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from distributed_training_amd.ops import lm

pytestmark = pytest.mark.gpu
DEV = "cuda"
FUZZ = settings(max_examples=12, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@FUZZ
@given(n=st.integers(1, 300), c8=st.integers(1, 512), rms=st.booleans())
def test_norm_shapes(n, c8, rms):
    C = 8 * c8
    g = torch.Generator(device=DEV).manual_seed(n * 1000 + C)
    x = (torch.randn(n, C, device=DEV, generator=g) * 2 + 0.5).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(C, device=DEV, generator=g)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(C, device=DEV, generator=g)).bfloat16().requires_grad_()
    dy = torch.randn(n, C, device=DEV, generator=g).bfloat16()
    y = lm.rms_norm(x, w) if rms else lm.layer_norm(x, w, b)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr if rms else F.layer_norm(xr, (C,), wr, br)
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2 and _rel(x.grad, xr.grad) < 3e-2 and _rel(w.grad, wr.grad) < 3e-2


@FUZZ
@given(s=st.integers(1, 700), heads=st.sampled_from([(4, 4), (4, 2), (8, 1), (6, 3)]), d=st.sampled_from([64, 128]),
       causal=st.booleans())
def test_attention_shapes(s, heads, d, causal):
    H, Hkv = heads
    g = torch.Generator(device=DEV).manual_seed(s * 31 + H + d)
    q = torch.randn(1, s, H, d, device=DEV, generator=g).bfloat16().requires_grad_()
    k = torch.randn(1, s, Hkv, d, device=DEV, generator=g).bfloat16().requires_grad_()
    v = torch.randn(1, s, Hkv, d, device=DEV, generator=g).bfloat16().requires_grad_()
    do = torch.randn(1, s, H, d, device=DEV, generator=g).bfloat16()
    o = lm.attention(q, k, v, causal=causal)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = lm.attention_reference(qr, kr, vr, causal=causal)
    orf.backward(do.float())
    assert _rel(o, orf) < 1.5e-2
    for got, want in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        # norm-relative, with a floor: at one key dQ = dK = 0 exactly, and the kernel's
        # P * (dP - delta) leaves bf16-rounding residue there (as every flash backward does)
        err = (got.float() - want).norm().item()
        assert err < 3e-2 * want.norm().item() + 1e-3 * want.numel() ** 0.5, (err, want.norm().item())


@FUZZ
@given(n=st.integers(1, 200), v=st.integers(2, 70000))
def test_cross_entropy_shapes(n, v):
    g = torch.Generator(device=DEV).manual_seed(n * 100003 + v)
    logits = (torch.randn(n, v, device=DEV, generator=g) * 2).bfloat16().requires_grad_()
    t = torch.randint(0, v, (n,), device=DEV, generator=g)
    loss = lm.cross_entropy(logits, t)
    loss.backward()
    lr = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(lr, t)
    ref.backward()
    torch.testing.assert_close(loss.float(), ref, rtol=3e-3, atol=3e-3)
    assert _rel(logits.grad, lr.grad) < 3e-2


# ---------------------------------------------------------------- GEMM fuzzing
# Every hand-written GEMM family against fp32 ``A.float() @ B.float()`` on random tile-multiple shapes:
# the 64-deep tiles 1-8 (four-phase 1-4, two-phase 5-8; ``| 128`` = per-fragment instead of LDS-staged
# epilogue), their stream-K forms (``| 64``), the 192-wide tiles 11 / 12 and the 4-wave W4 tile 9 (K tails,
# edge tiles), with the fused epilogues in the layouts the model uses them in: bias / GELU dual store /
# alpha + residual on the forward (NT) layout, x gelu'(h) on the input-gradient (NN) layout.
GEMM_FUZZ = settings(max_examples=50, deadline=None, derandomize=True,
                     suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
K64_TILES = {1: (256, 256), 2: (256, 128), 3: (128, 128), 4: (128, 256),
             5: (256, 256), 6: (256, 128), 7: (128, 128), 8: (128, 256)}
T192 = {11: (256, 192), 12: (128, 192)}
ALL_LAYOUTS = [(False, False), (False, True), (True, True), (True, False)]


def _gemm_close(got, want, K):
    tol = 4e-3 * want.abs().max().item() + 1e-3 * K ** 0.5
    err = (got.float() - want).abs().max().item()
    assert err <= tol, (err, tol)


def _gemm_check(M, N, K, a_t, b_t, tile, epi, seed, sk_cnt=None):
    """One GEMM of the family ``tile`` with epilogue ``epi`` ("none", "f32", "bias", "gelu", "res",
    "dgelu") against fp32 PyTorch on the same bf16 operands."""
    from distributed_training_amd.ops import native

    C = native()
    g = torch.Generator(device=DEV).manual_seed(seed)
    a = torch.randn(*((K, M) if a_t else (M, K)), device=DEV, generator=g).bfloat16()
    b = (0.5 * torch.randn(*((K, N) if b_t else (N, K)), device=DEV, generator=g)).bfloat16()
    ref = (a.float().t() if a_t else a.float()) @ (b.float() if b_t else b.float().t())
    kw = {"tile": tile, "sk_cnt": sk_cnt}
    if epi in ("none", "f32"):
        got, = C.gemm64(a, b, a_t, b_t, out_f32=epi == "f32", **kw)
        _gemm_close(got, ref, K)
    elif epi == "bias":
        bias = torch.randn(N, device=DEV, generator=g).bfloat16()
        got, = C.gemm64(a, b, a_t, b_t, bias=bias, **kw)
        _gemm_close(got, ref + bias.float(), K)
    elif epi == "gelu":  # dual store: pre-activation h and gelu(h) of the rounded h
        bias = torch.randn(N, device=DEV, generator=g).bfloat16()
        h, act = C.gemm64(a, b, a_t, b_t, bias=bias, epi=2,
                          out2=torch.empty(M, N, dtype=torch.bfloat16, device=DEV), **kw)
        _gemm_close(h, ref + bias.float(), K)
        torch.testing.assert_close(act.float(), F.gelu(h.float(), approximate="tanh"), rtol=1.6e-2, atol=1e-2)
    elif epi == "res":  # round(round(alpha A B^T) + res)
        res = torch.randn(M, N, device=DEV, generator=g).bfloat16()
        got, = C.gemm64(a, b, a_t, b_t, alpha=0.5, epi=32, res=res, **kw)
        _gemm_close(got, (0.5 * ref).bfloat16().float() + res.float(), K)
    elif epi == "dgelu":  # the input gradient through a GELU: (dy W) * gelu'(h)
        h = torch.randn(M, N, device=DEV, generator=g).bfloat16()
        got, = C.gemm64(a, b, a_t, b_t, epi=16, res=h, **kw)
        xr = h.float().requires_grad_(True)
        gg, = torch.autograd.grad(F.gelu(xr, approximate="tanh").sum(), xr)
        _gemm_close(got, ref * gg, K)
    else:
        raise AssertionError(epi)


def _epi_for(layout, draw_epi):
    if layout == (False, False):
        return draw_epi
    if layout == (False, True) and draw_epi in ("dgelu", "bias"):
        return "dgelu"
    return "f32" if draw_epi in ("gelu", "res") else "none"


@GEMM_FUZZ
@given(tile=st.sampled_from(sorted(K64_TILES)), mt=st.integers(1, 4), nt=st.integers(1, 4), kt=st.integers(1, 20),
       layout=st.sampled_from(ALL_LAYOUTS), epi=st.sampled_from(["none", "f32", "bias", "gelu", "res", "dgelu"]),
       per_fragment=st.booleans())
def test_gemm64_tiles_fuzz(tile, mt, nt, kt, layout, epi, per_fragment):
    bm, bn = K64_TILES[tile]
    e = _epi_for(layout, epi)
    t = tile | (128 if per_fragment and e != "f32" else 0)
    _gemm_check(mt * bm, nt * bn, 64 * kt, *layout, t, e, seed=tile * 7919 + mt * 131 + nt * 17 + kt)


@GEMM_FUZZ
@given(tile=st.sampled_from([5, 6, 7, 8, 11, 12]), mt=st.integers(1, 4), nt=st.integers(1, 4),
       kt=st.integers(1, 48), layout=st.sampled_from([(False, False), (False, True), (True, True)]),
       epi=st.sampled_from(["none", "f32", "bias", "res"]))
def test_gemm64_stream_k_fuzz(tile, mt, nt, kt, layout, epi):
    from distributed_training_amd.ops import lm, native

    if tile in T192:
        layout = (False, False)
    bm, bn = {**K64_TILES, **T192}[tile]
    M, N, K = mt * bm, nt * bn, 64 * kt
    tiles, _grid, _span = native().gemm64_sk_plan(M, N, K, tile | 64)
    assert tiles == mt * nt
    cnt = lm._sk_cnt(torch.device(DEV, torch.cuda.current_device()))
    _gemm_check(M, N, K, *layout, tile | 64, _epi_for(layout, epi), seed=tile * 104729 + mt * 31 + nt * 7 + kt,
                sk_cnt=cnt)
    torch.cuda.synchronize()
    assert int(cnt[:tiles].abs().sum().item()) == 0  # the arrival counters are left zero


@GEMM_FUZZ
@given(tile=st.sampled_from(sorted(T192)), mt=st.integers(1, 6), nt=st.integers(1, 6), kt=st.integers(1, 24),
       epi=st.sampled_from(["none", "f32", "bias", "gelu", "res"]), per_fragment=st.booleans())
def test_gemm64_192_fuzz(tile, mt, nt, kt, epi, per_fragment):
    bm, bn = T192[tile]
    t = tile | (128 if per_fragment and epi != "f32" else 0)
    _gemm_check(mt * bm, nt * bn, 64 * kt, False, False, t, epi, seed=tile * 6007 + mt * 37 + nt * 11 + kt)


@GEMM_FUZZ
@given(m8=st.integers(1, 96), n8=st.integers(1, 96), k8=st.integers(1, 96), layout=st.sampled_from(ALL_LAYOUTS),
       epi=st.sampled_from(["none", "f32", "bias", "gelu", "res"]))
def test_gemm_w4_fuzz(m8, n8, k8, layout, epi):
    """Tile 9 (csrc/gemm_w4.hip): any M, N, K multiples of 8 -- edge tiles and K tails."""
    e = _epi_for(layout, epi)
    if e == "dgelu":
        e = "none"
    _gemm_check(8 * m8, 8 * n8, 8 * k8, *layout, 9, e, seed=m8 * 9973 + n8 * 97 + k8)
