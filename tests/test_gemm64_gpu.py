"""The 64-deep-stage GEMM (csrc/gemm_k64.hip) against an fp32 PyTorch reference of
the same op on the same bf16 inputs: every operand layout (forward NT, input-gradient
NN, weight-gradient TN, and TT) x every tile, pipelines shorter than the DMA
look-ahead (K = 64, 128), exact small-integer checks that catch any fragment /
swizzle / transposition mistake, and the fused epilogues (bias, alpha, GELU with the
dual store of pre-activation and activation, x gelu'(h), + residual, fp32 out)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

LAYOUTS = [(False, False), (False, True), (True, True), (True, False)]
TILES = {1: (256, 256), 2: (256, 128), 3: (128, 128), 4: (128, 256)}
TILES.update({t + 4: TILES[t] for t in (1, 2, 3, 4)})  # 5-8: the two-phase K loop


def _ops(M, N, K, a_t, b_t, gen, scale=1.0):
    a = (torch.randn(K, M, generator=gen) if a_t else torch.randn(M, K, generator=gen)) * scale
    b = (torch.randn(K, N, generator=gen) if b_t else torch.randn(N, K, generator=gen)) * scale
    a, b = a.bfloat16().cuda(), b.bfloat16().cuda()
    A = a.float().t() if a_t else a.float()
    B = b.float() if b_t else b.float().t()
    return a, b, A @ B


def _close(got, want, K):
    tol = 4e-3 * want.abs().max().item() + 1e-3 * K ** 0.5
    err = (got.float() - want).abs().max().item()
    assert err <= tol, (err, tol)


@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6, 7, 8])
def test_gemm64_exact_small_integers(a_t, b_t, tile):
    """Small integers: every product and partial sum is exact in fp32 -- any fragment-order,
    swizzle or pipeline-staging mistake shows as a mismatch (asymmetric operands)."""
    from distributed_training_amd.ops import native

    bm, bn = TILES[tile]
    gen = torch.Generator().manual_seed(tile * 10 + 2 * a_t + b_t)
    for M, N, K in ((2 * bm, 3 * bn, 64), (bm, bn, 128), (3 * bm, 2 * bn, 640)):
        a = torch.randint(-3, 4, (K, M) if a_t else (M, K), generator=gen).float()
        b = torch.randint(-3, 4, (K, N) if b_t else (N, K), generator=gen).float()
        want = (a.t() if a_t else a) @ (b if b_t else b.t())
        got, = native().gemm64(a.bfloat16().cuda(), b.bfloat16().cuda(), a_t, b_t, out_f32=True, tile=tile)
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), want), (a_t, b_t, tile, M, N, K)


@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
@pytest.mark.parametrize("tile,M,N,K", [(1, 512, 512, 256), (2, 512, 384, 192), (3, 384, 256, 1088),
                                        (4, 256, 768, 768), (0, 1024, 768, 768), (5, 512, 512, 256),
                                        (7, 384, 256, 1088), (8, 256, 768, 768)])
def test_gemm64_random(a_t, b_t, tile, M, N, K):
    from distributed_training_amd.ops import native

    if tile and (M % TILES[tile][0] or N % TILES[tile][1]):
        pytest.skip("shape not a multiple of the tile")
    gen = torch.Generator().manual_seed(M + N + K + 7 * a_t + 3 * b_t)
    a, b, want = _ops(M, N, K, a_t, b_t, gen)
    got, = native().gemm64(a, b, a_t, b_t, tile=tile)
    torch.cuda.synchronize()
    _close(got, want, K)


@pytest.mark.parametrize("tile", [1, 3, 5, 7, 5 | 128])
def test_gemm64_epilogues(tile):
    from distributed_training_amd.ops import native

    gen = torch.Generator().manual_seed(5 + tile)
    M, N, K = 512, 768, 384
    xs = torch.randn(M, K + 64, generator=gen).bfloat16().cuda()[:, 16:16 + K]  # row stride K + 64
    w = (torch.randn(N, K, generator=gen) * 0.1).bfloat16().cuda()
    bias = torch.randn(N, generator=gen).bfloat16().cuda()
    res = torch.randn(M, N, generator=gen).bfloat16().cuda()
    ref = xs.float() @ w.float().t()
    # GELU in the epilogue (single output)
    got, = native().gemm64(xs, w, bias=bias, epi=2, tile=tile)
    _close(got, F.gelu(ref + bias.float(), approximate="tanh"), K)
    # GELU dual store: h (pre-activation, rounded once) and gelu(h) of the ROUNDED h -- what the
    # unfused gemm + gelu_fwd pair gives, so backward (dgelu of the stored h) is consistent
    h, act = native().gemm64(xs, w, bias=bias, epi=2, out2=torch.empty(M, N, dtype=torch.bfloat16, device="cuda"),
                             tile=tile)
    want_h = ref + bias.float()
    _close(h, want_h, K)
    torch.testing.assert_close(act.float(), F.gelu(h.float(), approximate="tanh"), rtol=1.6e-2, atol=1e-2)
    # alpha + residual: round(round(alpha x W^T) + res)
    got, = native().gemm64(xs, w, alpha=0.5, epi=32, res=res, tile=tile)
    _close(got, (0.5 * ref).bfloat16().float() + res.float(), K)
    # x gelu'(res): the input gradient through a GELU (dgrad NN layout: dy [M, K] @ W [K, N])
    wn = (torch.randn(K, N, generator=gen) * 0.1).bfloat16().cuda()
    dy = torch.randn(M, K, generator=gen).bfloat16().cuda()
    got, = native().gemm64(dy, wn, False, True, epi=16, res=res, tile=tile)
    xr = res.float().requires_grad_(True)
    gg, = torch.autograd.grad(F.gelu(xr, approximate="tanh").sum(), xr)
    _close(got, (dy.float() @ wn.float()) * gg, K)
    # fp32 output into a strided destination
    out = torch.zeros(M, N + 32, device="cuda")
    native().gemm64(xs, w, out=out[:, :N], out_f32=True, tile=tile)
    torch.cuda.synchronize()
    _close(out[:, :N], ref, K)
    assert out[:, N:].abs().max().item() == 0.0


def test_gemm64_rejects_bad_shapes():
    from distributed_training_amd.ops import native

    a = torch.zeros(256, 96, dtype=torch.bfloat16, device="cuda")  # K not a multiple of 64
    b = torch.zeros(256, 96, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(RuntimeError, match="not covered"):
        native().gemm64(a, b)
    assert native().gemm64_tile(8192, 768, 768) != 0 and native().gemm64_tile(100, 768, 768) == 0


@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
@pytest.mark.parametrize("tile", [1, 2, 3, 4])
def test_gemm64_persistent_multi_tile_exact(a_t, b_t, tile):
    """More tiles than resident workgroups (576 > 256 / 512 slots): each workgroup walks several
    tiles with the DMA pipeline running across tile boundaries and epilogues in between --
    exact on small integers, every tile checked (also the K = 64 single-step case)."""
    from distributed_training_amd.ops import native

    bm, bn = TILES[tile]
    gen = torch.Generator().manual_seed(100 + tile * 10 + 2 * a_t + b_t)
    for M, N, K in ((32 * bm, 18 * bn, 192), (32 * bm, 18 * bn, 64)):
        a = torch.randint(-3, 4, (K, M) if a_t else (M, K), generator=gen).float()
        b = torch.randint(-3, 4, (K, N) if b_t else (N, K), generator=gen).float()
        want = (a.t() if a_t else a).cuda() @ (b if b_t else b.t()).cuda()
        got, = native().gemm64(a.bfloat16().cuda(), b.bfloat16().cuda(), a_t, b_t, out_f32=True, tile=tile)
        torch.cuda.synchronize()
        assert torch.equal(got, want), (a_t, b_t, tile, M, N, K, (got - want).abs().max().item())


@pytest.mark.parametrize("a_t,b_t", LAYOUTS[:3])
@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6, 7, 8, 5 | 32, 7 | 32])
def test_gemm64_busy_chip(a_t, b_t, tile):
    """Llama-sized problems (1024-2048 workgroups, 64 K-steps, every CU busy), where DMA latency
    varies: a wait placed one barrier too late for the leading wave group of the staggered 8-wave
    loops read stale LDS here (rel. error 0.17 on the 256 x 128 two-phase tile before the fix) while
    every small-shape test passed (profiles/k64_twophase_race_fix.txt).  Random N(0,1) operands, three
    launches each, against an fp32 product of the same bf16 inputs.  Tile ids | 32: the flat
    global_load_lds DMA form (default: buffer descriptors)."""
    from distributed_training_amd.ops import native

    gen = torch.Generator(device="cuda").manual_seed(tile * 7 + 2 * a_t + b_t)
    M, N, K = 8192, 4096, 4096
    a = torch.randn((K, M) if a_t else (M, K), generator=gen, device="cuda").bfloat16()
    b = (torch.randn((K, N) if b_t else (N, K), generator=gen, device="cuda") * 0.02).bfloat16()
    want = (a.float().t() if a_t else a.float()) @ (b.float() if b_t else b.float().t())
    scale = want.abs().max().item()
    for _ in range(3):
        got, = native().gemm64(a, b, a_t, b_t, tile=tile)
        err = (got.float() - want).abs().max().item() / scale
        assert err < 8e-3, (tile, a_t, b_t, err)


@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 256), (304, 520, 384), (1000, 200, 1280),
                                   (8192, 50304 // 16, 768), (64, 1000, 128),
                                   # K tails (not a multiple of two 64-deep K-tiles): zero-filled DMA lanes
                                   (256, 512, 72), (304, 264, 520), (64, 64, 8), (512, 256, 1016)])
def test_gemm_w4_exact_and_edges(a_t, b_t, M, N, K):
    """Tile 9 (csrc/gemm_w4.hip: 4 waves, 256 x 256, intra-wave interleave) in every operand layout: exact
    on small integers at full tiles and at EDGE tiles in both dimensions (K-major rows / M-N-major chunks
    past M / N clamped in the DMA, stores predicated), and with K tails (any K multiple of 8: the DMA lanes
    past K read zeros through out-of-range buffer offsets)."""
    from distributed_training_amd.ops import native

    gen = torch.Generator().manual_seed(M * 7 + N + K + 2 * a_t + b_t)
    a = torch.randint(-3, 4, (K, M) if a_t else (M, K), generator=gen).float()
    b = torch.randint(-3, 4, (K, N) if b_t else (N, K), generator=gen).float()
    want = (a.t() if a_t else a) @ (b if b_t else b.t())
    out = torch.full((M, N), float("nan"), device="cuda")
    got, = native().gemm64(a.bfloat16().cuda(), b.bfloat16().cuda(), a_t, b_t, out, out_f32=True, tile=9)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), want), (a_t, b_t, M, N, K)


@pytest.mark.parametrize("tile", [9, 10])
@pytest.mark.parametrize("epi", [0, 2, 32])
def test_gemm_w4_epilogues(epi, tile):
    """Tile 9 with bias / alpha and the fused epilogues (GELU dual store, + residual) vs fp32 torch."""
    from distributed_training_amd.ops import native

    gen = torch.Generator().manual_seed(90 + epi)
    M, N, K = 520, 776, 512
    a = torch.randn(M, K, generator=gen).bfloat16().cuda()
    b = (torch.randn(N, K, generator=gen) * 0.05).bfloat16().cuda()
    bias = torch.randn(N, generator=gen).bfloat16().cuda()
    ref = a.float() @ b.float().t() + bias.float()
    if epi == 2:
        h, g = native().gemm64(a, b, False, False, torch.empty(M, N, device="cuda", dtype=torch.bfloat16),
                               torch.empty(M, N, device="cuda", dtype=torch.bfloat16), False, 1.0, bias, 2, None, tile)
        _close(h, ref, K)
        _close(g, F.gelu(h.float(), approximate="tanh"), K)
    elif epi == 32:
        res = torch.randn(M, N, generator=gen).bfloat16().cuda()
        y, = native().gemm64(a, b, False, False, None, None, False, 1.0, bias, 32, res, tile)
        _close(y, ref + res.float(), K)
    else:
        y, = native().gemm64(a, b, False, False, None, None, False, 0.5, bias, 0, None, tile)
        _close(y, 0.5 * (a.float() @ b.float().t()) + bias.float(), K)


@pytest.mark.parametrize("tile", [10])
@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
@pytest.mark.parametrize("M,N,K", [(512, 768, 256), (304, 520, 384), (8192, 50304 // 16, 768), (256, 512, 72),
                                   (8192, 8448, 192), (6400, 9000, 384)])
def test_gemm_w4_staged_epilogue_exact(a_t, b_t, M, N, K, tile):
    """Tile 10: the W4 kernel with the LDS-staged bf16 epilogue (whole 256-B row pieces per store), edges
    predicated (the big shapes: many rounds of tiles, edge tiles and K tails): exact against fp32 on small
    integers whose sums stay exactly representable in bf16."""
    from distributed_training_amd.ops import native

    gen = torch.Generator().manual_seed(M + 3 * N + K + 2 * a_t + b_t)
    a = torch.randint(-1, 2, (K, M) if a_t else (M, K), generator=gen).float()
    b = torch.randint(-1, 2, (K, N) if b_t else (N, K), generator=gen).float()
    want = ((a.t() if a_t else a) @ (b if b_t else b.t())).clamp(-256, 256)
    a = a * (torch.rand(a.shape, generator=gen) < 0.25)  # sparse: |sum| <= K / 4 ... clamp checks below
    want = (a.t() if a_t else a) @ (b if b_t else b.t())
    assert want.abs().max() <= 256
    out = torch.full((M, N), float("nan"), device="cuda").bfloat16()
    got, = native().gemm64(a.bfloat16().cuda(), b.bfloat16().cuda(), a_t, b_t, out, tile=tile)
    torch.cuda.synchronize()
    assert torch.equal(got.float().cpu(), want), (a_t, b_t, M, N, K)


@pytest.mark.parametrize("tile", [1, 3, 5, 6, 7, 8])
@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
def test_gemm64_staged_epilogue_exact(a_t, b_t, tile):
    """Every k64 tile with one bf16 output takes the LDS-staged epilogue (the whole tile image through the
    LDS, whole-row stores); tile | 128 forces the per-fragment form: both exact against fp32 on small
    integers whose sums stay exactly representable in bf16, on a grid of many tiles."""
    from distributed_training_amd.ops import native

    M, N, K = 1024, 1536, 512
    gen = torch.Generator().manual_seed(77 + 4 * tile + 2 * a_t + b_t)
    a = torch.randint(-1, 2, (K, M) if a_t else (M, K), generator=gen).float()
    b = torch.randint(-1, 2, (K, N) if b_t else (N, K), generator=gen).float()
    a = a * (torch.rand(a.shape, generator=gen) < 0.25)
    want = (a.t() if a_t else a) @ (b if b_t else b.t())
    assert want.abs().max() <= 256
    for t in (tile, tile | 128):
        out = torch.full((M, N), float("nan"), device="cuda").bfloat16()
        got, = native().gemm64(a.bfloat16().cuda(), b.bfloat16().cuda(), a_t, b_t, out, tile=t)
        torch.cuda.synchronize()
        assert torch.equal(got.float().cpu(), want), (t, a_t, b_t)


@pytest.mark.parametrize("tile", [1, 3, 5, 6, 7, 8])
def test_gemm64_staged_fused_epilogues_bitwise(tile):
    """The staged epilogue of the fused forms -- GELU dual store (two passes through the LDS image),
    x gelu'(res) and + res (the res tile staged with whole-row loads, replaced in place) -- bit-identical
    to the per-fragment epilogue (tile | 128), with bias and alpha; a res whose row stride is not a
    multiple of 8 takes the per-fragment path and still agrees."""
    from distributed_training_amd.ops import native

    C = native()
    gen = torch.Generator().manual_seed(31 + tile)
    M, N, K = 1024, 1536, 384
    x = torch.randn(M, K, generator=gen).bfloat16().cuda()
    w = (torch.randn(N, K, generator=gen) * 0.1).bfloat16().cuda()
    wn = (torch.randn(K, N, generator=gen) * 0.1).bfloat16().cuda()
    bias = torch.randn(N, generator=gen).bfloat16().cuda()
    res = torch.randn(M, N, generator=gen).bfloat16().cuda()
    res_odd = torch.randn(M, N + 4, generator=gen).bfloat16().cuda()[:, :N]  # row stride N + 4

    def both(fn):
        a, b = fn(tile), fn(tile | 128)
        torch.cuda.synchronize()
        for u, v in zip(a, b):
            assert torch.equal(u, v), tile
        return a

    h, act = both(lambda t: C.gemm64(x, w, bias=bias, epi=2, out2=torch.empty(M, N, dtype=torch.bfloat16, device="cuda"),
                                     tile=t))
    torch.testing.assert_close(act.float(), F.gelu(h.float(), approximate="tanh"), rtol=1.6e-2, atol=1e-2)
    both(lambda t: C.gemm64(x, w, alpha=0.5, bias=bias, epi=32, res=res, tile=t))
    both(lambda t: C.gemm64(x, w, epi=32, res=res_odd, tile=t))
    both(lambda t: C.gemm64(x, wn, False, True, epi=16, res=res, tile=t))
    both(lambda t: C.gemm64(x, wn, False, True, bias=bias, epi=16, res=res_odd, tile=t))


@pytest.mark.parametrize("tile,M,N,K", [(5, 512, 512, 256), (6, 512, 384, 192), (7, 384, 256, 1088), (8, 256, 512, 64),
                                        (5, 2048, 2048, 1024), (7, 1024, 1536, 512)])
def test_gemm64_swiglu_backward_epilogue(tile, M, N, K):
    """EPI_DSWIGLU (64): the product g = dy W (N-major W, the down projection's input gradient) turned
    into [da | db] of silu(a) * b in the LDS-staged epilogue, against fp32 PyTorch on the same bf16
    inputs; and the other tiles / the W4 tile / a bias are refused."""
    from distributed_training_amd.ops import native

    C = native()
    gen = torch.Generator().manual_seed(tile * 7 + K)
    dy = (0.5 * torch.randn(M, K, generator=gen)).bfloat16().cuda()
    w = (0.05 * torch.randn(K, N, generator=gen)).bfloat16().cuda()
    ab = (2.0 * torch.randn(M, 2 * N, generator=gen)).bfloat16().cuda()
    got = C.gemm64(dy, w, False, True, None, None, False, 1.0, None, 64, ab, tile)[0]
    assert got.shape == (M, 2 * N)
    g = dy.float() @ w.float()
    a, b = ab.float()[:, :N], ab.float()[:, N:]
    s = torch.sigmoid(a)
    want = torch.cat([g * b * s * (1 + a * (1 - s)), g * a * s], dim=1)
    err = (got.float() - want).abs().max().item()
    assert err <= 1e-2 * want.abs().max().item(), err
    for bad in (1, 3, 10):  # four-phase / W4: not instantiated with this epilogue
        if C.gemm64_tile(M, N, K, bad):
            with pytest.raises(RuntimeError):
                C.gemm64(dy, w, False, True, None, None, False, 1.0, None, 64, ab, bad)
    with pytest.raises(RuntimeError):
        C.gemm64(dy, w, False, True, None, None, False, 1.0, torch.zeros(N, dtype=torch.bfloat16, device="cuda"),
                 64, ab, tile)


# ---- the 192-wide tiles (11 = 256 x 192, 8 waves in a 4 x 2 grid with the B halves staged as one image;
# 12 = 128 x 192, 4 waves): K-major A and B only (the forward layout)
TILES_192 = {11: (256, 192), 12: (128, 192)}


@pytest.mark.parametrize("tile", [11, 12])
def test_gemm64_192_exact_small_integers(tile):
    """Exact small-integer products through both epilogues (fp32 per-fragment, bf16 staged with its CPR = 24
    chunk map, and the staged form forced off), pipelines shorter than the DMA look-ahead and many tiles."""
    from distributed_training_amd.ops import native

    bm, bn = TILES_192[tile]
    gen = torch.Generator().manual_seed(tile)
    for M, N, K in ((2 * bm, 3 * bn, 64), (bm, bn, 128), (3 * bm, 2 * bn, 640), (8 * bm, 4 * bn, 192)):
        a = torch.randint(-3, 4, (M, K), generator=gen).float()
        b = torch.randint(-3, 4, (N, K), generator=gen).float()
        want = a @ b.t()
        got, = native().gemm64(a.bfloat16().cuda(), b.bfloat16().cuda(), out_f32=True, tile=tile)
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), want), (tile, M, N, K)
        a01 = a.clamp(-1, 1) * (torch.rand(a.shape, generator=gen) < 0.25)
        want = a01 @ b.clamp(-1, 1).t()
        for t in (tile, tile | 128):
            got, = native().gemm64(a01.bfloat16().cuda(), b.clamp(-1, 1).bfloat16().cuda(), tile=t)
            torch.cuda.synchronize()
            assert torch.equal(got.float().cpu(), want), (t, M, N, K)


@pytest.mark.parametrize("tile", [11, 12])
def test_gemm64_192_epilogues_and_layouts(tile):
    """Bias, GELU dual store, + residual, alpha: staged bit-identical to per-fragment and close to fp32;
    the transposed layouts are refused loudly (no silent fallback)."""
    from distributed_training_amd.ops import native

    C = native()
    gen = torch.Generator().manual_seed(40 + tile)
    M, N, K = 1024, 2304, 384
    x = torch.randn(M, K, generator=gen).bfloat16().cuda()
    w = (torch.randn(N, K, generator=gen) * 0.1).bfloat16().cuda()
    bias = torch.randn(N, generator=gen).bfloat16().cuda()
    res = torch.randn(M, N, generator=gen).bfloat16().cuda()
    ref = x.float() @ w.float().t()
    outs = []
    for t in (tile, tile | 128):
        h, act = C.gemm64(x, w, bias=bias, epi=2, out2=torch.empty(M, N, dtype=torch.bfloat16, device="cuda"), tile=t)
        r, = C.gemm64(x, w, alpha=0.5, bias=bias, epi=32, res=res, tile=t)
        outs.append((h, act, r))
    torch.cuda.synchronize()
    for u, v in zip(*outs):
        assert torch.equal(u, v), tile
    h, act, r = outs[0]
    _close(h, ref + bias.float(), K)
    torch.testing.assert_close(act.float(), F.gelu(h.float(), approximate="tanh"), rtol=1.6e-2, atol=1e-2)
    _close(r, 0.5 * ref + bias.float() + res.float(), K)
    for a_t, b_t in ((False, True), (True, False), (True, True)):
        a = x.t().contiguous() if a_t else x
        b = w.t().contiguous() if b_t else w
        with pytest.raises(RuntimeError):
            C.gemm64(a, b, a_t, b_t, tile=tile)
            torch.cuda.synchronize()


@pytest.mark.parametrize("tile", [11, 12, 11 | 128])
@pytest.mark.parametrize("M,N,K", [(8192, 2304, 768), (8192, 3072, 768), (8192, 768, 3072)])
def test_gemm64_192_busy_chip(tile, M, N, K):
    """GPT-2-shaped problems at full occupancy (the staggered 8-wave loop's waits under real DMA latency;
    the 4-wave tile at two workgroups per CU): random operands, three launches, against fp32."""
    from distributed_training_amd.ops import native

    gen = torch.Generator(device="cuda").manual_seed(tile + M + N + K)
    a = torch.randn(M, K, generator=gen, device="cuda").bfloat16()
    b = (torch.randn(N, K, generator=gen, device="cuda") * 0.02).bfloat16()
    want = a.float() @ b.float().t()
    scale = want.abs().max().item()
    for _ in range(3):
        got, = native().gemm64(a, b, tile=tile)
        err = (got.float() - want).abs().max().item() / scale
        assert err < 8e-3, (tile, err)


# ---- stream-K forms (tile id | 64): equal runs of (tile, K-tile) units per workgroup; a cut tile is summed
# by its last-arriving contributor in K order (deterministic), counters left zero
SK = 64
SK_TILES = {5: (256, 256), 6: (256, 128), 7: (128, 128), 8: (128, 256), 11: (256, 192), 12: (128, 192)}
SK_LAYOUTS = [(False, False), (False, True), (True, True)]


def _sk_cnt():
    from distributed_training_amd.ops import lm

    return lm._sk_cnt(torch.device("cuda", torch.cuda.current_device()))


# (the 192-wide tiles 11 / 12 take K-major operands only)
@pytest.mark.parametrize("a_t,b_t,tile", [(a, b, t) for a, b in SK_LAYOUTS for t in (5, 6, 7, 8, 11, 12)
                                          if t < 11 or not (a or b)])
def test_gemm64_stream_k_exact(a_t, b_t, tile):
    """Small integers (exact in fp32 whatever the summation order) through the stream-K form at tile counts and
    K depths that cut tiles into two and three parts (span = ceil(nk / 2) when the tiles are few), fp32 and
    staged bf16 outputs; the arrival counters are zero afterwards."""
    from distributed_training_amd.ops import native

    C = native()
    bm, bn = SK_TILES[tile]
    cnt = _sk_cnt()
    gen = torch.Generator().manual_seed(100 + tile + 2 * a_t + b_t)
    for M, N, K in ((3 * bm, 5 * bn, 448), (bm, 2 * bn, 64 * 9), (2 * bm, 3 * bn, 64 * 48), (bm, bn, 64)):
        tiles, grid, span = C.gemm64_sk_plan(M, N, K, tile | SK)
        assert tiles == (M // bm) * (N // bn) and span >= (K // 64 + 1) // 2
        a = torch.randint(-3, 4, (K, M) if a_t else (M, K), generator=gen).float()
        b = torch.randint(-3, 4, (K, N) if b_t else (N, K), generator=gen).float()
        want = (a.t() if a_t else a) @ (b if b_t else b.t())
        got, = C.gemm64(a.bfloat16().cuda(), b.bfloat16().cuda(), a_t, b_t, out_f32=True, tile=tile | SK, sk_cnt=cnt)
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), want), (tile, a_t, b_t, M, N, K)
        a01 = a.clamp(-1, 1) * (torch.rand(a.shape, generator=gen) < 0.25)
        want = (a01.t() if a_t else a01) @ (b.clamp(-1, 1) if b_t else b.clamp(-1, 1).t())
        for t in (tile | SK, tile | SK | 128):
            got, = C.gemm64(a01.bfloat16().cuda(), b.clamp(-1, 1).bfloat16().cuda(), a_t, b_t, tile=t, sk_cnt=cnt)
            torch.cuda.synchronize()
            assert torch.equal(got.float().cpu(), want), (t, a_t, b_t, M, N, K)
    assert int(cnt.abs().sum().item()) == 0


@pytest.mark.parametrize("tile", [6, 7, 12])
def test_gemm64_stream_k_epilogues_deterministic(tile):
    """The fused epilogues through the stream-K form (bias, GELU dual store, + residual; x gelu'(res) in the
    input-gradient layout) match the plain tile's to bf16 rounding and repeat bit-identically."""
    from distributed_training_amd.ops import native

    C = native()
    cnt = _sk_cnt()
    gen = torch.Generator().manual_seed(60 + tile)
    M, N, K = 1024, 768 if tile != 12 else 1536, 64 * 30
    x = torch.randn(M, K, generator=gen).bfloat16().cuda()
    w = (torch.randn(N, K, generator=gen) * 0.05).bfloat16().cuda()
    wn = (torch.randn(K, N, generator=gen) * 0.05).bfloat16().cuda()
    bias = torch.randn(N, generator=gen).bfloat16().cuda()
    res = torch.randn(M, N, generator=gen).bfloat16().cuda()

    def run(t):
        h, act = C.gemm64(x, w, bias=bias, epi=2, out2=torch.empty(M, N, dtype=torch.bfloat16, device="cuda"),
                          tile=t, sk_cnt=cnt)
        r, = C.gemm64(x, w, alpha=0.5, bias=bias, epi=32, res=res, tile=t, sk_cnt=cnt)
        outs = [h, act, r]
        if tile != 12:
            d, = C.gemm64(x, wn, False, True, epi=16, res=res, tile=t, sk_cnt=cnt)
            outs.append(d)
        return outs

    plain, sk1, sk2 = run(tile), run(tile | SK), run(tile | SK)
    torch.cuda.synchronize()
    for u, v in zip(sk1, sk2):
        assert torch.equal(u, v), tile
    for u, v in zip(sk1, plain):
        torch.testing.assert_close(u.float(), v.float(), rtol=2e-2, atol=2e-2)
    assert int(cnt.abs().sum().item()) == 0


@pytest.mark.parametrize("tile,a_t,b_t,M,N,K", [
    (6, False, True, 8192, 768, 3072),     # GPT-2 input gradients (192 tiles of 256 x 128)
    (7, False, True, 8192, 768, 2304),
    (12, False, False, 8192, 768, 3072),   # GPT-2 fc2 forward
    (5, True, True, 6144, 4096, 8192),     # Llama qkv weight gradient (384 tiles of 256 x 256)
    (6, False, False, 8192, 768, 768),
])
def test_gemm64_stream_k_busy_chip(tile, a_t, b_t, M, N, K):
    """Full-chip stream-K launches at the shapes it is for, random operands against fp32, three launches
    bit-identical (the cut tiles' parts are summed in K order whoever arrives last)."""
    from distributed_training_amd.ops import native

    C = native()
    cnt = _sk_cnt()
    gen = torch.Generator(device="cuda").manual_seed(tile + M + N + K)
    a = torch.randn((K, M) if a_t else (M, K), generator=gen, device="cuda").bfloat16()
    b = (torch.randn((K, N) if b_t else (N, K), generator=gen, device="cuda") * 0.02).bfloat16()
    want = (a.float().t() if a_t else a.float()) @ (b.float() if b_t else b.float().t())
    scale = want.abs().max().item()
    first = None
    for _ in range(3):
        got, = C.gemm64(a, b, a_t, b_t, tile=tile | SK, sk_cnt=cnt)
        err = (got.float() - want).abs().max().item() / scale
        assert err < 8e-3, (tile, err)
        if first is None:
            first = got.clone()
        else:
            assert torch.equal(got, first), tile
    assert int(cnt.abs().sum().item()) == 0
