"""Autograd ops for the transformer models, backed by the gfx950 kernels of
``csrc/attention.hip`` and ``csrc/lm_ops.hip``.

GPU tensors always take the HIP kernels (bf16 activations required -- the
models run under bf16 mixed precision on GPU; anything else raises).  CPU
tensors use the equivalent PyTorch math, which is also the numerics reference
of the GPU tests.

Projection GEMMs (forward x W^T + b, input gradient dy W, weight gradient
dy^T x, the LM head) go through :func:`gemm`: the gfx950 GEMMs of
``csrc/gemm_k64.hip`` / ``csrc/gemm_w4.hip`` (bias / scale / GELU / residual fused
in their epilogues) or hipBLASLt, per shape (see :func:`_pick`: a tracked per-shape table
measured on MI355X, in-run timing only for shapes it lacks; ``DTA_GEMM=dta`` / ``torch`` force
one).  Single-use weight gradients are deferred and computed in grouped launches of the 64-deep
kernel (``gemm_k64_group_kernel``, bias gradients from the same MFMA pipe).
"""
from __future__ import annotations

import math
import os
from typing import Any, Callable, Dict, Optional, Tuple, Union

import torch
import torch.nn.functional as F
from torch.autograd import Function

from . import native


def _need_bf16(*ts: Any) -> None:
    for t in ts:
        if t.dtype != torch.bfloat16:
            raise TypeError(f"GPU transformer ops need bf16 tensors (got {t.dtype}); "
                            "train the LM configs with mixed_precision=bf16")


# ------------------------------------------------------------------ attention
def attention_reference(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
                        scale: Optional[float] = None) -> torch.Tensor:
    """[B, S, H, D] / [B, S, Hkv, D] -> [B, S, H, D], fp32 math."""
    B, S, H, D = q.shape
    Hkv = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    if Hkv != H:
        kf = kf.repeat_interleave(H // Hkv, dim=1)
        vf = vf.repeat_interleave(H // Hkv, dim=1)
    s = (qf @ kf.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    return (p @ vf).transpose(1, 2).to(q.dtype)


class _FlashAttn(Function):
    @staticmethod
    def forward(ctx: Any, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool, scale: float) -> torch.Tensor:
        o, lse = native().attn_fwd(q, k, v, bool(causal), float(scale), -1)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx: Any, do: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        q, k, v, o, lse = ctx.saved_tensors
        do = do.contiguous()
        dq, dk, dv = native().attn_bwd(do, q, k, v, o, lse, bool(ctx.causal), float(ctx.scale), -1)
        return dq, dk, dv, None, None


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
              scale: Optional[float] = None) -> torch.Tensor:
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if q.is_cuda:
        _need_bf16(q, k, v)
        return _FlashAttn.apply(q, k, v, causal, scale)
    return attention_reference(q, k, v, causal, scale)


def _split_qkv(qkv: torch.Tensor, H: int, Hkv: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    B, S, W = qkv.shape
    D = W // (H + 2 * Hkv)
    t = qkv.view(B, S, H + 2 * Hkv, D)
    return t[:, :, :H], t[:, :, H:H + Hkv], t[:, :, H + Hkv:]


class _PackedAttn(Function):
    """Attention straight on the fused QKV projection output [B, S, (H+2Hkv)*D]:
    q/k/v are strided views (no copies), optional RoPE is applied in place to
    the q|k columns of one rotated copy (or of ``qkv`` itself with ``inplace``: the
    caller owns the projection output and nothing else reads it -- the Linear
    backward saves its input, not its output -- saving a 96 MB copy per Llama
    layer), and backward writes dq/dk/dv into ONE
    packed gradient buffer -- autograd never has to zero-fill and add three
    slice gradients into the projection output's gradient."""

    @staticmethod
    def forward(ctx: Any, qkv: torch.Tensor, H: int, Hkv: int, causal: bool, scale: float, cos: torch.Tensor,
                sin: torch.Tensor, inplace: bool = False) -> torch.Tensor:
        B, S, W = qkv.shape
        D = W // (H + 2 * Hkv)
        if cos is not None:
            if not inplace:
                qkv = qkv.clone()
            native().rope_(qkv.view(B, S, H + 2 * Hkv, D)[:, :, :H + Hkv], cos, sin, False, -1)
        q, k, v = _split_qkv(qkv, H, Hkv)
        o, lse = native().attn_fwd(q, k, v, bool(causal), float(scale), -1)
        ctx.save_for_backward(qkv, o, lse, cos, sin)
        ctx.cfg = (H, Hkv, bool(causal), float(scale), cos is not None)
        return o

    @staticmethod
    def backward(ctx: Any, do: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        qkv, o, lse, cos, sin = ctx.saved_tensors
        H, Hkv, causal, scale, has_rope = ctx.cfg
        B, S, W = qkv.shape
        D = W // (H + 2 * Hkv)
        dqkv = torch.empty_like(qkv)
        q, k, v = _split_qkv(qkv, H, Hkv)
        dq, dk, dv = _split_qkv(dqkv, H, Hkv)
        # d(rope(x))/dx = the inverse rotation: applied to dQ / dK in the backward kernels' epilogues (in
        # fp32, before the rounding; no separate pass over the q|k columns)
        native().attn_bwd(do.contiguous(), q, k, v, o, lse, causal, scale, -1, dq, dk, dv,
                          cos if has_rope else None, sin if has_rope else None)
        return dqkv, None, None, None, None, None, None, None


def attention_packed(qkv: torch.Tensor, n_head: int, n_kv_head: int, causal: bool = True, scale: Optional[float] = None,
                     rope: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, rope_inplace: bool = False) -> torch.Tensor:
    """``qkv`` [B, S, (H + 2 Hkv) D] -> attention output [B, S, H, D] (RoPE on q, k if given).
    ``rope_inplace``: rotate the q|k columns of ``qkv`` itself on GPU (the caller's projection output,
    read by nothing else) instead of a rotated copy."""
    B, S, W = qkv.shape
    D = W // (n_head + 2 * n_kv_head)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    cos, sin = rope if rope is not None else (None, None)
    if cos is not None and cos.dtype != torch.float32:  # e.g. after module.bfloat16(): tables stay fp32 in the kernel
        cos, sin = cos.float(), sin.float()
    if qkv.is_cuda:
        _need_bf16(qkv)
        return _PackedAttn.apply(qkv, n_head, n_kv_head, causal, scale, cos, sin, bool(rope_inplace))
    q, k, v = _split_qkv(qkv, n_head, n_kv_head)
    if rope is not None:
        q, k = rope_reference(q, cos, sin), rope_reference(k, cos, sin)
    return attention_reference(q, k, v, causal, scale)


# ------------------------------------------------------------------ norms
# gamma / beta gradients of the norms, deferred like the weight gradients (see _DEFER): the norm-backward
# kernel leaves its per-workgroup partials and the column sums of every queued norm are finished by ONE
# launch at the next flush (csrc/lm_ops.hip colsum_batch_kernel) instead of one ~5 us launch per norm
# (25 per GPT-2 step).  Entries: (fp32 partials [nblk, C], an alias of the flat-gradient slice [C]).
_NORM_DEFER: list = []


def _defer_ok(p: Optional[torch.Tensor]) -> bool:
    gd = getattr(p, "_dta_gdest", None) if p is not None else None
    return gd is None or bool(getattr(gd, "defer_ok", False))


def _norm_backward(dy2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor,
                   rms: bool, dres: Optional[torch.Tensor], pw: torch.Tensor, pb: Optional[torch.Tensor],
                   need_w: bool, need_b: bool) -> Tuple[torch.Tensor, Optional[torch.Tensor], Optional[torch.Tensor]]:
    """dx and the gamma / beta gradients (into their flat-gradient slices when allowed); with both slices
    available and deferral on, the gamma / beta column sums are queued for the batched flush."""
    cw = _grad_dest(pw) if need_w else None
    cb = _grad_dest(pb) if (not rms and need_b) else None
    # deferred only for a gamma (beta) used ONCE in this backward: a second use would get no
    # slice (_grad_dest) and autograd would sum the returned slice before the batched flush wrote it
    if (_group_threshold() and os.environ.get("DTA_NORM_DEFER", "1") != "0" and cw is not None
            and (rms or not need_b or cb is not None) and _defer_ok(pw) and _single_use(pw)
            and (rms or not need_b or _single_use(pb))
            and (rms or _defer_ok(pb)) and cw.is_contiguous() and (cb is None or cb.is_contiguous())):
        dx, dwp, dbp = native().norm_bwd(dy2, x2, w, mean, rstd, rms, -1, dres, None, None, True)
        _NORM_DEFER.append((dwp, cw.view(-1)))  # (aliases, never the tensors returned to autograd)
        GEMM_STATS["deferred_norm"] += 1
        if cb is not None:
            _NORM_DEFER.append((dbp, cb.view(-1)))
        _queue_end_join()
        return dx, cw, cb
    return tuple(native().norm_bwd(dy2, x2, w, mean, rstd, rms, -1, dres, cw, cb))


def _count_norm_uses(ctx: Any, w: torch.Tensor, b: Optional[torch.Tensor], iw: int) -> None:
    """A norm's gamma / beta count as weight uses (``_single_use``) like a Linear's weight."""
    if ctx.needs_input_grad[iw]:
        _count_use(w)
    if b is not None and ctx.needs_input_grad[iw + 1]:
        _count_use(b)


class _Norm(Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, rms: bool, eps: float) -> torch.Tensor:
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, mean, rstd, _ = native().norm_fwd(x2, w.contiguous(), None if rms else b.contiguous(), rms, eps, -1)
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.rms, ctx.shape = rms, shape
        ctx.params = (w, b)  # their .grad decides a direct write into the flat gradient (_grad_dest)
        _count_norm_uses(ctx, w, b, 1)
        return y.view(shape)

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        x2, w, mean, rstd = ctx.saved_tensors
        pw, pb = ctx.params
        dx, dw, db = _norm_backward(dy.reshape(x2.shape).contiguous(), x2, w.contiguous(), mean, rstd, ctx.rms, None,
                                    pw, pb, ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        return dx.view(ctx.shape), (dw if ctx.needs_input_grad[1] else None), (None if ctx.rms else db), None, None


class _AddNorm(Function):
    """(x_new, y) = (x + res, norm(x + res)) in one pass; backward adds the
    residual-stream gradient of x_new inside the norm-backward kernel."""

    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, b: torch.Tensor, rms: bool,
                eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, mean, rstd, xsum = native().norm_fwd(x2, w.contiguous(), None if rms else b.contiguous(), rms, eps, -1,
                                                res.reshape(x2.shape).contiguous())
        ctx.save_for_backward(xsum, w, mean, rstd)
        ctx.rms, ctx.shape = rms, shape
        ctx.params = (w, b)
        _count_norm_uses(ctx, w, b, 2)
        # an unused output (the final norm's residual stream) gets no zero-filled gradient: no
        # [tokens, C] fill and no zero residual read by the norm-backward kernel
        ctx.set_materialize_grads(False)
        return xsum.view(shape), y.view(shape)

    @staticmethod
    def backward(ctx: Any, g_x: Optional[torch.Tensor], g_y: Optional[torch.Tensor]) -> Tuple[Optional[torch.Tensor], ...]:
        xsum, w, mean, rstd = ctx.saved_tensors
        if g_y is None:
            return g_x, g_x, None, None, None, None
        pw, pb = ctx.params
        dres = None if g_x is None else g_x.reshape(xsum.shape).contiguous()
        dx, dw, db = _norm_backward(g_y.reshape(xsum.shape).contiguous(), xsum, w.contiguous(), mean, rstd, ctx.rms,
                                    dres, pw, pb, ctx.needs_input_grad[2], ctx.needs_input_grad[3])
        dx = dx.view(ctx.shape)
        return dx, dx, (dw if ctx.needs_input_grad[2] else None), (None if ctx.rms else db), None, None


def add_layer_norm(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float = 1e-5) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns ``(x + res, layer_norm(x + res))``."""
    if x.is_cuda:
        _need_bf16(x, res, w, b)
        return _AddNorm.apply(x, res, w, b, False, eps)
    xn = x + res
    return xn, F.layer_norm(xn, (xn.shape[-1],), w, b, eps)


def add_rms_norm(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns ``(x + res, rms_norm(x + res))``."""
    if x.is_cuda:
        _need_bf16(x, res, w)
        return _AddNorm.apply(x, res, w, None, True, eps)
    xn = x + res
    return xn, rms_norm(xn, w, eps)


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    if x.is_cuda:
        _need_bf16(x, w, b)
        return _Norm.apply(x, w, b, False, eps)
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    if x.is_cuda:
        _need_bf16(x, w)
        return _Norm.apply(x, w, None, True, eps)
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype) * w


# ------------------------------------------------------------------ GEMM dispatch
_GEMM_CHOICE: Dict[tuple, int] = {}  # (kind, M, N, K) -> dta tile id (1..3) or 0 = hipBLASLt
GEMM_STATS: Dict[str, int] = {"dta": 0, "torch": 0, "deferred_wgrad": 0, "group_launches": 0, "deferred_norm": 0}


def _time_us(fns: Dict[int, Callable[[], object]], rounds: int = 5, reps: int = 4) -> Dict[int, float]:
    """Median per-call time of each candidate, rounds interleaved (clock / cache state
    shared fairly; the first call of each -- code object load, library heuristics -- untimed)."""
    for fn in fns.values():
        fn()
        fn()
    res: Dict[int, list] = {k: [] for k in fns}
    for _ in range(rounds):
        for k, fn in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                fn()
            e.record()
            e.synchronize()
            res[k].append(s.elapsed_time(e) * 1e3 / reps)
    return {k: sorted(v)[len(v) // 2] for k, v in res.items()}


_CACHE_LOADED = [False]


def _cache_path() -> Optional[str]:
    return os.environ.get("DTA_GEMM_CACHE") or None


def _load_cache() -> None:
    """``DTA_GEMM_CACHE=file.json``: per-shape choices of an earlier run (keys ``kind MxNxK``),
    used before the tracked table -- an explicit override for experiments."""
    _CACHE_LOADED[0] = True
    path = _cache_path()
    if not path or not os.path.exists(path):
        return
    import json

    try:
        with open(path) as f:
            for k, v in json.load(f).items():
                kind, dims = k.rsplit(" ", 1)
                M, N, K = (int(x) for x in dims.split("x"))
                _GEMM_CHOICE.setdefault((kind, M, N, K), int(v))
    except (OSError, ValueError):
        pass


def _save_cache() -> None:
    path = _cache_path()
    if not path:
        return
    import json

    tmp = f"{path}.tmp{os.getpid()}"
    try:
        with open(tmp, "w") as f:
            json.dump({f"{k[0]} {k[1]}x{k[2]}x{k[3]}": v for k, v in sorted(_GEMM_CHOICE.items())}, f, indent=0)
        os.replace(tmp, path)
    except OSError:
        pass


# ---- the tracked per-shape table (verdict r4: picks must not depend on a first-use timing inside a running
# step -- two boxes must pick the same kernel).  ops/gemm_table_mi355x.json is measured by
# scripts/gemm_table.py on an idle MI355X: every candidate of every GPT-2 / Llama-3 8B GEMM shape and kind,
# interleaved rounds on random operands, the fastest median kept.  A shape in the table takes its pick with no
# timing at all; a shape missing from it is timed in-run (more rounds than before) and logged.
# DTA_GEMM_TABLE=0 ignores the table; DTA_GEMM_VERIFY=1 also times table shapes in-run and warns when the
# table's pick measures more than 3 % slower than the best candidate there.
TABLE_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_table_mi355x.json")
_TABLE: Dict[tuple, int] = {}
_TABLE_LOADED = [False]
GEMM_PICK_SOURCE: Dict[tuple, str] = {}  # key -> "table" | "timed" | "forced" | "cache"
GEMM_TIMES: Dict[tuple, Dict[int, float]] = {}  # key -> median us per candidate (timed / verified keys)


def _gfx950() -> bool:
    try:
        return "gfx950" in torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
    except Exception:  # noqa: BLE001 - no device / no attribute: no table
        return False


# ---- the library GEMMs' own solution choice: PyTorch TunableOp results measured on MI355X
# (ops/tunableop_mi355x.csv; hipBLASLt / rocBLAS solutions searched per shape: profiles/tunableop_ab_r5v.jsonl) for the GEMMs the
# table leaves on the library -- GPT-2's c_fc forward, LM-head forward and input gradient take solutions other
# than the heuristic's: step 10.30 / 10.29 -> 10.17 / 10.22 ms same box (profiles/tunableop_ab_r5v.jsonl).  Read
# only (tuning off, nothing written); a file whose validators (torch / HIP / hipBLASLt / rocBLAS versions, arch)
# do not match this install is ignored by torch.  DTA_TUNABLEOP=0, or PYTORCH_TUNABLEOP_* set by the user: left
# alone.
TUNABLEOP_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_mi355x.csv")
_TUNABLEOP_SET = [False]


def _library_tuning() -> None:
    if _TUNABLEOP_SET[0]:
        return
    _TUNABLEOP_SET[0] = True
    if (os.environ.get("DTA_TUNABLEOP", "1") == "0" or any(k.startswith("PYTORCH_TUNABLEOP") for k in os.environ)
            or not os.path.exists(TUNABLEOP_PATH) or not torch.cuda.is_available()):
        return
    import torch.cuda.tunable as tunable

    tunable.set_filename(TUNABLEOP_PATH, False)
    tunable.tuning_enable(False)
    tunable.enable(True)


def gemm_table() -> Dict[tuple, int]:
    """The tracked table as {(kind, M, N, K): impl id} ({} off gfx950 or with DTA_GEMM_TABLE=0).  An entry's
    ``in_step_pick`` (with its ``in_step_evidence``: same-box step A/B runs) overrides the isolated-timing
    ``pick`` where the two disagree -- a kernel timed back to back on warm operands can rank differently
    inside the training step (cold operands, the step's clock)."""
    if not _TABLE_LOADED[0]:
        _TABLE_LOADED[0] = True
        if os.environ.get("DTA_GEMM_TABLE", "1") != "0" and os.path.exists(TABLE_PATH) and _gfx950():
            import json

            _library_tuning()
            with open(TABLE_PATH) as f:
                for k, v in json.load(f)["entries"].items():
                    kind, dims = k.rsplit(" ", 1)
                    M, N, K = (int(x) for x in dims.split("x"))
                    _TABLE[(kind, M, N, K)] = int(v.get("in_step_pick", v["pick"]))
    return _TABLE


def _rounds() -> int:
    v = os.environ.get("DTA_GEMM_ROUNDS", "").strip()
    return max(3, int(v)) if v else 9

# implementation ids in _GEMM_CHOICE: 0 = hipBLASLt (torch), 10 + t = csrc/gemm_k64.hip tile t (64-deep
# stages; tiles 9 / 10 = csrc/gemm_w4.hip, which also covers K % 64 != 0 -- the round-2 kernel that did is gone)
K64 = 10
# csrc/gemm_k64.hip tiles the dispatcher times: 5 / 6 / 8 = the 8-wave 256x256 / 256x128 / 128x256
# tiles with the two-phase K loop (3-11 % faster than their four-phase forms 1 / 2 / 4 at every
# GPT-2 and Llama shape: profiles/gemm_k64_vs_hipblaslt.txt), 3 / 7 = 128x128 in both forms
K64_TILES = (10, 5, 6, 3, 7, 8)  # 10: csrc/gemm_w4.hip (4 waves, 256 x 256; staged epilogue where one bf16 output)
# 192-wide tiles, K-major A and B only (the forward layout): 11 = 256 x 192 (8 waves), 12 = 128 x 192 (4 waves,
# two workgroups per CU) -- GPT-2's N = 768 / 2304 / 3072 / 50304 in whole tile columns, so the qkv forward is
# 768 tiles (3 rounds of 256 CUs) instead of 288 / 576 (1.1 / 2.3 rounds) at the 256- / 128-wide tiles
K64_TILES_KMAJOR = (11, 12)
# a hand-written candidate wins a shape when it is at most this much slower than the library (1.0: the
# faster one; a 2 % preference measured 0.25 ms/step slower on the GPT-2 DDP step, same-box A/B)
_PREFER_DTA = 1.0


def gemm_candidates(M: int, N: int, K: int, a_t: bool = False, b_t: bool = False, sk: bool = True,
                    big: bool = False) -> list:
    """Hand-written GEMM implementations that cover an M x N x K problem in the given operand layout
    (ids as in _GEMM_CHOICE; ``sk``: with the stream-K forms where they can help; ``big``: an operand spans
    2 GiB or more, past the buffer descriptors' 32-bit offsets -- the tiles that DMA only through descriptors,
    the 192-wide, the stream-K forms and W4, are left out).  Memoised per shape."""
    key = (M, N, K, bool(a_t), bool(b_t), bool(sk), bool(big))
    c = _CANDS.get(key)
    if c is None:
        c = _CANDS[key] = _gemm_candidates(M, N, K, a_t, b_t, sk and not big)
        if big:  # (csrc/gemm_w4.hip too: descriptor DMA only)
            c = _CANDS[key] = [x for x in c if x - K64 not in K64_TILES_KMAJOR + (10,)]
    return c


def _big(*ts: Optional[torch.Tensor]) -> bool:
    """Some operand's bytes reach past 2 GiB from its base (csrc/gemm_k64.hip: descriptor DMA off)."""
    for t in ts:
        if t is not None and t.numel() and 2 * ((t.shape[0] - 1) * t.stride(0) + t.shape[-1]) >= 0x7FFFFFFF:
            return True
    return False


_CANDS: Dict[tuple, list] = {}


def _gemm_candidates(M: int, N: int, K: int, a_t: bool, b_t: bool, sk: bool) -> list:
    C = native()
    kmaj = not (a_t or b_t)
    tiles = K64_TILES + (K64_TILES_KMAJOR if kmaj else ())
    out = [K64 + t for t in tiles if C.gemm64_tile(M, N, K, t)]
    if sk and not (a_t and not b_t):
        out += [K64 + (t | SK_BIT) for t in _SK_TILES + (_SK_TILES_KMAJOR if kmaj else ())
                if C.gemm64_tile(M, N, K, t | SK_BIT) and _sk_useful(M, N, K, t)]
    return out


def _pick(kind: str, M: int, N: int, K: int, cands: Dict[int, Callable[[], object]], prefer: float = _PREFER_DTA) -> int:
    """Implementation for one (possibly fused) GEMM shape: ``cands`` maps implementation ids to
    callables computing the SAME fused result (0 = hipBLASLt + separate epilogue kernels).  In
    order: a ``DTA_GEMM_CACHE`` entry; ``DTA_GEMM=torch`` / ``dta`` (forced); the tracked table
    (:func:`gemm_table`); else in-run interleaved timing (median of :func:`_rounds` rounds): the
    fastest hand-written candidate unless the library is faster (``prefer``: the factor by which
    the hand-written one may be slower and still win -- 0.85 for the GELU dual store, whose in-step
    cost exceeds its timed cost).  Memoised per (kind, M, N, K) and process."""
    if not _CACHE_LOADED[0]:
        _load_cache()
    key = (kind, M, N, K)
    c = _GEMM_CHOICE.get(key)
    if c is not None and (c in cands or c == 0):
        GEMM_PICK_SOURCE.setdefault(key, "cache")
        return c
    mode = os.environ.get("DTA_GEMM", "auto")
    dta = [k for k in cands if k != 0]
    src = "forced"
    t = gemm_table().get(key) if mode == "auto" else None
    if t is not None and not (t == 0 or t in cands):
        t = None
    if mode == "torch" or not dta:
        c = 0
    elif t is not None:
        c, src = t, "table"
        if os.environ.get("DTA_GEMM_VERIFY", "0") == "1" and not _capturing():
            times = _time_us(cands, rounds=_rounds())
            GEMM_TIMES[key] = times
            best = min(times, key=times.get)
            if times[c] > 1.03 * times[best]:
                import logging

                logging.getLogger(__name__).warning(
                    "GEMM %s %dx%dx%d: tracked pick %s measures %.1f us here, %s %.1f us", kind, M, N, K,
                    _impl_name(c), times[c], _impl_name(best), times[best])
    elif mode == "dta" or _capturing():
        c = dta[0]
        auto = native().gemm64_tile(M, N, K, 0)
        if K64 + auto in dta:
            c = K64 + auto
    else:
        times = _time_us(cands, rounds=_rounds())
        GEMM_TIMES[key] = times
        best = min(dta, key=times.get)
        c = best if 0 not in times or times[best] <= prefer * times[0] else 0
        src = "timed"
        if _TABLE:  # (a table exists but lacks this shape: say so)
            import logging

            logging.getLogger(__name__).info("GEMM %s %dx%dx%d not in the tracked table: timed in-run -> %s",
                                             kind, M, N, K, _impl_name(c))
    if c and (c - K64) & SK_BIT and _sk_cnt(torch.device("cuda", torch.cuda.current_device())) is None:
        c = K64 + ((c - K64) & ~SK_BIT)  # (no counters yet, inside a graph capture: the tile's plain form)
    _GEMM_CHOICE[key] = c
    GEMM_PICK_SOURCE[key] = src
    if mode == "auto":
        _save_cache()
    return c


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _impl_name(c: int) -> str:
    if not c:
        return "hipblaslt"
    t = c - K64
    return f"k64/t{t & ~SK_BIT}sk" if t & SK_BIT else f"k64/t{t}"


# ---- stream-K forms of the two-phase tiles (csrc/gemm_k64.hip SkArgs): tile id | SK_BIT.  The grid is the
# tile's resident workgroups and each takes an equal run of (tile, K-tile) units, so a shape whose tile count
# leaves part of the chip idle in its last round (GPT-2's N = 768 input gradients: 192 tiles of 256 x 128 on
# 256 CUs; Llama's qkv weight gradient: 384 of 256 x 256) keeps every CU busy; a tile cut between workgroups
# is finished by the last to arrive, the parts summed in K order (deterministic).
SK_BIT = 64
_SK_TILES = (5, 6, 7, 8)            # any layout but TT
_SK_TILES_KMAJOR = (11, 12)         # K-major A and B
_SK_CNT: Dict[int, torch.Tensor] = {}  # per device: the arrival counters (zero between launches)
_SK_CNT_LEN = 1 << 17


def _sk_cnt(dev: torch.device) -> Optional[torch.Tensor]:
    """The device's stream-K arrival counters (allocated zeroed on first use outside graph capture; the kernel
    leaves them zero).  GEMMs of one device run on one stream at a time (the compute stream, or the capture
    stream while a step graph is recorded), so one buffer per device serves them all."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    c = _SK_CNT.get(idx)
    if c is None and not _capturing():
        c = _SK_CNT[idx] = torch.zeros(_SK_CNT_LEN, dtype=torch.int32, device=dev)
    return c


_NUM_CUS: Dict[int, int] = {}


def _num_cus() -> int:
    """Compute units of the current device (256 on a whole MI355X; fewer in a CU-partition mode) --
    what ``dta_gemm_k64_sk_plan`` sizes the stream-K grid from."""
    if not torch.cuda.is_available():  # (CPU: the dispatch rules are unit-tested with a stand-in kernel library)
        return 256
    idx = torch.cuda.current_device()
    n = _NUM_CUS.get(idx)
    if n is None:
        n = _NUM_CUS[idx] = int(torch.cuda.get_device_properties(idx).multi_processor_count)
    return n


def _sk_useful(M: int, N: int, K: int, t: int) -> bool:
    """A stream-K candidate where the plain tile's last round would leave >= 10 % of the slots idle and the
    reduction is deep (K >= 8192): every cut tile costs an fp32 slab per part (128-256 KB, written and read
    back at the end of a workgroup's run), which the shallow shapes do not earn back -- GPT-2's K = 768-3072
    input gradients measured 30-60 % slower in stream-K form, its K = 8192 weight gradients and K = 50304
    LM-head input gradient faster (profiles/gemm_table_sk_r5t.jsonl)."""
    if K < 8192:
        return False
    tiles, grid, _span = native().gemm64_sk_plan(M, N, K, t | SK_BIT)
    if tiles <= 0 or tiles > _SK_CNT_LEN:
        return False
    slots = _num_cus() * (2 if t in (7, 12) else 1)  # (the kernel's plan sizes its grid from the same count)
    rounds = -(-tiles // slots)
    return tiles < 0.9 * rounds * slots


def _cnt_for(impl: int, x: torch.Tensor) -> Optional[torch.Tensor]:
    return _sk_cnt(x.device) if (impl - K64) & SK_BIT else None


def _run_gemm(impl: int, a: torch.Tensor, b: torch.Tensor, a_t: bool, b_t: bool, out: Optional[torch.Tensor] = None,
              alpha: float = 1.0, bias: Optional[torch.Tensor] = None,
              alpha_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
    return native().gemm64(a, b, a_t, b_t, out, None, False, alpha, bias, 0, None, impl - K64, -1, alpha_dev,
                           _cnt_for(impl, a))[0]


def _gemm_ok(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None) -> bool:
    return (a.stride(-1) == 1 and b.stride(-1) == 1 and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0 and (bias is None or bias.is_contiguous())
            and (out is None or (out.is_contiguous() and out.data_ptr() % 16 == 0)))


def gemm(a: torch.Tensor, b: torch.Tensor, a_t: bool = False, b_t: bool = False, bias: Optional[torch.Tensor] = None,
         alpha: float = 1.0, kind: str = "", out: Optional[torch.Tensor] = None,
         scale_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 ``alpha * op(a) op(b)^T (+ bias)`` on GPU, a: [M, K] (a_t: [K, M]), b: [N, K] (b_t: [K, N]);
    hand-written kernel or hipBLASLt per shape (see module doc).  ``scale_dev`` (fp32 [1] on the GPU, no
    bias): the product is also multiplied by it -- inside the hand-written kernel's epilogue (in fp32,
    before the rounding), or by a separate pass after the library GEMM (after it; the LM head's scale is
    1 / token count, a power of two at the configs' token counts, so both round identically there).
    Every timed candidate includes its scaling, so the pick compares the costs the step pays."""
    M, K = (a.shape[1], a.shape[0]) if a_t else (a.shape[0], a.shape[1])
    N = b.shape[1] if b_t else b.shape[0]

    def run_torch() -> torch.Tensor:
        A = a.t() if a_t else a
        B = b if b_t else b.t()
        if bias is not None and alpha == 1.0:
            return torch.addmm(bias, A, B) if out is None else torch.addmm(bias, A, B, out=out)
        y = torch.mm(A, B) if out is None else torch.mm(A, B, out=out)
        if alpha != 1.0:
            y.mul_(alpha)
        if scale_dev is not None:
            y.mul_(scale_dev)  # (one pass, the product in fp32: no separate cast of the scale)
        return y if bias is None else y.add_(bias)

    impl = 0
    if _gemm_ok(a, b, bias, out):
        cands: Dict[int, Callable[[], object]] = {0: run_torch}
        for t in gemm_candidates(M, N, K, a_t, b_t, big=_big(a, b)):
            cands[t] = (lambda t=t: _run_gemm(t, a, b, a_t, b_t, out, alpha, bias, scale_dev))
        impl = _pick(kind + ("b" if bias is not None else ""), M, N, K, cands)
    if impl:
        GEMM_STATS["dta"] += 1
        return _run_gemm(impl, a, b, a_t, b_t, out, alpha, bias, scale_dev)
    GEMM_STATS["torch"] += 1
    return run_torch()


def gemm_gelu_dual(x2: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
    """``h = x W^T + b`` and ``a = gelu_tanh(h)`` (of the rounded h) -- the GPT-2 MLP up-projection
    with its activation: the 64-deep GEMM with the GELU in its epilogue storing BOTH (one pass, no
    re-read of h), or hipBLASLt + the GELU kernel, whichever measured faster for the shape (the
    FUSED costs are compared)."""
    M, K = x2.shape
    N = w.shape[0]
    C = native()

    def run_torch() -> Tuple[torch.Tensor, torch.Tensor]:
        h = torch.addmm(b, x2, w.t()) if b is not None else torch.mm(x2, w.t())
        return h, C.gelu_fwd(h, -1)

    def run_k64(t: int) -> Tuple[torch.Tensor, ...]:
        h = torch.empty(M, N, dtype=x2.dtype, device=x2.device)
        return tuple(C.gemm64(x2, w, False, False, h, torch.empty_like(h), False, 1.0, b, 2, None, t, -1, None,
                              _cnt_for(K64 + t, x2)))

    impl = 0
    if _gemm_ok(x2, w, b) and N % 8 == 0:
        cands: Dict[int, Callable[[], object]] = {0: run_torch}
        for c in gemm_candidates(M, N, K, big=_big(x2, w)):
            cands[c] = (lambda t=c - K64: run_k64(t))
        # the dual store must win by 15 %: its two output streams cost more inside the step than in
        # the back-to-back timing (GPT-2 fc: per-fragment 85.8 us in-step vs 69-76 timed, staged 78-82
        # vs 64.8; hipBLASLt + GELU kernel 47.1 + 23.1 us in-step -- profiles/gpt2_ddp_1gpu_kernels_r4.txt,
        # _r4c.txt, _r4f.txt)
        impl = _pick("fwd_gelu" + ("b" if b is not None else ""), M, N, K, cands, prefer=0.85)
    if impl:
        GEMM_STATS["dta"] += 1
        return run_k64(impl - K64)
    GEMM_STATS["torch"] += 1
    return run_torch()


# ------------------------------------------------------------------ linear
def _grad_dest(p: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """The slice of the DDP engine's flat gradient buffer that ``p``'s gradient
    goes to, when this backward may write it there directly: the engine hands
    fresh gradients over (``zero_grad(set_to_none=True)``), ``p.grad`` is unset
    and no other use of ``p`` in this backward has claimed the slice (a second
    use would overwrite it before autograd sums the two).  Autograd then adopts
    the returned view as ``p.grad`` and the engine's per-bucket copy kernel has
    nothing to move (parallel/ddp.py)."""
    if p is None:
        return None
    gdest = getattr(p, "_dta_gdest", None)  # FSDP unit views (parallel/fsdp.py _Unit.piece_dest)
    if gdest is not None:
        d = gdest()
        return d if d is not None and d.dtype == p.dtype else None
    tag = getattr(p, "_dta_flat", None)
    if tag is None or p.grad is not None:
        return None
    group, i = tag
    if not group.steal_ok or not group.grad.is_cuda or group.grad.dtype != p.dtype or i in group.direct_claimed:
        return None
    group.direct_claimed.add(i)
    return group.grad_view(i)


# ------------------------------------------------------------------ end-of-backward join
# Nothing on the backward's critical path reads a weight gradient (the chain is dgrad -> norm /
# activation / attention backward -> the next layer's dgrad), so weight gradients may be deferred
# (below) and must be joined before anything reads them: every DDP bucket launch and the end of
# the backward call :func:`wgrad_join`.  (Round 2 also ran them on a second HIP stream; it won in
# 6 of 8 same-box pairs but lost 25-45 % on one box -- the hardware scheduler's interleaving of
# two queues is not under this code's control -- and was removed in round 4.)
_SIDE_CB = [False]  # the end-of-backward join callback is queued
_FWD_GEN = [0]


_CLOSED_GEN = [0]  # every forward generation <= this one has had its backward finalized
_GEN_USES = [0]    # weight uses (that will be differentiated) counted in the current generation


def new_forward_generation() -> None:
    """Start counting native-Linear weight uses afresh (called per DDP forward)."""
    if _GEN_USES[0] == 0:  # (a no-grad forward: no backward will close it)
        _CLOSED_GEN[0] = _FWD_GEN[0]
    # After a normal backward the end-of-backward join has emptied the queue, so this reset is a
    # no-op there; after a backward that RAISED (generation left open) it drops the abandoned step's
    # deferred (dy, x, dest) entries and re-arms the join callback -- otherwise the next backward
    # would never queue its flush (_SIDE_CB stuck) and would flush stale entries into the same
    # flat-gradient slices as its own (two groups writing one destination in one launch).
    _SIDE_CB[0] = False
    _DEFER.clear()
    _NORM_DEFER.clear()
    _DEFER_TILES[0] = 0
    _FWD_GEN[0] += 1
    _GEN_USES[0] = 0


def abandon_step() -> None:
    """A step stopped midway (a failed graph capture): drop what its backward queued."""
    _SIDE_CB[0] = False
    _DEFER.clear()
    _NORM_DEFER.clear()
    _DEFER_TILES[0] = 0
    _GEN_USES[0] = 0
    _CLOSED_GEN[0] = _FWD_GEN[0]


def close_forward_generations() -> None:
    """The backward of every forward so far is finished (the DDP engine's end-of-backward
    finalize): a weight's uses in those generations no longer count against a later one."""
    _CLOSED_GEN[0] = _FWD_GEN[0]


def _count_use(w: torch.Tensor) -> None:
    g = getattr(w, "_dta_gen", -1)
    if g != _FWD_GEN[0]:
        # two forwards before one backward (e.g. a loss summed over two calls): a use in an
        # earlier generation whose backward has not run yet is a second use of the weight in
        # that coming backward, so the weight is not single-use (no deferred / side-stream
        # gradient: its returned slice would be summed before the deferred GEMM wrote it)
        prev_open = g > _CLOSED_GEN[0] and getattr(w, "_dta_uses", 0) > 0
        w._dta_gen = _FWD_GEN[0]
        w._dta_uses = 1 if prev_open else 0
    w._dta_uses += 1
    _GEN_USES[0] += 1


def _single_use(w: Optional[torch.Tensor]) -> bool:
    return w is not None and _FWD_GEN[0] > 0 and getattr(w, "_dta_gen", -1) == _FWD_GEN[0] \
        and getattr(w, "_dta_uses", 0) == 1


def wgrad_join(device: Optional[torch.device] = None) -> None:
    """Every weight gradient of this backward written: the deferred ones launched
    (:func:`wgrad_flush`) on the current stream."""
    wgrad_flush()


def _end_of_backward_join() -> None:
    _SIDE_CB[0] = False
    wgrad_flush()


def _queue_end_join() -> None:
    if not _SIDE_CB[0]:
        from torch.autograd import Variable

        Variable._execution_engine.queue_callback(_end_of_backward_join)
        _SIDE_CB[0] = True


# ------------------------------------------------------------------ deferred, grouped weight gradients
# At GPT-2 sizes one layer's weight gradients (2304x768, 768x768, 3072x768, 768x3072 over
# 8192 tokens) are too small to fill 256 CUs on their own, which is why the per-call kernel
# splits the token reduction (fp32 slabs, ~650 TF/s).  Nothing reads a weight gradient
# before the DDP bucket launch / the end of the backward, so the single-use weights whose
# gradients go straight into flat-buffer slices are DEFERRED instead: their (dy, x) pairs
# are queued, and once the queue holds >= DTA_WGRAD_GROUP 256 x 256 output tiles (default
# 200: two GPT-2 layers = 216 tiles) ONE grouped launch computes all of them over the full
# token reduction -- no split, no slabs, bias gradients from the same MFMA pipe
# (csrc/gemm_k64.hip gemm_k64_group_kernel).  The queue is flushed before every DDP bucket
# launch and at the end of the backward (same stream: no further synchronisation); under the
# FSDP engine (unit pieces, ``_Piece.defer_ok``) a unit's reduce-scatter waits for the flush that
# writes its pieces (parallel/fsdp.py ``_launch_waiting``).
_DEFER: list = []
_DEFER_TILES = [0]
# called after every flush launched its groups (the DDP engine's per-bucket optimizer
# step waits for the weight gradients of its bucket: parallel/ddp.py overlap_optimizer)
FLUSH_LISTENERS: list = []


def wgrad_pending() -> bool:
    """Weight (or norm gamma / beta) gradients are queued (their flat-buffer slices are not written yet)."""
    return bool(_DEFER) or bool(_NORM_DEFER)


def _group_threshold() -> int:
    v = os.environ.get("DTA_WGRAD_GROUP", "200")
    return max(0, int(v)) if v.strip() else 0


def wgrad_flush() -> None:
    """Launch the queued weight gradients (grouped, at most gemm64_group_max() per launch) and the queued
    norm gamma / beta column sums (one batched launch)."""
    if not _DEFER and not _NORM_DEFER:
        return
    C = native()
    if _DEFER:
        items = list(_DEFER)
        _DEFER.clear()
        _DEFER_TILES[0] = 0
        # csrc/gemm_k64.hip's grouped kernel (64-deep two-phase loop; every queued reduction is a multiple of
        # 64 tokens, _weight_grad).  csrc/gemm_w4.hip's grouped kernel (impl 2) measured slower on every
        # weight-gradient shape (profiles/gemm_w4_vs_k64_hipblaslt.txt) and has no bias gradients.
        gmax = C.gemm64_group_max()
        for i in range(0, len(items), gmax):
            part = items[i:i + gmax]
            C.gemm_wgrad_group([it[0] for it in part], [it[1] for it in part], [it[2] for it in part],
                               [it[3] for it in part], -1, 1)
        GEMM_STATS["group_launches"] += (len(items) + gmax - 1) // gmax
    if _NORM_DEFER:
        jobs = list(_NORM_DEFER)
        _NORM_DEFER.clear()
        C.colsum_batch([j[0] for j in jobs], [j[1] for j in jobs], -1)
    for fn in list(FLUSH_LISTENERS):
        fn()


_DEFER_MAX_TILES = 48  # 256 x 256 output tiles: larger weight gradients fill the chip by themselves (gemm())


def _weight_grad(dy2: torch.Tensor, x2: torch.Tensor, with_bias: bool = False, w: Optional[torch.Tensor] = None,
                 b: Optional[torch.Tensor] = None) -> Union[torch.Tensor, Tuple[torch.Tensor, Optional[torch.Tensor]]]:
    """dW = dy^T x (and, ``with_bias``, db = column sums of dy: returns (dW, db)).
    A single-use weight whose gradient goes straight into its flat-gradient slice is DEFERRED
    (queued for a grouped launch of the 64-deep kernel, bias gradient from the same MFMA pipe:
    see ``_DEFER``) -- at GPT-2 sizes one weight gradient (768 x 768 .. 3072 x 768 over 8192
    tokens) cannot fill 256 CUs by itself, a group of them can.  Anything else (a weight used
    twice, no flat slice, shapes off the 256 grid) goes through :func:`gemm` (hand-written or
    hipBLASLt per shape) and the bias-gradient kernel.  With the parameters ``w`` / ``b`` given,
    the results go straight into their flat gradient slices when :func:`_grad_dest` allows it."""
    K, M = dy2.shape
    N = x2.shape[1]
    cw = _grad_dest(w)
    cb = _grad_dest(b) if with_bias else None
    thr = _group_threshold()
    if thr and M % 256 == 0 and N % 256 == 0 and K % 64 == 0 and dy2.stride(1) == 1 and x2.stride(1) == 1 \
            and (M // 256) * (N // 256) <= _DEFER_MAX_TILES and x2.stride(0) % 8 == 0 \
            and cw is not None and (cb is not None or not with_bias) \
            and _defer_ok(w) \
            and _single_use(w) and cw.stride(0) % 8 == 0 \
            and cw.data_ptr() % 16 == 0 and (cb is None or cb.data_ptr() % 16 == 0):
        # deferred: computed by a grouped launch at the next flush (see _DEFER).  The queue
        # holds ALIASES of the slices, never the tensors returned to autograd: a second
        # reference to a returned gradient makes AccumulateGrad clone it instead of
        # adopting it -- a copy of the slice taken BEFORE the deferred GEMM wrote it,
        # which the DDP bucket copy then moved back over the GEMM's result whenever a
        # flush fell between this backward and the bucket's launch (stale gradients)
        _DEFER.append((dy2, x2, cw.view(cw.shape), None if cb is None else cb.view(cb.shape)))
        _DEFER_TILES[0] += (M // 256) * (N // 256)
        GEMM_STATS["deferred_wgrad"] += 1
        _queue_end_join()
        if _DEFER_TILES[0] >= thr or len(_DEFER) >= 4 * native().gemm64_group_max():
            wgrad_flush()
        return (cw, cb) if with_bias else cw
    if cw is not None and not (cw.is_contiguous() and cw.data_ptr() % 16 == 0):
        cw = None  # (an unaligned slice stays claimed: autograd's result is copied in)
    dw = gemm(dy2, x2, True, True, kind="wgrad", out=cw)
    if not with_bias:
        return dw
    db = native().bias_grad(dy2, False, -1)
    if cb is not None:
        cb.copy_(db)
        db = cb
    return dw, db


class _Linear(Function):
    """y = x W^T (+ b): forward and input-gradient GEMMs through :func:`gemm`
    (bias fused in the epilogue), weight (and bias) gradients deferred into a grouped
    launch or through :func:`gemm` (see _weight_grad)."""

    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        ctx.params = (w, b)  # the Parameters themselves (their .grad decides a direct write)
        if ctx.needs_input_grad[1]:
            _count_use(w)  # (a weight used once may take the side-stream weight gradient)
        x2 = x.reshape(-1, x.shape[-1])
        return gemm(x2, w, bias=b, kind="fwd").view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        x, w = ctx.saved_tensors
        pw, pb = ctx.params
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gemm(dy2, w, False, True, kind="dgrad").view(*x.shape[:-1], w.shape[1])
        want_b = ctx.has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            r = _weight_grad(dy2, x.reshape(-1, x.shape[-1]), with_bias=want_b, w=pw, b=pb if want_b else None)
            dw, db = r if want_b else (r, None)
        elif want_b:
            db = native().bias_grad(dy2, False, -1)
        return dx, dw, db


def _dgelu_dgrad(dy2: torch.Tensor, w: torch.Tensor, h2: torch.Tensor) -> torch.Tensor:
    """dh = (dy W) * gelu_tanh'(h): the input gradient of ``gelu(h) W^T + b`` -- on a hand-written
    GEMM with the GELU derivative in its epilogue (one pass, no dA round trip through HBM), or
    hipBLASLt followed by the GELU-backward kernel, whichever measured faster for the shape."""
    M, K = dy2.shape
    N = w.shape[1]
    C = native()
    ok = (w.is_contiguous() and w.data_ptr() % 16 == 0 and dy2.data_ptr() % 16 == 0 and h2.is_contiguous()
          and h2.data_ptr() % 16 == 0 and N % 8 == 0)

    def run(impl: int) -> torch.Tensor:
        return C.gemm64(dy2, w, False, True, None, None, False, 1.0, None, 16, h2, impl - K64, -1, None,
                        _cnt_for(impl, dy2))[0]

    def run_torch() -> torch.Tensor:
        return C.gelu_bwd(torch.mm(dy2, w), h2, -1)

    impl = 0
    if ok:
        cands: Dict[int, Callable[[], object]] = {0: run_torch}
        for t in gemm_candidates(M, N, K, False, True, big=_big(dy2, w)):
            cands[t] = (lambda t=t: run(t))
        impl = _pick("dgelu", M, N, K, cands)
    if impl:
        GEMM_STATS["dta"] += 1
        return run(impl)
    GEMM_STATS["torch"] += 1
    return run_torch()


_DSW_TILES = (5, 6, 7, 8)  # the two-phase 64-deep tiles: the SwiGLU-backward epilogue's instantiations


def _swiglu_dgrad(dy2: torch.Tensor, w: torch.Tensor, ab2: torch.Tensor) -> torch.Tensor:
    """d[a | b] of ``silu(a) * b`` through ``y = (silu(a) b) W^T``: on a hand-written GEMM whose epilogue
    reads the [a | b] rows and writes [da | db] (``csrc/gemm_k64.hip`` EPI_DSWIGLU: no [tokens, F] round
    trip of the product through HBM), or hipBLASLt followed by the SwiGLU-backward kernel, whichever is
    faster for the shape (the tracked table / per-shape timing, kind ``dswiglu``)."""
    M, K = dy2.shape
    N = w.shape[1]
    C = native()
    ok = (w.is_contiguous() and w.data_ptr() % 16 == 0 and dy2.data_ptr() % 16 == 0 and ab2.is_contiguous()
          and ab2.data_ptr() % 16 == 0 and ab2.shape[1] == 2 * N and N % 8 == 0)

    def run(impl: int) -> torch.Tensor:
        return C.gemm64(dy2, w, False, True, None, None, False, 1.0, None, 64, ab2, impl - K64)[0]

    def run_torch() -> torch.Tensor:
        return C.swiglu_bwd(torch.mm(dy2, w), ab2, -1)

    impl = 0
    if ok:
        cands: Dict[int, Callable[[], object]] = {0: run_torch}
        for t in _DSW_TILES:
            if C.gemm64_tile(M, N, K, t):
                cands[K64 + t] = (lambda t=t: run(K64 + t))
        impl = _pick("dswiglu", M, N, K, cands)
    if impl:
        GEMM_STATS["dta"] += 1
        return run(impl)
    GEMM_STATS["torch"] += 1
    return run_torch()


class _SwigluLinear(Function):
    """y = (silu(a) * b) W^T for ab = [a | b] (Llama's SwiGLU MLP down projection with its activation).
    Backward: dW from the weight-gradient path of :class:`_Linear` (the activation saved in forward),
    d[a | b] through :func:`_swiglu_dgrad` (the SwiGLU backward folded into the input-gradient GEMM)."""

    @staticmethod
    def forward(ctx: Any, ab: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        abc = ab.contiguous()
        act = native().swiglu_fwd(abc, -1)
        ctx.save_for_backward(abc, act, w)
        ctx.params = (w, None)
        if ctx.needs_input_grad[1]:
            _count_use(w)
        return gemm(act.reshape(-1, act.shape[-1]), w, kind="fwd").view(*ab.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        ab, act, w = ctx.saved_tensors
        pw, _ = ctx.params
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dab = dw = None
        if ctx.needs_input_grad[0]:
            dab = _swiglu_dgrad(dy2, w, ab.reshape(-1, ab.shape[-1])).view(ab.shape)
        if ctx.needs_input_grad[1]:
            dw = _weight_grad(dy2, act.reshape(-1, act.shape[-1]), with_bias=False, w=pw, b=None)
        return dab, dw


def swiglu_linear(ab: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``linear(swiglu(ab), w)`` with the SwiGLU backward fused into the input-gradient GEMM on GPU."""
    if ab.is_cuda and ab.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 \
            and ab.shape[-1] % 16 == 0 and w.shape[0] % 8 == 0:
        return _SwigluLinear.apply(ab, w)
    return linear(swiglu(ab), w)


class _GeluLinear(Function):
    """y = gelu_tanh(h) W^T + b (the second half of a GPT-2 MLP).  Backward:
    dW / db from the weight-gradient path of :class:`_Linear`, and dh through
    :func:`_dgelu_dgrad` (the GELU backward folded into the input-gradient GEMM)."""

    @staticmethod
    def forward(ctx: Any, h: torch.Tensor, w: torch.Tensor, b: torch.Tensor, a: Optional[torch.Tensor] = None) -> torch.Tensor:
        hc = h.contiguous()
        if a is None:
            a = native().gelu_fwd(hc, -1)
        ctx.save_for_backward(hc, a, w)
        ctx.has_b = b is not None
        ctx.params = (w, b)
        if ctx.needs_input_grad[1]:
            _count_use(w)
        a2 = a.reshape(-1, a.shape[-1])
        return gemm(a2, w, bias=b, kind="fwd").view(*h.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        h, a, w = ctx.saved_tensors
        pw, pb = ctx.params
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dh = dw = db = None
        if ctx.needs_input_grad[0]:
            dh = _dgelu_dgrad(dy2, w, h.reshape(-1, h.shape[-1])).view(h.shape)
        want_b = ctx.has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            r = _weight_grad(dy2, a.reshape(-1, a.shape[-1]), with_bias=want_b, w=pw, b=pb if want_b else None)
            dw, db = r if want_b else (r, None)
        elif want_b:
            db = native().bias_grad(dy2, False, -1)
        return dh, dw, db, None


class _LinearGelu(Function):
    """(h, a) = (x W^T + b, gelu_tanh(h)): the GPT-2 MLP up-projection with its activation
    computed in the GEMM's epilogue (:func:`gemm_gelu_dual`).  ``a`` is the input of the
    down-projection (:class:`_GeluLinear` with ``a`` given), which differentiates through
    the GELU itself and returns the gradient of ``h`` -- so ``a`` carries no gradient here
    and backward is exactly :class:`_Linear`'s."""

    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        ctx.params = (w, b)
        if ctx.needs_input_grad[1]:
            _count_use(w)
        x2 = x.reshape(-1, x.shape[-1])
        h, a = gemm_gelu_dual(x2, w, b)
        shp = (*x.shape[:-1], w.shape[0])
        h, a = h.view(shp), a.view(shp)
        ctx.mark_non_differentiable(a)
        # no zero-filled gradient for ``a`` (autograd would materialise one per layer: a
        # [tokens, 4C] bf16 fill -- 50 MB and ~9 us per GPT-2 layer in the rocprof trace)
        ctx.set_materialize_grads(False)
        return h, a

    @staticmethod
    def backward(ctx: Any, dh: Optional[torch.Tensor], da: Optional[torch.Tensor]) -> Tuple[Optional[torch.Tensor], ...]:
        if dh is None:  # (h unused downstream: nothing to propagate)
            return None, None, None
        return _Linear.backward(ctx, dh)


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """``(h, gelu(h))`` for ``h = linear(x, w, b)``; feed both to :func:`gelu_linear` (``a=``)."""
    if x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 \
            and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0:
        return _LinearGelu.apply(x, w, b)
    h = linear(x, w, b)
    return h, gelu(h).detach()


def gelu_linear(h: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None,
                a: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``linear(gelu(h), w, b)`` with the GELU backward fused into the input-gradient GEMM on GPU;
    ``a``: gelu(h) already computed (by :func:`linear_gelu`'s epilogue)."""
    if h.is_cuda and h.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 \
            and h.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0:
        return _GeluLinear.apply(h, w, b, a)
    return linear(gelu(h), w, b)


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    if x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 \
            and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0:
        return _Linear.apply(x, w, b)
    return F.linear(x, w, b)


class Linear(torch.nn.Linear):
    """``nn.Linear`` (same parameters / state-dict keys) routed through :func:`linear`."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return linear(x, self.weight, self.bias)


class LMHead(torch.nn.Linear):
    """The untied output projection as a module of its own (same parameter / state-dict key as
    ``nn.Linear``): ``head(y, targets)`` is the fused head + token cross-entropy
    (:func:`linear_cross_entropy`), ``head(y)`` the logits.  Being a module call makes it an
    FSDP unit of its own (parallel/fsdp.py ``lm_wrap_policy``): gathered by a prefetch during the
    last blocks, its gradient reduce-scattered as soon as the head's backward -- the first of
    the backward -- is done."""

    def forward(self, y: torch.Tensor, targets: Optional[torch.Tensor] = None) -> torch.Tensor:
        if targets is not None:
            return linear_cross_entropy(y, self.weight, targets)
        return linear(y, self.weight, self.bias)


class Embedding(torch.nn.Embedding):
    """``nn.Embedding`` (same parameter / key) through :func:`embedding` (the native backward).
    Its backward reads no weight values, so as an FSDP unit it is never re-gathered for backward."""

    fsdp_backward_needs_params = False

    def forward(self, idx: torch.Tensor) -> torch.Tensor:
        return embedding(idx, self.weight)


# ------------------------------------------------------------------ activations
class _Gelu(Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor) -> torch.Tensor:
        xc = x.contiguous()
        ctx.save_for_backward(xc)
        return native().gelu_fwd(xc, -1)

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> torch.Tensor:
        (x,) = ctx.saved_tensors
        return native().gelu_bwd(dy.contiguous(), x, -1)


def gelu(x: torch.Tensor) -> torch.Tensor:
    if x.is_cuda:
        _need_bf16(x)
        return _Gelu.apply(x)
    return F.gelu(x, approximate="tanh")


class _SwiGLU(Function):
    @staticmethod
    def forward(ctx: Any, ab: torch.Tensor) -> torch.Tensor:
        abc = ab.contiguous()
        ctx.save_for_backward(abc)
        return native().swiglu_fwd(abc, -1)

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> torch.Tensor:
        (ab,) = ctx.saved_tensors
        return native().swiglu_bwd(dy.contiguous(), ab, -1)


def swiglu(ab: torch.Tensor) -> torch.Tensor:
    """``silu(a) * b`` for ``ab = [a | b]`` along the last dim."""
    if ab.is_cuda:
        _need_bf16(ab)
        return _SwiGLU.apply(ab)
    a, b = ab.chunk(2, dim=-1)
    return F.silu(a) * b


# ------------------------------------------------------------------ rotary
def rope_tables(seq_len: int, head_dim: int, theta: float = 10000.0,
                device: Any = None) -> Tuple[torch.Tensor, torch.Tensor]:
    # (on the host explicitly: under a ``torch.device("meta")`` build the tables still get values)
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64, device="cpu") / head_dim))
    t = torch.arange(seq_len, dtype=torch.float64, device="cpu")
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def rope_reference(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    S, D = x.shape[1], x.shape[-1]
    c = cos[:S].view(1, S, 1, D // 2).to(torch.float32)
    s = sin[:S].view(1, S, 1, D // 2).to(torch.float32)
    x1, x2 = x.float()[..., : D // 2], x.float()[..., D // 2:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)


class _Rope(Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
        y = x.contiguous().clone()
        native().rope_(y, cos, sin, False, -1)
        ctx.save_for_backward(cos, sin)
        return y

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        cos, sin = ctx.saved_tensors
        dx = dy.contiguous().clone()
        native().rope_(dx, cos, sin, True, -1)
        return dx, None, None


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """Rotate-half RoPE on [B, S, heads, D]."""
    if x.is_cuda:
        _need_bf16(x)
        return _Rope.apply(x, cos, sin)
    return rope_reference(x, cos, sin)


# ------------------------------------------------------------------ embedding
def _claimed_slice(p: torch.Tensor) -> Optional[torch.Tensor]:
    """The flat-buffer slice of ``p`` when another use of ``p`` in this backward already
    wrote its gradient there (:func:`_grad_dest` claimed it; autograd has not accumulated
    yet): a further contribution can be added into it in place."""
    gd = getattr(p, "_dta_gdest", None)
    if gd is not None:  # FSDP unit view: its piece of the unit's gradient buffer (parallel/fsdp.py _Piece)
        cs = getattr(gd, "claimed_slice", None)
        d = cs() if cs is not None else None
        return d if d is not None and d.dtype == p.dtype else None
    tag = getattr(p, "_dta_flat", None)
    if tag is None or p.grad is not None:
        return None
    group, i = tag
    if not group.steal_ok or i not in group.direct_claimed or group.grad.dtype != p.dtype:
        return None
    return group.grad_view(i)


def _rows16(t: torch.Tensor) -> bool:
    return t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0


def _sorted_ids(ids: torch.Tensor, V: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(sorted ids, source positions) as ``torch.sort(ids, stable=True)``: one single-workgroup
    launch (``csrc/sort_ids.hip``) up to ``sort_ids_max()`` ids -- GPT-2's 8192 token ids took
    6-8 launches through torch.sort -- else torch.sort.  Ids outside [0, V) come back as V
    (the run kernel skips them either way)."""
    if ids.dtype == torch.long and ids.numel() <= native().sort_ids_max():
        sid, perm = native().sort_ids(ids.contiguous(), V)
        return sid, perm
    return torch.sort(ids, stable=True)


class _Embedding(Function):
    """``F.embedding`` whose backward is the deterministic sorted-run kernel of
    ``csrc/lm_ops.hip`` (no zero-filled dense gradient + scatter + add).  When the weight's
    gradient slice already holds another use's gradient (GPT-2's tied LM head writes there
    first), the token rows are added into it in place and autograd gets None for the
    weight: the two uses are summed without the [V, C] add, the zero fill and the DDP
    bucket copy of the sum."""

    @staticmethod
    def forward(ctx: Any, idx: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        ctx.save_for_backward(idx)
        ctx.wparam = w
        return F.embedding(idx, w)

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        (idx,) = ctx.saved_tensors
        w = ctx.wparam
        if not ctx.needs_input_grad[1]:
            return None, None
        sid, perm = _sorted_ids(idx.reshape(-1), w.shape[0])
        dy2 = dy.reshape(-1, w.shape[1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        into = _claimed_slice(w)
        if into is not None and _rows16(into):
            native().embedding_bwd_(sid, perm, dy2, into, -1)
            return None, None
        dw = _grad_dest(w)
        if dw is None or not _rows16(dw):  # (an unaligned slice stays claimed: autograd's result is copied in)
            dw = torch.zeros_like(w)
        else:
            dw.zero_()
        native().embedding_bwd_(sid, perm, dy2, dw, -1)
        return None, dw


def embedding(idx: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """Embedding lookup (the native deterministic backward on GPU for bf16 tables)."""
    if idx.is_cuda and w.dtype == torch.bfloat16 and w.shape[1] % 8 == 0 and w.stride(1) == 1 \
            and w.stride(0) % 8 == 0:
        return _Embedding.apply(idx, w)
    return F.embedding(idx, w)


class _AddPosition(Function):
    """``x + w[:S]`` for a learned absolute-position table ``w`` (GPT-2's ``wpe``): the
    positions 0..S-1 are the table's first S rows, so they are read as a view -- no position
    ids, no gather and, in the backward, no sort for the sorted-run embedding kernel (the
    position-id form cost ~50 us per GPT-2 step: arange, gather, a 1024-key radix sort and
    the run kernel).  The backward sums dy over the batch with one reduction written straight
    into the table's gradient slice (rows past S zeroed)."""

    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        ctx.S = x.shape[-2]
        ctx.wparam = w
        return x + w[: ctx.S]

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        dw = None
        if ctx.needs_input_grad[1]:
            w, S = ctx.wparam, ctx.S
            dw = _grad_dest(w)
            if dw is None or not dw.is_contiguous():
                dw = torch.empty_like(w)
            torch.sum(dy.reshape(-1, S, w.shape[1]), 0, out=dw[:S])
            if S < w.shape[0]:
                dw[S:].zero_()
        return (dy if ctx.needs_input_grad[0] else None), dw


def add_position(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``x [..., S, C] + w[:S]``: learned absolute positions added without position ids
    (the GPU path writes the table's gradient in place, ``_AddPosition``)."""
    if x.is_cuda and w.is_cuda:
        return _AddPosition.apply(x, w)
    return x + w[: x.shape[-2]]


# ------------------------------------------------------------------ loss
def _ce_mean(loss_rows: torch.Tensor, target: torch.Tensor, ignore_index: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(mean loss, count) with count = max(1, #(target != ignore_index)): f32 device scalars from ONE
    launch (``csrc/lm_ops.hip`` ce_mean_kernel) -- no host sync, and none of the 7-9 small torch
    launches of compare / sum / clamp / cast / sum / divide."""
    loss, count = native().ce_mean(loss_rows, target.reshape(-1), ignore_index)
    return loss, count


class _CrossEntropy(Function):
    @staticmethod
    def forward(ctx: Any, logits: torch.Tensor, target: torch.Tensor, ignore_index: int) -> torch.Tensor:
        # no host sync: the valid-token count stays on the device
        dlogits = torch.empty_like(logits)
        loss_rows = native().cross_entropy_fwd_bwd(logits, dlogits, target, 1.0, ignore_index, -1)
        loss, count = _ce_mean(loss_rows, target, ignore_index)
        ctx.save_for_backward(dlogits, count)
        return loss

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        dlogits, count = ctx.saved_tensors
        return dlogits * (g / count).to(dlogits.dtype), None, None


class _LinearCrossEntropy(Function):
    """loss = CE(x W^T, target) with the logits never leaving this op: the
    fused CE kernel overwrites the logits buffer with the (unscaled) logit
    gradient in the same pass that computes the loss, and backward folds
    grad/count into the two small GEMM outputs -- no separate dlogits tensor
    (N x V bf16: 0.8 GB at GPT-2 B=8, 2.1 GB at Llama-3 S=8192), no scaling
    pass over it."""

    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, w: torch.Tensor, target: torch.Tensor, ignore_index: int) -> torch.Tensor:
        x2 = x.reshape(-1, x.shape[-1])
        logits = gemm(x2, w, kind="head_fwd")
        loss_rows = native().cross_entropy_fwd_bwd(logits, logits, target, 1.0, ignore_index, -1)
        loss, count = _ce_mean(loss_rows, target, ignore_index)
        ctx.save_for_backward(x2, w, logits, count)
        ctx.xshape = x.shape
        ctx.wparam = w  # (its gradient may go straight into a flat gradient slice: _grad_dest)
        return loss

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        x2, w, dlogits, count = ctx.saved_tensors
        # grad / count stays on the device (no host sync in backward); it scales the two GEMM products in
        # the hand-written kernels' epilogues (no extra pass: 0.36 ms per Llama step for the [V, C] weight
        # gradient), after the library GEMM otherwise
        s = (g.float() / count).reshape(1)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = gemm(dlogits, w, False, True, kind="head_dgrad", scale_dev=s).view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            dw = gemm(dlogits, x2, True, True, kind="head_wgrad", out=_grad_dest(ctx.wparam), scale_dev=s)
        return dx, dw, None, None


class _ChunkedLinearCrossEntropy(Function):
    """The LM head + CE in row blocks of ``chunk`` tokens, with both gradients formed in the
    FORWARD: per block, the head GEMM writes the block's logits into one reused [chunk, V]
    buffer, the CE kernel turns them into the (unscaled) logit gradient in place, and the
    input-gradient GEMM (rows of dX) and the weight-gradient GEMM (accumulated over the
    blocks, hipBLASLt beta = 1 after the first) consume it before the next block overwrites
    it.  No [T, V] tensor exists at any time: peak memory drops by (T - chunk) x V x 2 B where
    the weight gradient goes straight into the engine's final gradient slice from the forward on
    (DDP after zero_grad(set_to_none), FSDP at one rank: ``_dta_gdest_fwd``); elsewhere the op
    holds a [V, C] buffer of its own from forward to backward.
    Backward only scales: dX and dW by grad / count (device scalars, no host sync), dW
    written straight into the engine's gradient slice when it may be (:func:`_grad_dest`).
    Same GEMM count as :class:`_LinearCrossEntropy`; what it costs is the block GEMMs'
    efficiency (narrower input-gradient outputs, a bf16 read-modify-write of dW per block).
    Reference: the loss of ``/root/reference/src/distributed_trainer.py:163`` (F.cross_entropy)."""

    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, w: torch.Tensor, target: torch.Tensor, ignore_index: int,
                chunk: int, grad: bool) -> torch.Tensor:
        x2 = x.reshape(-1, x.shape[-1])
        T, V = x2.shape[0], w.shape[0]
        # grad: autograd records this call (needs_input_grad is set from requires_grad even under no_grad --
        # an evaluation forward must neither compute nor write gradients, least of all into an engine's slice)
        need_dx, need_dw = grad and ctx.needs_input_grad[0], grad and ctx.needs_input_grad[1]
        loss_rows = torch.empty(T, dtype=torch.float32, device=x.device)
        buf = torch.empty(min(chunk, T), V, dtype=x.dtype, device=x.device)
        dx = torch.empty_like(x2) if need_dx else None
        dw, dw_final = None, False
        if need_dw:
            # the weight gradient straight into the engine's gradient slice when it is final already in
            # the forward (DDP after zero_grad(set_to_none); FSDP at one rank): no [V, C] buffer of its own
            gd = getattr(w, "_dta_gdest", None)
            f = getattr(w, "_dta_gdest_fwd", None) or getattr(gd, "forward_dest", None)
            dw = f() if f is not None else (_grad_dest(w) if gd is None else None)
            dw_final = dw is not None
            if dw is None:
                dw = torch.empty_like(w)
        C = native()
        # (several blocks: dW accumulates in bf16 -- hipBLASLt's beta = 1 adds each block's fp32 product to the
        # running sum and rounds once per block, so the result carries up to T / chunk bf16 roundings instead of
        # one.  An fp32 [V, C] running sum would round once but costs 4 V C bytes -- at Llama-3 8B as much as the
        # logits the row blocks save; the drift is bounded by test_chunked_head_ce_dw_drift_many_blocks.)
        for i, r0 in enumerate(range(0, T, chunk)):
            r1 = min(T, r0 + chunk)
            lg = buf[:r1 - r0]
            xc = x2[r0:r1]
            gemm(xc, w, kind="head_fwd", out=lg)
            loss_rows[r0:r1] = C.cross_entropy_fwd_bwd(lg, lg, target[r0:r1], 1.0, ignore_index, -1)
            if need_dx:
                gemm(lg, w, False, True, kind="head_dgrad", out=dx[r0:r1])
            if need_dw:
                if i == 0:
                    gemm(lg, xc, True, True, kind="head_wgrad", out=dw)
                else:
                    dw.addmm_(lg.t(), xc)
        del buf
        loss, count = _ce_mean(loss_rows, target, ignore_index)
        ctx.count = count
        ctx.dx, ctx.dw = dx, dw  # (this op's own results, not inputs or outputs: plain attributes)
        ctx.dw_final = dw_final
        ctx.xshape = x.shape
        ctx.wparam = w
        return loss

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor) -> Tuple[Optional[torch.Tensor], ...]:
        if getattr(ctx, "consumed", False):
            # the gradients were formed in the forward and handed over by the first backward
            raise RuntimeError("the chunked LM head + CE (head_ce_chunk) supports one backward per forward "
                               "(retain_graph=True and a second backward are not supported)")
        ctx.consumed = True
        s = (g.float() / ctx.count).reshape(())
        dx, dw = ctx.dx, ctx.dw
        ctx.dx = ctx.dw = None
        if dx is not None:
            dx = dx.mul_(s).view(ctx.xshape)
        if dw is not None:
            dest = None if ctx.dw_final else _grad_dest(ctx.wparam)
            dw = torch.mul(dw, s, out=dest) if dest is not None else dw.mul_(s)
        return dx, dw, None, None, None, None


HEAD_CE_CHUNK = int(os.environ.get("DTA_HEAD_CE_CHUNK", "0"))


def set_head_ce_chunk(rows: int) -> None:
    """Row-block size of the LM head + CE (:class:`_ChunkedLinearCrossEntropy`); 0 = one block
    holding the whole [T, V] logits (:class:`_LinearCrossEntropy`).  ``train.head_ce_chunk``."""
    global HEAD_CE_CHUNK
    HEAD_CE_CHUNK = max(0, int(rows))


def linear_cross_entropy(x: torch.Tensor, w: torch.Tensor, target: torch.Tensor, ignore_index: int = -100,
                         chunk: Optional[int] = None) -> torch.Tensor:
    """Mean token cross-entropy of ``x @ w.T`` against ``target`` (the LM head + loss).  ``chunk``
    (default :data:`HEAD_CE_CHUNK`): row blocks that never hold the [T, V] logits, see
    :class:`_ChunkedLinearCrossEntropy`."""
    if x.is_cuda:
        _need_bf16(x, w)
        chunk = HEAD_CE_CHUNK if chunk is None else chunk
        t = target.reshape(-1).contiguous()
        if chunk and chunk % 8 == 0 and t.numel() > chunk:
            return _ChunkedLinearCrossEntropy.apply(x, w, t, ignore_index, int(chunk), torch.is_grad_enabled())
        return _LinearCrossEntropy.apply(x, w, t, ignore_index)
    logits = F.linear(x, w).reshape(-1, w.shape[0])
    return F.cross_entropy(logits.float(), target.reshape(-1), ignore_index=ignore_index)


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Mean token cross-entropy over ``logits [N, V]`` (fused fwd+bwd kernel on GPU)."""
    if logits.is_cuda:
        _need_bf16(logits)
        return _CrossEntropy.apply(logits.contiguous(), target.contiguous(), ignore_index)
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index)
