#!/usr/bin/env python3
"""Flash-attention microbenchmark: this framework's gfx950 kernels vs torch SDPA
at the GPT-2 small and Llama-3 8B shapes.  Causal FLOPs counted as the
unmasked half (fwd 2*B*H*S^2*D, bwd 2.5x that)."""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch
import torch.nn.functional as F

from distributed_training_amd.ops import native

SHAPES = {
    "gpt2": (8, 1024, 12, 12, 64),
    "llama8b": (1, 8192, 32, 8, 128),
    "llama8b_s2k": (4, 2048, 32, 8, 128),
}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    names = sys.argv[1:] or list(SHAPES)
    dev = torch.device("cuda", 0)
    C = native()
    for name in names:
        B, S, H, Hkv, D = SHAPES[name]
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
        k = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16, generator=g)
        v = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16, generator=g)
        do = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
        sc = D ** -0.5
        o, lse = C.attn_fwd(q, k, v, True, sc, -1)
        t_fwd = timeit(lambda: C.attn_fwd(q, k, v, True, sc, -1))
        t_bwd = timeit(lambda: C.attn_bwd(do, q, k, v, o, lse, True, sc, -1))
        # the forward's workgroup forms (csrc/attention.hip fwd_waves: 4 / 8 waves)
        fwd_var, fwd_var_err = {}, {}
        for wv in ("4", "8"):
            os.environ["DTA_ATTN_FWD_WAVES"] = wv
            fwd_var[wv] = round(timeit(lambda: C.attn_fwd(q, k, v, True, sc, -1)) * 1e6, 1)
            ov, lv = C.attn_fwd(q, k, v, True, sc, -1)
            fwd_var_err[wv] = [(ov.float() - o.float()).abs().max().item(), (lv - lse).abs().max().item()]
        os.environ.pop("DTA_ATTN_FWD_WAVES", None)
        fl = 2.0 * B * H * S * S * D  # causal fwd (4*S^2*D/2)
        # torch SDPA reference (expects [B, H, S, D]; GQA expanded)
        rep = H // Hkv
        qt = q.transpose(1, 2).detach().requires_grad_()
        kt = k.repeat_interleave(rep, dim=2).transpose(1, 2).detach().requires_grad_()
        vt = v.repeat_interleave(rep, dim=2).transpose(1, 2).detach().requires_grad_()
        dot = do.transpose(1, 2)
        t_tf = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=True))
        ot = F.scaled_dot_product_attention(qt, kt, vt, is_causal=True)
        t_tb = timeit(lambda: torch.autograd.grad(ot, (qt, kt, vt), dot, retain_graph=True))
        # the models' path: strided q/k/v views of one packed QKV projection output
        # (row stride (H + 2 Hkv) D), RoPE applied, packed dQKV written by backward
        from distributed_training_amd.ops import lm

        qkv = torch.randn(B, S, (H + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16, generator=g)
        qkv.requires_grad_()
        cos, sin = lm.rope_tables(S, D, 500000.0, device=dev)
        t_pf = timeit(lambda: lm.attention_packed(qkv, H, Hkv, True, rope=(cos, sin)))
        op = lm.attention_packed(qkv, H, Hkv, True, rope=(cos, sin))
        t_pb = timeit(lambda: torch.autograd.grad(op, qkv, do, retain_graph=True))
        err = (o.float() - ot.detach().transpose(1, 2).float()).abs().max().item()
        print(json.dumps({"shape": name, "B": B, "S": S, "H": H, "Hkv": Hkv, "D": D,
                          "fwd_us": round(t_fwd * 1e6, 1), "bwd_us": round(t_bwd * 1e6, 1),
                          "fwd_tflops": round(fl / t_fwd / 1e12, 1), "bwd_tflops": round(2.5 * fl / t_bwd / 1e12, 1),
                          "sdpa_fwd_us": round(t_tf * 1e6, 1), "sdpa_bwd_us": round(t_tb * 1e6, 1),
                          "packed_rope_fwd_us": round(t_pf * 1e6, 1), "packed_rope_bwd_us": round(t_pb * 1e6, 1),
                          "max_abs_err_vs_sdpa": err, "fwd_variants_us": fwd_var,
                          "fwd_variants_maxdiff_o_lse": fwd_var_err}), flush=True)


if __name__ == "__main__":
    main()
