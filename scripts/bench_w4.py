#!/usr/bin/env python3
"""The GEMM shapes of GPT-2 small / Llama-3 8B -- forward (x W^T, NT), input gradient (dy W, NN), weight
gradient (dy^T x, TN): csrc/gemm_w4.hip (tile 9: 4 waves, 256 x 256, intra-wave read / MFMA overlap) vs
the best csrc/gemm_k64.hip tile vs torch (hipBLASLt).  Random N(0,1) bf16 operands, candidates timed in
interleaved rounds in ONE process (cdna_hip_programming.md rule 24), median per candidate; max relative
error of each kernel vs hipBLASLt.  One JSON line per (shape, kind).

    python scripts/bench_w4.py [gpt2,llama] [rounds] [tiles=5,6,7,8,3] [kinds=fwd,dgrad,wgrad]
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_training_amd.ops import native  # noqa: E402

T = 8192
MODELS = {
    "gpt2": [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072), ("head", 50304, 768)],
    "llama": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
              ("head", 128256, 4096)],
}


def bench(fns, rounds=5, reps=8):
    for fn in fns.values():
        fn()
        fn()
    torch.cuda.synchronize()
    res = {k: [] for k in fns}
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


def relerr(got, ref):
    return (got.float() - ref.float()).abs().max().item() / max(ref.float().abs().max().item(), 1e-6)


def main():
    models = sys.argv[1].split(",") if len(sys.argv) > 1 else ["gpt2", "llama"]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    tiles = [int(t) for t in sys.argv[3].split(",")] if len(sys.argv) > 3 else [5, 6, 7, 8, 3]
    kinds = sys.argv[4].split(",") if len(sys.argv) > 4 else ["fwd", "dgrad", "wgrad"]
    C = native()
    for model in models:
        for name, nout, nin in MODELS[model]:
            x = torch.randn(T, nin, device="cuda").bfloat16()
            w = (torch.randn(nout, nin, device="cuda") * 0.02).bfloat16()
            dy = torch.randn(T, nout, device="cuda").bfloat16()
            for kind in kinds:
                # (a, b, a_t, b_t): C = op(a) op(b)^T
                a, b, a_t, b_t = {"fwd": (x, w, False, False), "dgrad": (dy, w, False, True),
                                  "wgrad": (dy, x, True, True)}[kind]
                At = a.t() if a_t else a
                Bt = b if b_t else b.t()
                M, K = At.shape
                N = Bt.shape[1]
                ref = At @ Bt
                outs = {"torch": torch.empty_like(ref)}
                fns = {"torch": lambda: torch.mm(At, Bt, out=outs["torch"])}
                for t in tiles + [9, 10]:
                    if C.gemm64_tile(M, N, K, t):
                        outs[t] = torch.empty_like(ref)
                        fns[t] = (lambda t=t, a=a, b=b, a_t=a_t, b_t=b_t:
                                  C.gemm64(a, b, a_t, b_t, outs[t], None, False, 1.0, None, 0, None, t))
                times = bench(fns, rounds)
                for k in fns:
                    fns[k]()
                torch.cuda.synchronize()
                err = {str(k): relerr(outs[k], ref) for k in fns if k != "torch"}
                flop = 2.0 * M * N * K
                k64 = {k: v for k, v in times.items() if k not in ("torch", 9)}
                best = min(k64, key=k64.get) if k64 else None
                row = {"model": model, "gemm": name, "kind": kind, "M": M, "N": N, "K": K,
                       "torch_us": round(times["torch"], 1), "torch_tf": round(flop / times["torch"] / 1e6, 0),
                       "w4_us": round(times.get(9, float("nan")), 1),
                       "w4_tf": round(flop / times[9] / 1e6, 0) if 9 in times else None,
                       "torch_over_w4": round(times["torch"] / times[9], 3) if 9 in times else None,
                       "k64_best": best, "k64_us": round(times[best], 1) if best else None,
                       "times": {str(k): round(v, 1) for k, v in times.items()}, "max_rel_err": err}
                print(json.dumps(row), flush=True)
                del ref, outs
            del x, w, dy
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
