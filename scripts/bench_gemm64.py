#!/usr/bin/env python3
"""csrc/gemm_k64.hip (64-deep stages, phase-interleaved half-tile DMA; tiles 9 / 10 = csrc/gemm_w4.hip)
vs torch (hipBLASLt) on the GPT-2 small / Llama-3 8B
projection shapes -- forward (x W^T), input gradient (dy W), weight gradient
(dy^T x) -- plus the FUSED costs the dispatcher compares: c_fc forward with the
GELU dual store vs hipBLASLt + gelu_fwd, and the GELU-backward dgrad vs hipBLASLt +
gelu_bwd.  Random N(0,1) bf16 operands (zeros inflate the clock: DVFS).  Candidates
are timed in interleaved rounds in ONE process (cdna_hip_programming.md rule 24);
the median per candidate is reported.  One JSON line per (shape, kind).

    python scripts/bench_gemm64.py [gpt2,llama] [rounds]
"""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

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
    C = native()
    for model in models:
        for name, nout, nin in MODELS[model]:
            x = torch.randn(T, nin, device="cuda").bfloat16()
            w = (torch.randn(nout, nin, device="cuda") * 0.02).bfloat16()
            dy = torch.randn(T, nout, device="cuda").bfloat16()
            bias = (torch.randn(nout, device="cuda") * 0.1).bfloat16()
            fl = 2.0 * T * nout * nin
            cases = {
                "fwd": ((T, nout, nin), lambda: F.linear(x, w), lambda t: C.gemm64(x, w, tile=t)[0]),
                "dgrad": ((T, nin, nout), lambda: torch.mm(dy, w), lambda t: C.gemm64(dy, w, False, True, tile=t)[0]),
                "wgrad": ((nout, nin, T), lambda: torch.mm(dy.t(), x), lambda t: C.gemm64(dy, x, True, True, tile=t)[0]),
            }
            for kind, ((M, N, K), tfn, new) in cases.items():
                ref = tfn()
                fns = {"torch": tfn}
                errs = {}
                for t in range(1, 11):  # 5-8: tiles 1-4 with the two-phase K loop; 9 / 10: csrc/gemm_w4.hip
                    if C.gemm64_tile(M, N, K, t):
                        fns[f"k64_t{t}"] = (lambda t=t: new(t))
                        errs[f"k64_t{t}"] = float(f"{relerr(new(t), ref):.2e}")
                times = bench(fns, rounds)
                best = min((k for k in times if k.startswith("k64")), key=times.get, default=None)
                row = {"model": model, "gemm": name, "kind": kind, "M": M, "N": N, "K": K,
                       "us": {k: round(v, 1) for k, v in times.items()},
                       "TF": {k: round(fl / v / 1e6) for k, v in times.items()},
                       "k64_auto": C.gemm64_tile(M, N, K, 0), "k64_best": best,
                       "torch_over_k64": round(times["torch"] / times[best], 3) if best else None,
                       "relerr": errs}
                print(json.dumps(row), flush=True)
                del ref
            # fused costs the dispatcher compares (GPT-2 MLP): c_fc + GELU dual store, dgrad through GELU
            if model == "gpt2" and name == "fc":
                h = torch.empty(T, nout, dtype=torch.bfloat16, device="cuda")
                a = torch.empty_like(h)

                def lib_fwd():
                    hh = torch.addmm(bias, x, w.t())
                    return hh, C.gelu_fwd(hh, -1)

                fns = {"torch+gelu_fwd": lib_fwd}
                for t in range(1, 9):
                    if C.gemm64_tile(T, nout, nin, t):
                        fns[f"k64_t{t}_dual"] = (lambda t=t: C.gemm64(x, w, bias=bias, epi=2, out=h, out2=a, tile=t))
                times = bench(fns, rounds)
                print(json.dumps({"model": model, "gemm": "fc+gelu", "kind": "fwd_fused", "M": T, "N": nout, "K": nin,
                                  "us": {k: round(v, 1) for k, v in times.items()}}), flush=True)
                w2 = (torch.randn(nin, nout, device="cuda") * 0.02).bfloat16()  # c_proj weight [768, 3072]
                dy2 = torch.randn(T, nin, device="cuda").bfloat16()
                fns = {"torch+gelu_bwd": lambda: C.gelu_bwd(torch.mm(dy2, w2), h, -1)}
                for t in range(1, 9):
                    if C.gemm64_tile(T, nout, nin, t):
                        fns[f"k64_t{t}_dgelu"] = (lambda t=t: C.gemm64(dy2, w2, False, True, epi=16, res=h, tile=t))
                times = bench(fns, rounds)
                print(json.dumps({"model": model, "gemm": "fc2_dgrad+dgelu", "kind": "dgrad_fused", "M": T,
                                  "N": nout, "K": nin, "us": {k: round(v, 1) for k, v in times.items()}}), flush=True)


if __name__ == "__main__":
    main()
