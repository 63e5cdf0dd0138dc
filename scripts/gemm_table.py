"""Measure the tracked GEMM table (distributed_training_amd/ops/gemm_table_mi355x.json) on an idle MI355X.

1. The (kind, M, N, K) keys: one forward + backward of a 1-layer GPT-2 small (8 x 1024 tokens) and a
   1-layer Llama-3 8B (8192 tokens) in bf16 with DTA_GEMM=torch (every GEMM call site records its key;
   a layer's shapes repeat in every layer).
2. Every key: operands of its kind (random, full-range bf16), every candidate -- hipBLASLt (+ its separate
   epilogue kernels) and each hand-written tile that covers the shape, as the SAME fused op -- timed by
   ops/lm.py ``_pick`` itself (interleaved rounds, median; DTA_GEMM_ROUNDS, default here 15), table off.
3. The fastest median wins (the GELU dual store keeps its 15 % handicap, see gemm_gelu_dual).

    python scripts/gemm_table.py --out distributed_training_amd/ops/gemm_table_mi355x.json
    python scripts/gemm_table.py --check distributed_training_amd/ops/gemm_table_mi355x.json   # re-measure, compare
    python scripts/gemm_table.py --only dswiglu --merge distributed_training_amd/ops/gemm_table_mi355x.json --out F
        # measure only these kinds; the other entries copied from the --merge table

``--check`` re-measures and reports, per key, whether this box picks the same implementation and the
hand-written / library ratio (the cross-box determinism check of verdict r4 item 1).
"""
import argparse
import datetime
import json
import os
import sys

os.environ.setdefault("DTA_GEMM_ROUNDS", "15")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_training_amd.ops import lm  # noqa: E402

DEV = torch.device("cuda")


def _r(*shape, scale=1.0):
    return ((torch.rand(*shape, device=DEV) * 2 - 1) * scale).to(torch.bfloat16)


def collect_keys(gpt2_batches=(8,)):
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.models.llama import Llama, LlamaConfig

    os.environ["DTA_GEMM"] = "torch"
    keys = set()
    runs = [(lambda: GPT2(GPT2Config(n_layer=1)), b, 1024) for b in gpt2_batches]
    runs.append((lambda: Llama(LlamaConfig(n_layer=1)), 1, 8192))
    for build, B, S in runs:
        torch.manual_seed(0)
        m = build().to(DEV).to(torch.bfloat16)
        idx = torch.randint(0, m.vocab_size, (B, S + 1), device=DEV)
        lm._GEMM_CHOICE.clear()
        loss = m(idx[:, :-1], idx[:, 1:])
        loss.backward()
        torch.cuda.synchronize()
        keys |= set(lm._GEMM_CHOICE)
        del m, loss
        torch.cuda.empty_cache()
    os.environ["DTA_GEMM"] = "auto"
    lm._GEMM_CHOICE.clear()
    return sorted(keys)


def probe(kind, M, N, K):
    """Run the op of ``kind`` once on fresh operands (its _pick call times every candidate)."""
    head = kind.startswith("head_")
    s = torch.full((1,), 1.0 / 8192, device=DEV) if head else None
    if kind in ("fwd", "fwdb", "head_fwd"):
        lm.gemm(_r(M, K), _r(N, K, scale=0.02), bias=_r(N) if kind == "fwdb" else None,
                kind="head_fwd" if head else "fwd")
    elif kind in ("dgrad", "head_dgrad"):
        lm.gemm(_r(M, K), _r(K, N, scale=0.02), False, True, kind=kind, scale_dev=s)
    elif kind in ("wgrad", "head_wgrad"):
        lm.gemm(_r(K, M), _r(K, N), True, True, kind=kind, out=torch.empty(M, N, device=DEV, dtype=torch.bfloat16),
                scale_dev=s)
    elif kind in ("fwd_gelu", "fwd_gelub"):
        lm.gemm_gelu_dual(_r(M, K), _r(N, K, scale=0.02), _r(N) if kind == "fwd_gelub" else None)
    elif kind == "dgelu":
        lm._dgelu_dgrad(_r(M, K), _r(K, N, scale=0.02), _r(M, N))
    elif kind == "dswiglu":
        lm._swiglu_dgrad(_r(M, K), _r(K, N, scale=0.02), _r(M, 2 * N, scale=2.0))
    else:
        raise ValueError(f"unknown GEMM kind {kind}")
    torch.cuda.synchronize()


def measure(keys):
    os.environ["DTA_GEMM_TABLE"] = "0"
    os.environ["DTA_GEMM"] = "auto"
    out = {}
    for key in keys:
        kind, M, N, K = key
        lm._GEMM_CHOICE.pop(key, None)
        probe(kind, M, N, K)
        pick = lm._GEMM_CHOICE[key]
        times = lm.GEMM_TIMES.get(key, {})
        lib = times.get(0)
        best_dta = min((v for k, v in times.items() if k != 0), default=None)
        ent = {"pick": pick, "pick_name": lm._impl_name(pick),
               "us": {lm._impl_name(k): round(v, 1) for k, v in sorted(times.items())},
               "lib_over_best_dta": round(lib / best_dta, 3) if lib and best_dta else None}
        out[f"{kind} {M}x{N}x{K}"] = ent
        print(json.dumps({"key": f"{kind} {M}x{N}x{K}", **ent}), flush=True)
        torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--check", default="")
    ap.add_argument("--only", default="", help="comma-separated kinds to measure (default: every key)")
    ap.add_argument("--merge", default="", help="table whose entries the measured ones are added to / replace")
    ap.add_argument("--gpt2-batches", default="8", help="GPT-2 batch sizes (x 1024 tokens) whose GEMM keys to collect")
    ap.add_argument("--new-only", action="store_true", help="measure only keys missing from the --merge table")
    args = ap.parse_args()
    keys = collect_keys(tuple(int(b) for b in args.gpt2_batches.split(",")))
    if args.only:
        kinds = set(args.only.split(","))
        keys = [k for k in keys if k[0] in kinds]
    if args.new_only and args.merge:
        with open(args.merge) as f:
            have = json.load(f)["entries"]
        keys = [k for k in keys if f"{k[0]} {k[1]}x{k[2]}x{k[3]}" not in have]
    print(f"[gemm_table] {len(keys)} keys", flush=True)
    entries = measure(keys)
    if args.merge:
        with open(args.merge) as f:
            base = json.load(f)["entries"]
        for k, e in entries.items():  # same-box in-step A/B overrides stay with their key
            e.update({f: v for f, v in base.get(k, {}).items() if f.startswith("in_step_")})
        base.update(entries)
        entries = base
    props = torch.cuda.get_device_properties(0)
    doc = {"arch": props.gcnArchName, "device": props.name, "rounds": int(os.environ["DTA_GEMM_ROUNDS"]),
           "generated": datetime.datetime.utcnow().strftime("%Y-%m-%d %H:%M UTC"), "script": "scripts/gemm_table.py",
           "entries": entries}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(doc, f, indent=1, sort_keys=True)
        print(f"[gemm_table] wrote {args.out}", flush=True)
    if args.check:
        with open(args.check) as f:
            ref = json.load(f)["entries"]
        same = [k for k in entries if k in ref and ref[k]["pick"] == entries[k]["pick"]]
        diff = [k for k in entries if k in ref and ref[k]["pick"] != entries[k]["pick"]]
        print(json.dumps({"check": args.check, "keys": len(entries), "same_pick": len(same), "different_pick": diff,
                          "missing_from_table": [k for k in entries if k not in ref]}), flush=True)


if __name__ == "__main__":
    main()
