#!/bin/bash
# Embedding backward under DDP and FSDP (tests), GPT-2 FSDP / DDP step times.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lm_ops_gpu.py -k "embedding" -x -v --timeout 120 --timeout-method thread > gpurun_out/emb_tests2.log 2>&1 || { tail -40 gpurun_out/emb_tests2.log; exit 1; }
tail -2 gpurun_out/emb_tests2.log
: > gpurun_out/emb_ab2.jsonl
for s in fsdp ddp fsdp; do
  timeout -k 10 300 python bench_lm.py --model gpt2 --strategy $s >> gpurun_out/emb_ab2.jsonl 2>/dev/null
done
python - <<'PY'
import json
for l in open("gpurun_out/emb_ab2.jsonl"):
    d = json.loads(l); print(d["metric"], d["ms_per_step"], d["value"], d["final_loss"])
PY
