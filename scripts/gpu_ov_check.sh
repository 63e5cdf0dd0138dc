#!/bin/bash
# Optimizer-in-backward: GPU tests, then GPT-2 DDP A/B pairs (per-bucket update inside the backward vs step() after it).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_lm_ops_gpu.py tests/test_ipc_gpu.py -k "in_backward or deferred or engines_multi_rank_shared_gpu and ddp" -x -v --timeout 120 --timeout-method thread > gpurun_out/ov_tests.log 2>&1 || { tail -40 gpurun_out/ov_tests.log; exit 1; }
tail -3 gpurun_out/ov_tests.log
: > gpurun_out/ov_ab.jsonl
for i in 1 2; do
  timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp >> gpurun_out/ov_ab.jsonl 2>/dev/null
  timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --overlap-opt >> gpurun_out/ov_ab.jsonl 2>/dev/null
done
python - <<'PY'
import json
for l in open("gpurun_out/ov_ab.jsonl"):
    d = json.loads(l); print(d["optimizer_in_backward"], d["ms_per_step"], d["value"], d["final_loss"])
PY
