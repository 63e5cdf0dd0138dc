#!/bin/bash
# Native embedding backward (tests + GPT-2 DDP step) and the AdamW bandwidth probe.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lm_ops_gpu.py -k "embedding or deferred or in_backward" -x -v --timeout 120 --timeout-method thread > gpurun_out/emb_tests.log 2>&1 || { tail -40 gpurun_out/emb_tests.log; exit 1; }
tail -2 gpurun_out/emb_tests.log
: > gpurun_out/emb_ab.jsonl
for i in 1 2; do
  timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp >> gpurun_out/emb_ab.jsonl 2>/dev/null
done
cut -c1-200 gpurun_out/emb_ab.jsonl
timeout -k 10 120 python scripts/bw_probe.py
