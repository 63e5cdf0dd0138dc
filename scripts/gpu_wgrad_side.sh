#!/bin/bash
# GPT-2 DDP step with the weight gradients on side streams (DTA_WGRAD_STREAM=tile:split, DTA_WGRAD_STREAMS=n) vs the main stream.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp DTA_GEMM_CACHE=/tmp/gemm_cache.json
mkdir -p gpurun_out
: > gpurun_out/wgrad_side.jsonl
for cfg in 1:2/1 1:3/1 1:3/2 1:2/3 0:2/1 1:2/2 1:6/1 0:4/1; do
  v=${cfg%/*}; n=${cfg#*/}
  DTA_WGRAD_STREAM=$v DTA_WGRAD_STREAMS=$n timeout -k 10 200 python bench_lm.py --model gpt2 --strategy ddp --steps 20 --warmup 5 > gpurun_out/ws.out 2> gpurun_out/ws.err
  echo "{\"DTA_WGRAD_STREAM\": \"$v\", \"streams\": $n, \"ms\": $(grep '^{' gpurun_out/ws.out | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')}" | tee -a gpurun_out/wgrad_side.jsonl
done
