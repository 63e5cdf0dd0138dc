#!/bin/bash
# Whole-step hipGraph: GPU test, then GPT-2 DDP same-box pairs (eager vs graph replay).
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lm_ops_gpu.py -k "graphed" -x -v --timeout 120 --timeout-method thread > gpurun_out/graph_tests.log 2>&1; rc=$?; tail -3 gpurun_out/graph_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error" gpurun_out/graph_tests.log | head -20; exit 1; }
: > gpurun_out/graph_ab.txt
for i in 1 2 3; do for v in "--no-graph" ""; do
  timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp $v --json-out /tmp/r.json > /dev/null 2> gpurun_out/graph_bench.err || { tail -20 gpurun_out/graph_bench.err; exit 1; }
  python -c "import json; d=json.load(open('/tmp/r.json')); print(d['step_graph'], d['ms_per_step'], d['final_loss'])" >> gpurun_out/graph_ab.txt
done; done
cat gpurun_out/graph_ab.txt
