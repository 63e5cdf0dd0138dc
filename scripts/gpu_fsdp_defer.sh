#!/bin/bash
# FSDP with deferred grouped weight gradients: FSDP GPU tests, then GPT-2 FSDP same-box A/B (deferral off / on).
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
: timeout -k 10 600 python -u -m pytest tests/test_ipc_gpu.py tests/test_lm_ops_gpu.py tests/test_engine_gpu.py -k "fsdp or engines or deferred or embedding" -x -v --timeout 120 --timeout-method thread > gpurun_out/fsdp_defer_tests.log 2>&1
: > gpurun_out/fsdp_ab.txt
for i in 1 2 3; do for g in 0 200; do
  DTA_WGRAD_GROUP=$g timeout -k 10 300 python bench_lm.py --model gpt2 --strategy fsdp --json-out /tmp/r.json > /dev/null 2> gpurun_out/fsdp_bench.err || { tail -20 gpurun_out/fsdp_bench.err; exit 1; }
  python -c "import json; d=json.load(open('/tmp/r.json')); print('group=$g', d['ms_per_step'], d['final_loss'])" >> gpurun_out/fsdp_ab.txt
done; done
cat gpurun_out/fsdp_ab.txt
