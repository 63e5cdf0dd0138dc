#!/bin/bash
# FSDP claim fix + native embedding under FSDP: tests, then GPT-2 FSDP / DDP step times.
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lm_ops_gpu.py tests/test_ipc_gpu.py -k "embedding or first_claim or engines or offload" -x -v --timeout 120 --timeout-method thread > gpurun_out/emb_fsdp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/emb_fsdp_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/emb_fsdp_tests.log | head -20; exit 1; }
: > gpurun_out/emb_fsdp_ab.txt
for i in 1 2; do for s in fsdp ddp; do
  timeout -k 10 300 python bench_lm.py --model gpt2 --strategy $s --json-out /tmp/r.json > /dev/null 2> gpurun_out/emb_fsdp_bench.err || { tail -20 gpurun_out/emb_fsdp_bench.err; exit 1; }
  python -c "import json; d=json.load(open('/tmp/r.json')); print('$s', d['ms_per_step'], d['final_loss'])" >> gpurun_out/emb_fsdp_ab.txt
done; done
cat gpurun_out/emb_fsdp_ab.txt
