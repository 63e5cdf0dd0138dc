#!/bin/bash
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_lm_ops_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1 || { tail -40 gpurun_out/pytest_gemm.log; exit 1; }
tail -2 gpurun_out/pytest_gemm.log
for m in auto torch; do
  DTA_GEMM=$m timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp > gpurun_out/lm_gpt2_ddp_$m.json 2> gpurun_out/lm_gpt2_ddp_$m.err
  cut -c1-400 gpurun_out/lm_gpt2_ddp_$m.json
done
if [ "${LLAMA:-1}" = "1" ]; then
for m in auto torch; do
  DTA_GEMM=$m timeout -k 10 400 python bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 3 --warmup 2 > gpurun_out/lm_llama_$m.json 2> gpurun_out/lm_llama_$m.err
  cut -c1-400 gpurun_out/lm_llama_$m.json
done
fi
