#!/bin/bash
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lm_ops_gpu.py tests/test_ipc_gpu.py tests/test_engine_gpu.py tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fsdp.log 2>&1 || { tail -60 gpurun_out/pytest_fsdp.log; exit 1; }
tail -2 gpurun_out/pytest_fsdp.log
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy fsdp > gpurun_out/lm_gpt2_fsdp.json 2> gpurun_out/lm_gpt2_fsdp.err
cut -c1-300 gpurun_out/lm_gpt2_fsdp.json
timeout -k 10 400 python bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 3 --warmup 2 > gpurun_out/lm_llama.json 2> gpurun_out/lm_llama.err
cut -c1-300 gpurun_out/lm_llama.json
DTA_PROFILE_OPS=1 timeout -k 10 300 python bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --layers 4 --steps 2 --warmup 1 > gpurun_out/llama_ops.json 2> gpurun_out/llama_ops.txt
grep -E "cat|copy_|Memcpy|SplitInto" gpurun_out/llama_ops.txt | cut -c1-60,120-200 || true
