#!/bin/bash
# Kernel trace of the GPT-2 DDP step with the optimizer inside the backward (where the per-bucket updates run).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/ov_trace
export DTA_GEMM_CACHE=$PWD/gpurun_out/gemm_cache.json
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --steps 2 --warmup 1 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ov_trace -o run -- python3 bench_lm.py --model gpt2 --strategy ddp --overlap-opt --steps 6 --warmup 2 > gpurun_out/ov_trace/bench.log 2>&1
ls gpurun_out/ov_trace
