#!/bin/bash
# Kernel statistics of the GPT-2 DDP step at one rank (GEMM dispatch tuned first, unprofiled).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/prof_gpt2
export DTA_GEMM_CACHE=$PWD/gpurun_out/gemm_cache.json
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --steps 2 --warmup 1 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- python3 bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 > gpurun_out/prof_gpt2/bench.log 2>&1
f=$(ls gpurun_out/prof_gpt2/*/run_kernel_stats.csv gpurun_out/prof_gpt2/run_kernel_stats.csv 2>/dev/null | head -n1 || true); python scripts/kstats.py "$f" 13 45 > gpurun_out/prof_gpt2/summary.txt 2>&1 || true
