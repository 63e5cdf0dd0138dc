#!/bin/bash
# Kernel profile of the Llama-3 8B FSDP step (1 GPU, seq 8192, activation checkpointing).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/prof_llama
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama -o run -- \
  python3 bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --ckpt --steps 2 --warmup 1 > gpurun_out/prof_llama/bench.log 2>&1
python scripts/kstats.py gpurun_out/prof_llama/run_kernel_stats.csv 3 40 > gpurun_out/prof_llama/summary.txt
