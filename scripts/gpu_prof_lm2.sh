#!/bin/bash
# Kernel profiles of the GPT-2 FSDP step and the Llama-3 8B FSDP step without activation checkpointing (1 GPU).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/prof_gpt2_fsdp gpurun_out/prof_llama_nockpt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2_fsdp -o run -- \
  python3 bench_lm.py --model gpt2 --strategy fsdp --steps 10 --warmup 3 > gpurun_out/prof_gpt2_fsdp/bench.log 2>&1
python scripts/kstats.py gpurun_out/prof_gpt2_fsdp/run_kernel_stats.csv 13 30 > gpurun_out/prof_gpt2_fsdp/summary.txt
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama_nockpt -o run -- \
  python3 bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 2 --warmup 1 > gpurun_out/prof_llama_nockpt/bench.log 2>&1
python scripts/kstats.py gpurun_out/prof_llama_nockpt/run_kernel_stats.csv 3 30 > gpurun_out/prof_llama_nockpt/summary.txt
