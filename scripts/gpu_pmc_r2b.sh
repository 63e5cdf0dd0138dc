#!/bin/bash
# MFMA-busy PMC pass of the current GPT-2 DDP step (eager kernels: --no-graph so every dispatch is attributed),
# then the Llama-3 8B FSDP bench (1 x 8192, no activation checkpointing).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/pmc_gpt2b
export DTA_GEMM_CACHE=$PWD/gpurun_out/gemm_cache.json
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --no-graph --steps 2 --warmup 1 > /dev/null 2>&1
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_gpt2b -o run -- python3 bench_lm.py --model gpt2 --strategy ddp --no-graph --steps 3 --warmup 1 > gpurun_out/pmc_gpt2b/bench.log 2>&1
f=$(find gpurun_out/pmc_gpt2b -name "*counter_collection.csv" | head -n1)
python scripts/pmc_summary.py "$f" > gpurun_out/pmc_gpt2b/summary.txt
head -25 gpurun_out/pmc_gpt2b/summary.txt
timeout -k 10 600 python bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 4 --warmup 2 > gpurun_out/llama.json 2> gpurun_out/llama.err
cut -c1-400 gpurun_out/llama.json
