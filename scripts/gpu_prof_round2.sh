#!/bin/bash
# Kernel statistics + MFMA-busy PMC pass of the GPT-2 DDP step and the Llama-3 8B FSDP step (4 layers).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/prof_gpt2 gpurun_out/pmc_gpt2 gpurun_out/prof_llama
# tune the GEMM dispatch once (unprofiled) so the profiles below contain no timing calls
export DTA_GEMM_CACHE=$PWD/gpurun_out/gemm_cache.json
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --steps 2 --warmup 1 > /dev/null 2>&1
timeout -k 10 400 python bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 1 --warmup 1 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- python3 bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 > gpurun_out/prof_gpt2/bench.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_gpt2 -o run -- python3 bench_lm.py --model gpt2 --strategy ddp --steps 3 --warmup 1 > gpurun_out/pmc_gpt2/bench.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama -o run -- python3 bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 2 --warmup 1 > gpurun_out/prof_llama/bench.log 2>&1
ls gpurun_out/prof_gpt2 gpurun_out/pmc_gpt2 gpurun_out/prof_llama
