#!/bin/bash
# Host synchronisations inside the GPT-2 DDP / FSDP steps, then kernel statistics of the DDP step.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/prof_gpt2c
export DTA_GEMM_CACHE=$PWD/gpurun_out/gemm_cache.json
DTA_SYNC_DEBUG=1 timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --steps 2 --warmup 1 > gpurun_out/sync_ddp.log 2>&1
DTA_SYNC_DEBUG=1 timeout -k 10 300 python bench_lm.py --model gpt2 --strategy fsdp --steps 2 --warmup 1 > gpurun_out/sync_fsdp.log 2>&1
grep -c "UserWarning" gpurun_out/sync_ddp.log gpurun_out/sync_fsdp.log || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2c -o run -- python3 bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 > gpurun_out/prof_gpt2c/bench.log 2>&1
python scripts/kstats.py gpurun_out/prof_gpt2c/run_kernel_stats.csv 13 45 > gpurun_out/prof_gpt2c/summary.txt
head -30 gpurun_out/prof_gpt2c/summary.txt
