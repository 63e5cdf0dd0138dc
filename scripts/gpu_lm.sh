#!/bin/bash
# LM benchmarks on one GPU (GPU box): GPT-2 small DDP + FSDP, Llama-3 8B FSDP, plus a kernel profile of GPT-2 DDP.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/prof_gpt2
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp > gpurun_out/lm_gpt2_ddp.json 2> gpurun_out/lm_gpt2_ddp.err
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy fsdp > gpurun_out/lm_gpt2_fsdp.json 2> gpurun_out/lm_gpt2_fsdp.err
cat gpurun_out/lm_gpt2_*.json
timeout -k 10 400 python bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --ckpt --steps 4 --warmup 2 \
  > gpurun_out/lm_llama8b_fsdp.json 2> gpurun_out/lm_llama8b_fsdp.err
cat gpurun_out/lm_llama8b_fsdp.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- \
  python3 bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 > gpurun_out/prof_gpt2/bench.log 2>&1
python scripts/kstats.py gpurun_out/prof_gpt2/run_kernel_stats.csv 13 30 > gpurun_out/prof_gpt2/summary.txt
timeout -k 10 300 python -u -m pytest tests/test_lm_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lm2.log 2>&1
