#!/bin/bash
# LM kernel tests + GPT-2 DDP bench + kernel profile (GPU box).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/prof_gpt2
timeout -k 10 300 python -u -m pytest tests/test_lm_ops_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_lm.log 2>&1
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp > gpurun_out/lm_gpt2_ddp.json 2> gpurun_out/lm_gpt2_ddp.err
cat gpurun_out/lm_gpt2_ddp.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- \
  python3 bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 > gpurun_out/prof_gpt2/bench.log 2>&1
python scripts/kstats.py gpurun_out/prof_gpt2/run_kernel_stats.csv 13 30 > gpurun_out/prof_gpt2/summary.txt
