#!/bin/bash
# Attention kernels on the GPU box: numerics tests, the microbenchmark, per-kernel times.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/prof_attn
timeout -k 10 300 python -u -m pytest tests/test_lm_ops_gpu.py -x -v --timeout 120 --timeout-method thread -k "attention" > gpurun_out/pytest_lm.log 2>&1
timeout -k 10 200 python scripts/bench_attn.py > gpurun_out/attn.jsonl 2> gpurun_out/attn.err
cat gpurun_out/attn.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attn -o run -- python3 scripts/bench_attn.py > gpurun_out/prof_attn/log 2>&1
python scripts/kstats.py gpurun_out/prof_attn/run_kernel_stats.csv 1 12
