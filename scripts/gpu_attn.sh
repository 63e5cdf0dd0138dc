#!/bin/bash
# Attention kernels on the GPU box: numerics tests, then the microbenchmark.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lm_ops_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_lm.log 2>&1
timeout -k 10 200 python scripts/bench_attn.py > gpurun_out/attn.jsonl 2> gpurun_out/attn.err
cat gpurun_out/attn.jsonl
