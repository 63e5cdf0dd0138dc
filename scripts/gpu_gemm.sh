#!/bin/bash
# Weight-gradient GEMM: numerics tests, then the stream-K / split-K timing sweep.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lm_ops_gpu.py -k "gemm_tn" > gpurun_out/pytest_gemm.log 2>&1 || { tail -30 gpurun_out/pytest_gemm.log; exit 1; }
tail -2 gpurun_out/pytest_gemm.log
timeout -k 10 300 python -u scripts/bench_gemm.py --no-linear > gpurun_out/gemm_sk.jsonl 2> gpurun_out/gemm_sk.err
cat gpurun_out/gemm_sk.jsonl
