#!/bin/bash
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1 || { tail -40 gpurun_out/pytest_gemm.log; exit 1; }
tail -2 gpurun_out/pytest_gemm.log
timeout -k 10 400 python -u scripts/bench_gemm_bf16.py ${MODELS:-gpt2,llama} > gpurun_out/gemm_bf16.jsonl
cat gpurun_out/gemm_bf16.jsonl
if [ "${COLD:-0}" = "1" ]; then timeout -k 10 200 python scripts/headline_cold.py > gpurun_out/headline_cold.json; cat gpurun_out/headline_cold.json; fi
