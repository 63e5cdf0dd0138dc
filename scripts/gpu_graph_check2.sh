#!/bin/bash
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_lm_ops_gpu.py -k "graph" -x -v --timeout 120 --timeout-method thread > gpurun_out/graph_tests2.log 2>&1; rc=$?; tail -4 gpurun_out/graph_tests2.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/graph_tests2.log | head -20; exit 1; }
