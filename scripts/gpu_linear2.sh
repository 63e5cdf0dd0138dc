#!/bin/bash
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused_linear_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
DTA_LINEAR_WAVE=0 timeout -k 10 300 python -u -m pytest tests/test_fused_linear_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
timeout -k 10 100 python bench.py --model linear --steps 2048 --warmup 64 | cut -c1-200
timeout -k 10 100 python bench.py --model linear --steps 20 --warmup 5 | cut -c1-200
DTA_LINEAR_WAVE=0 timeout -k 10 100 python bench.py --model linear --steps 2048 --warmup 64 | cut -c1-200
