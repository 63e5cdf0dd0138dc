#!/bin/bash
# persistent-MLP (headline) kernel: numerics tests, then the driver-style and long bench runs
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fused_ddp_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
for i in 1 2 3; do DTA_BENCH_TRACE=1 timeout -k 10 100 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '\[bench\].*\|\[fused_mlp\].*\|"value": [0-9.]*' | tr '\n' ' '; echo; done
for i in 1 2; do timeout -k 10 100 python bench.py --steps 20 --warmup 5 | cut -c1-190; done
timeout -k 10 100 python bench.py --steps 2048 --warmup 64 | cut -c1-190
