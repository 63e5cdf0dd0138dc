#!/bin/bash
# rocprofv3 kernel-trace + stats of the headline bench (run on the GPU box).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_bench}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 bench.py --steps 512 --warmup 64 > "$OUT/bench.log" 2>&1
