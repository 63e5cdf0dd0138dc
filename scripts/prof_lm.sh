#!/bin/bash
# rocprofv3 kernel stats of a GPT-2 small DDP step (GPU box).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_gpt2}
shift || true
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 bench_lm.py --model gpt2 --strategy ddp --batch 8 --seq 1024 --steps 10 --warmup 3 "$@" > "$OUT/bench.log" 2>&1
