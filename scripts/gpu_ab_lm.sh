#!/bin/bash
# A/B of GPT-2 DDP step-time knobs in one box: each line "ENV=VAL ENV2=VAL2" runs bench_lm once.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp DTA_GEMM_CACHE=${DTA_GEMM_CACHE:-/tmp/gemm_cache.json}
mkdir -p gpurun_out
while read -r cfg; do
  [ -z "$cfg" ] && continue
  env $cfg timeout -k 10 200 python bench_lm.py --model gpt2 --strategy ddp --steps 30 --warmup 5 > gpurun_out/ab.out 2> gpurun_out/ab.err
  echo "$cfg: $(grep '^{' gpurun_out/ab.out | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done < "${1:-gpurun_out/ab.cfg}"
