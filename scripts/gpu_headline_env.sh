#!/bin/bash
# Driver-style headline (--steps 20 --warmup 5) under HIP runtime settings, interleaved: each line of $1 is an env prefix.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
while read -r cfg; do
  [ -z "$cfg" ] && continue
  env $cfg timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/he.out 2> gpurun_out/he.err
  echo "$cfg: $(python -c 'import json,sys; d=json.loads(open("gpurun_out/he.out").read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])')"
done < "$1"
done
