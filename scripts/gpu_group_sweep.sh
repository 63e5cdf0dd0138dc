#!/bin/bash
# Grouped weight-gradient flush threshold (DTA_WGRAD_GROUP, 256x256 tiles per flush) on the GPT-2 DDP step, same box.
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/group_sweep.txt
for i in 1 2; do for g in 200 450 700 1400; do
  DTA_WGRAD_GROUP=$g timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --json-out /tmp/r.json > /dev/null 2> gpurun_out/group_sweep.err || { tail -20 gpurun_out/group_sweep.err; exit 1; }
  python -c "import json; d=json.load(open('/tmp/r.json')); print('group=$g', d['ms_per_step'], d['final_loss'])" >> gpurun_out/group_sweep.txt
done; done
cat gpurun_out/group_sweep.txt
