#!/bin/bash
# Optimizer inside the backward with the step graph (the per-bucket updates become parallel graph branches): same-box pairs.
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ov_graph.txt
for i in 1 2 3; do for v in "" "--overlap-opt"; do
  timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp $v --json-out /tmp/r.json > /dev/null 2> gpurun_out/ov_graph.err || { tail -20 gpurun_out/ov_graph.err; exit 1; }
  python -c "import json; d=json.load(open('/tmp/r.json')); print('ov=' + str(d['optimizer_in_backward']), d['step_graph'], d['ms_per_step'], d['final_loss'])" >> gpurun_out/ov_graph.txt
done; done
cat gpurun_out/ov_graph.txt
