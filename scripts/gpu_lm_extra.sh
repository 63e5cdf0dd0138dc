#!/bin/bash
# GPT-2 DDP at B=32 and with activation checkpointing (step graph on), one run each.
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/lm_extra.jsonl
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --batch 32 >> gpurun_out/lm_extra.jsonl 2> gpurun_out/lm_extra.err; echo "b32 rc=$?"
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --ckpt >> gpurun_out/lm_extra.jsonl 2>> gpurun_out/lm_extra.err; echo "ckpt rc=$?"
python - <<'PY'
import json
for l in open("gpurun_out/lm_extra.jsonl"):
    d = json.loads(l); print(d["config"]["global_batch"], d["config"]["activation_checkpointing"], d["step_graph"], d["ms_per_step"], d["value"], d["peak_mem_GB"])
PY
grep -i "graph unavailable\|error" gpurun_out/lm_extra.err | head -5 || true
