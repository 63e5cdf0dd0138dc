#!/bin/bash
# MLP DDP step forms (persistent one-shot / rs+ag, per-step program) with several processes on the box's GPU.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_ddp_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_xchg.log 2>&1
for n in 2 4; do
  for m in oneshot rsag helpers auto; do
    DTA_MLP_XMODE=$m timeout -k 10 120 python scripts/persistent_ddp_latency.py --procs $n --comm >> gpurun_out/xchg_latency.jsonl
  done
done
cat gpurun_out/xchg_latency.jsonl
