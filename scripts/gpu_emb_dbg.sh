#!/bin/bash
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
DTA_EMB_FSDP=1 DTA_EMB_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_lm_ops_gpu.py -k "tied_embedding_gradient_fsdp" -x -q -s --timeout 120 --timeout-method thread > gpurun_out/emb_dbg.log 2>&1; echo rc=$?
grep -E "^EMB|^HEAD|assert [0-9]|passed|failed" gpurun_out/emb_dbg.log | head -30
