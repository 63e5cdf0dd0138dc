#!/bin/bash
# round 5, call E: attention prefetch-depth / op-order diagnostics, backward ILV A/B (dQ + dK/dV),
# GPT-2 head weight-gradient pick A/B in-step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
: > gpurun_out/attn_diag_r5e.jsonl
for r in 1 2; do
  for pf in 3 4 6; do
    for ilv in 0 1; do
      DTA_ATTN_BWD_ILV=$ilv timeout -k 10 120 ./scripts/attn_diag_pf$pf "pf${pf}_ilv${ilv}" >> gpurun_out/attn_diag_r5e.jsonl || exit $?
    done
  done
done
cat gpurun_out/attn_diag_r5e.jsonl
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_lm_ops_gpu.py -k "attention" > gpurun_out/pytest_r5e.log 2>&1 || { tail -30 gpurun_out/pytest_r5e.log; exit 1; }
tail -1 gpurun_out/pytest_r5e.log
for r in 1 2; do
  bash $S lm g2e_w4_$r --model gpt2 --strategy ddp --steps 30 --warmup 5 || exit $?
  DTA_GEMM_CACHE=scripts/gemm_override_headwgrad_lib.json bash $S lm g2e_lib_$r --model gpt2 --strategy ddp --steps 30 --warmup 5 || exit $?
done
