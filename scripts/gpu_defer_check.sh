#!/bin/bash
# Deferred weight-gradient aliasing: the regression test with the fix, then (on the box's scratch
# copy only) with the queue holding the returned tensors again -- expected to FAIL -- and the
# GPT-2 DDP step time with the fix.
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
T="tests/test_lm_ops_gpu.py -k deferred"
timeout -k 10 300 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/defer_fixed.log 2>&1; echo "fixed rc=$?"; tail -2 gpurun_out/defer_fixed.log
cp distributed_training_amd/ops/lm.py /tmp/lm_fixed.py
sed -i 's/cw.view(cw.shape), None if cb is None else cb.view(cb.shape))/cw, cb)/' distributed_training_amd/ops/lm.py
grep -n "_DEFER.append" distributed_training_amd/ops/lm.py
timeout -k 10 300 python -u -m pytest $T -q --timeout 120 --timeout-method thread > gpurun_out/defer_old.log 2>&1; echo "old rc=$?"; grep -E "passed|failed|assert" gpurun_out/defer_old.log | tail -5
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp > gpurun_out/lm_old.json 2>/dev/null; echo "old rc=$?"
cp /tmp/lm_fixed.py distributed_training_amd/ops/lm.py
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp > gpurun_out/lm_new.json 2>/dev/null; echo "new rc=$?"
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp >> gpurun_out/lm_new.json 2>/dev/null; echo "new rc=$?"
cut -c1-330 gpurun_out/lm_old.json gpurun_out/lm_new.json
