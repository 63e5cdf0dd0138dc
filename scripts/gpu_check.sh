#!/bin/bash
# One GPU-box pass: GPU test suite, smoke, headline bench (driver's command), LM benches.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  tail -3 gpurun_out/pytest_gpu.log
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
if [ "${LM:-1}" = "1" ]; then
  timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp > gpurun_out/lm_gpt2_ddp.json 2> gpurun_out/lm_gpt2_ddp.err
  timeout -k 10 300 python bench_lm.py --model gpt2 --strategy fsdp > gpurun_out/lm_gpt2_fsdp.json 2> gpurun_out/lm_gpt2_fsdp.err
  cat gpurun_out/lm_*.json
fi
if [ "${LLAMA:-0}" = "1" ]; then
  timeout -k 10 400 python bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --ckpt --steps 4 --warmup 2 \
    > gpurun_out/lm_llama8b_fsdp.json 2> gpurun_out/lm_llama8b_fsdp.err
  cat gpurun_out/lm_llama8b_fsdp.json
fi
