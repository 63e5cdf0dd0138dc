#!/bin/bash
# GPT-2 small / Llama benchmarks on one GPU (GPU box).  Usage:
#   bash scripts/bench_lm_suite.sh "--model gpt2 --strategy ddp" "--model gpt2 --strategy fsdp --impl torch" ...
# (no arguments: GPT-2 DDP + FSDP, native and stock PyTorch)
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD
OUT=gpurun_out/lm_suite.log
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench_lm.py $1 --json-out /tmp/lm.json > /tmp/lm.log 2>&1 && cat /tmp/lm.json >> $OUT || { echo "FAIL $1" >> $OUT; tail -20 /tmp/lm.log >> $OUT; return 1; }; }
if [ $# -eq 0 ]; then
  set -- "--model gpt2 --strategy ddp" "--model gpt2 --strategy ddp --impl torch" \
         "--model gpt2 --strategy fsdp" "--model gpt2 --strategy fsdp --impl torch"
fi
for cfg in "$@"; do run "$cfg" || exit 1; done
