#!/bin/bash
# GPT-2 small / Llama benchmarks on one GPU: native vs stock PyTorch (GPU box).
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD
OUT=gpurun_out/lm_suite.log
run() { timeout -k 10 300 python bench_lm.py "$@" --json-out /tmp/lm.json > /tmp/lm.log 2>&1 && cat /tmp/lm.json >> $OUT || { echo "FAIL $*" >> $OUT; tail -20 /tmp/lm.log >> $OUT; return 1; }; }


run --model gpt2 --strategy fsdp --batch 8 --seq 1024 --steps 20 --warmup 5 || exit 1
run --model gpt2 --strategy fsdp --batch 8 --seq 1024 --steps 20 --warmup 5 --impl torch || exit 1
run --model llama_tiny --strategy fsdp --batch 4 --seq 2048 --steps 10 --warmup 3 || exit 1
