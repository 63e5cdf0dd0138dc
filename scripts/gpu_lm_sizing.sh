#!/bin/bash
# 288 GB sizing runs on one GPU: Llama-3 8B FSDP at seq 8192 WITHOUT activation
# checkpointing (activations fit beside the 128 GB of params / grads / AdamW
# state), and GPT-2 small DDP at larger per-GPU batches; native and stock PyTorch.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/lm_sizing.jsonl
: > $OUT
run() {
  timeout -k 10 500 python bench_lm.py "$@" > /tmp/lms.json 2> /tmp/lms.err || { echo "FAIL $*" >> $OUT; tail -5 /tmp/lms.err >> $OUT; return 0; }
  grep '^{' /tmp/lms.json >> $OUT
}
run --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 4 --warmup 2
run --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 3 --warmup 2 --impl torch
for b in 16 32; do
  run --model gpt2 --strategy ddp --batch $b --steps 10 --warmup 3
  run --model gpt2 --strategy ddp --batch $b --steps 10 --warmup 3 --impl torch
done
cat $OUT
