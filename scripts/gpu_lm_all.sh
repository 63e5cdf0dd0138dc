#!/bin/bash
# Every LM configuration of the README table on one GPU (native), JSON lines to gpurun_out/lm_all.jsonl.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/lm_all.jsonl
: > $OUT
run() {
  timeout -k 10 500 python bench_lm.py "$@" > /tmp/lma.json 2> /tmp/lma.err || { echo "FAIL $*" >> $OUT; tail -5 /tmp/lma.err >> $OUT; return 0; }
  grep '^{' /tmp/lma.json >> $OUT
}
run --model gpt2 --strategy ddp
run --model gpt2 --strategy ddp --batch 32 --steps 10 --warmup 3
run --model gpt2 --strategy fsdp
run --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 4 --warmup 2
run --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --ckpt --steps 4 --warmup 2
cat $OUT
