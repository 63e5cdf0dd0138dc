#!/bin/bash
# Full GPU pass: suite, smoke, headline (driver command + steady state), linear, LM benches, shared-GPU multi-rank rehearsal.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
: > gpurun_out/bench_all.jsonl
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/bench_all.jsonl
timeout -k 10 120 python bench.py --gpus 1 --steps 2048 --warmup 256 >> gpurun_out/bench_all.jsonl
timeout -k 10 120 python bench.py --gpus 1 --model linear --steps 2048 --warmup 64 >> gpurun_out/bench_all.jsonl
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp >> gpurun_out/bench_all.jsonl 2> gpurun_out/lm.err
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy fsdp >> gpurun_out/bench_all.jsonl 2>> gpurun_out/lm.err
cut -c1-200 gpurun_out/bench_all.jsonl
export DTA_SHARED_GPU=1
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 20 --warmup 5 > gpurun_out/shared_n$n.out 2> gpurun_out/shared_n$n.err
  grep '^{' gpurun_out/shared_n$n.out | cut -c1-160
done
for s in ddp fsdp; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29620 bench_lm.py --gpus 2 --model gpt2 --strategy $s --layers 4 --steps 5 --warmup 2 > gpurun_out/shared_lm_$s.out 2> gpurun_out/shared_lm_$s.err
  grep '^{' gpurun_out/shared_lm_$s.out | cut -c1-200
done
