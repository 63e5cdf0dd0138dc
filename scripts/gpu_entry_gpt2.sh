#!/bin/bash
# Reference-style entrypoint on the GPT-2 DDP config (step graph on, then off): epoch throughput lines.
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
for g in true false; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29650 \
    src/distributed_trainer.py model=gpt2_small train=gpt2_ddp train.dataset_size=256 train.total_epochs=2 train.step_graph=$g \
    hydra.run.dir=/tmp/entry_$g > gpurun_out/entry_gpt2_$g.log 2>&1; echo "step_graph=$g rc=$?"
  grep -E "samples/s|Error|error" gpurun_out/entry_gpt2_$g.log | tail -3
done
