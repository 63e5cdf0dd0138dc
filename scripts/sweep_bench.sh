#!/bin/bash
# Sweep fused-kernel knobs of the headline bench on one GPU (GPU box).
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD
OUT=gpurun_out/sweep.log
for o in 1 2 4 8; do
  timeout -k 10 60 python bench.py --own-tiles $o --steps 4096 --warmup 512 --json-out /tmp/b.json > /dev/null 2>&1 || exit 1
  echo "own_tiles=$o $(cat /tmp/b.json)" >> $OUT
done
for g in 8 64; do
  timeout -k 10 60 python bench.py --graph-steps $g --steps 4096 --warmup 512 --json-out /tmp/b.json > /dev/null 2>&1 || exit 1
  echo "graph_steps=$g $(cat /tmp/b.json)" >> $OUT
done
timeout -k 10 60 python bench.py --allreduce-world1 0 --steps 4096 --warmup 512 --json-out /tmp/b.json > /dev/null 2>&1 || exit 1
echo "allreduce_world1=0 $(cat /tmp/b.json)" >> $OUT
