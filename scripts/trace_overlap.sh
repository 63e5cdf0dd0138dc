#!/bin/bash
# Marker + kernel trace of ONE rank of a 2-rank run sharing the box's GPU
# (DTA_SHARED_GPU=1): rank 1 runs plain, rank 0 under rocprofv3 (the program
# itself after --).  Then scripts/overlap_report.py measures how much of the
# comm stream's collective time overlaps the compute stream's kernels.
#   bash scripts/trace_overlap.sh ddp|fsdp [model] [tag] [extra bench_lm args]
#   e.g. bash scripts/trace_overlap.sh fsdp llama3_8b llama4 --layers 4 --batch 1 --seq 2048
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=${1:-ddp}
MODEL=${2:-gpt2}
TAG=${3:-$S}
shift 3 || shift $#
OUT=gpurun_out/trace_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29700 + RANDOM % 200)) WORLD_SIZE=2 DTA_SHARED_GPU=1 DTA_ROCTX=1
if [ $# -eq 0 ]; then set -- --batch 4 --seq 1024 --bucket-mb 16; fi
ARGS="bench_lm.py --gpus 2 --model $MODEL --strategy $S --steps 4 --warmup 2 $*"
RANK=1 LOCAL_RANK=1 timeout -k 10 300 python3 $ARGS > "$OUT/rank1.log" 2>&1 &
R1=$!
RANK=0 LOCAL_RANK=0 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$OUT" -o run \
  -- python3 $ARGS > "$OUT/rank0.log" 2>&1
wait $R1
python3 scripts/overlap_report.py "$OUT" > "$OUT/overlap.txt"
cat "$OUT/overlap.txt"
