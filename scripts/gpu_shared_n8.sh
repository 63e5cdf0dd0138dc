#!/bin/bash
# 8-rank rehearsal of the driver's scaling command on ONE GPU (DTA_SHARED_GPU=1: gloo control plane, IPC data
# plane): the 8-rank calibration of every DDP step form and the JSON line.  Not a scaling number.
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp DTA_SHARED_GPU=1
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29688 bench.py --gpus 8 --steps 20 --warmup 5 > gpurun_out/shared_n8.out 2> gpurun_out/shared_n8.err
rc=$?; echo "rc=$rc"
grep '^{' gpurun_out/shared_n8.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['ms_per_step'], d.get('step_form'), d.get('calibration_ms'), d.get('shared_gpu'))"
exit $rc
