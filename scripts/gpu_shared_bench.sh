set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp DTA_SHARED_GPU=1
for n in 2 4 8; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 20 --warmup 5 > gpurun_out/shared_n$n.out 2> gpurun_out/shared_n$n.err
  grep '^{' gpurun_out/shared_n$n.out | cut -c1-60
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/shared_n$n.out') if l.startswith('{')][0]); print(d['value'], d['step_form'], d['calibration_ms'])"
done
