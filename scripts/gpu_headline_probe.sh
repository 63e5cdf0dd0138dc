set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_fused_ddp_gpu.py > gpurun_out/t_persist.log 2>&1
timeout -k 10 120 python3 scripts/headline_overhead.py > gpurun_out/overhead.json 2>gpurun_out/overhead.err
for i in 1 2 3; do timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/h20.log 2>/dev/null; done
timeout -k 10 120 python3 bench.py --gpus 1 --steps 2048 --warmup 256 >> gpurun_out/h20.log 2>/dev/null
tail -3 gpurun_out/t_persist.log; cat gpurun_out/overhead.json; cut -c1-200 gpurun_out/h20.log
