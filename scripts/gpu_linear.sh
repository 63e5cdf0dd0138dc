#!/bin/bash
# Fused Linear (reference default) program: tests, bench line, rocprof of the reference entrypoint; headline overhead probe.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/prof_linear
timeout -k 10 300 python -u -m pytest tests/test_fused_linear_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_linear.log 2>&1
tail -3 gpurun_out/pytest_linear.log
timeout -k 10 120 python bench.py --model linear --steps 2048 --warmup 64 > gpurun_out/bench_linear.json
cat gpurun_out/bench_linear.json
timeout -k 10 120 python bench.py --model linear --steps 20 --warmup 5 >> gpurun_out/bench_linear.json
tail -1 gpurun_out/bench_linear.json
cd gpurun_out/prof_linear
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d . -o run -- python3 -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 ../../src/multigpu_multi_node.py 10 2 --batch_size 32 > ref_entry.log 2>&1 || true
cd ../..
ls gpurun_out/prof_linear | head
timeout -k 10 120 python3 scripts/headline_overhead.py > gpurun_out/overhead.json 2> gpurun_out/overhead.err
cat gpurun_out/overhead.json
