#!/bin/bash
# One parametrized driver for GPU-box work (run through gpurun; chain tasks with &&):
#
#   bash scripts/gpu.sh tests [pytest args]         GPU test suite (default: all of tests/ -m gpu)
#   bash scripts/gpu.sh smoke                       __graft_entry__.smoke()
#   bash scripts/gpu.sh headline                    bench.py: the driver's command + steady state + linear
#   bash scripts/gpu.sh lm <tag> [bench_lm args]    bench_lm.py -> gpurun_out/lm_<tag>.json
#   bash scripts/gpu.sh prof <tag> <python args>    rocprofv3 kernel stats -> gpurun_out/prof_<tag>/summary.txt
#                                                   (per-step ms over PROF_STEPS executed steps, default 16 =
#                                                   bench_lm --steps 10 --warmup 3 with its 3 graph warm-ups)
#   bash scripts/gpu.sh pmc <tag> <ctrs> <python args>  one PMC pass (comma-separated counters)
#   bash scripts/gpu.sh shared <n> <tag> <script args>  n ranks sharing this GPU (DTA_SHARED_GPU=1, IPC comm)
#   bash scripts/gpu.sh gemm [models] [rounds]      scripts/bench_gemm64.py -> gpurun_out/gemm64_bench.jsonl
#   bash scripts/gpu.sh w4 [models] [rounds] [tiles]  scripts/bench_w4.py (forward GEMMs) -> gpurun_out/w4_bench.jsonl
#   bash scripts/gpu.sh table [--out F] [--check F]   scripts/gemm_table.py (the tracked GEMM table) -> gpurun_out/gemm_table.jsonl
#
# Every GPU step runs under its own timeout; a failing step ends the script (set -e).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
task=${1:-tests}
shift || true
case "$task" in
  tests)
    [ $# -eq 0 ] && set -- tests
    timeout -k 10 1000 python -u -m pytest "$@" -m gpu -x -v --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
    tail -2 gpurun_out/pytest_gpu.log ;;
  smoke)
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    tail -1 gpurun_out/smoke.log ;;
  headline)
    : > gpurun_out/headline.jsonl
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/headline.jsonl
    timeout -k 10 120 python bench.py --gpus 1 --steps 2048 --warmup 256 >> gpurun_out/headline.jsonl
    timeout -k 10 120 python bench.py --gpus 1 --model linear --steps 2048 --warmup 64 >> gpurun_out/headline.jsonl
    cut -c1-220 gpurun_out/headline.jsonl ;;
  lm)
    tag=$1; shift
    timeout -k 10 500 python bench_lm.py "$@" > gpurun_out/lm_$tag.json 2> gpurun_out/lm_$tag.err \
      || { tail -30 gpurun_out/lm_$tag.err; exit 1; }
    cut -c1-400 gpurun_out/lm_$tag.json ;;
  prof)
    tag=$1; shift
    out=gpurun_out/prof_$tag
    mkdir -p $out
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 "$@" \
      > $out/log 2>&1 || { tail -30 $out/log; exit 1; }
    python scripts/kstats.py $out/run_kernel_stats.csv ${PROF_STEPS:-16} 40 > $out/summary.txt
    head -30 $out/summary.txt ;;
  pmc)
    tag=$1; ctrs=$2; shift 2
    out=gpurun_out/pmc_$tag
    mkdir -p $out
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${ctrs//,/ } --output-format csv -d $out -o run -- python3 "$@" \
      > $out/log 2>&1 || { tail -30 $out/log; exit 1; }
    python scripts/pmc_summary.py $out/run_counter_collection.csv > $out/summary.txt
    head -25 $out/summary.txt ;;
  shared)
    n=$1; tag=$2; shift 2
    DTA_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + n)) "$@" > gpurun_out/shared_$tag.out 2> gpurun_out/shared_$tag.err \
      || { tail -30 gpurun_out/shared_$tag.err; exit 1; }
    grep '^{' gpurun_out/shared_$tag.out | cut -c1-300 || true ;;
  gemm)
    timeout -k 10 600 python scripts/bench_gemm64.py ${1:-gpt2,llama} ${2:-5} > gpurun_out/gemm64_bench.jsonl \
      2> gpurun_out/gemm64_bench.err || { tail -20 gpurun_out/gemm64_bench.err; exit 1; }
    python scripts/gemm64_table.py gpurun_out/gemm64_bench.jsonl ;;
  w4)
    timeout -k 10 600 python scripts/bench_w4.py ${1:-llama,gpt2} ${2:-5} ${3:-5,6,7,8,3} ${4:-fwd,dgrad,wgrad} > gpurun_out/w4_bench.jsonl \
      2> gpurun_out/w4_bench.err || { tail -20 gpurun_out/w4_bench.err; exit 1; }
    cut -c1-240 gpurun_out/w4_bench.jsonl ;;
  table)
    timeout -k 10 1200 python -u scripts/gemm_table.py "$@" > gpurun_out/gemm_table.jsonl 2> gpurun_out/gemm_table.err \
      || { tail -30 gpurun_out/gemm_table.err; exit 1; }
    tail -3 gpurun_out/gemm_table.jsonl | cut -c1-300 ;;
  *)
    echo "unknown task $task" >&2; exit 2 ;;
esac
