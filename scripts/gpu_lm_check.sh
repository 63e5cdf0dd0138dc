set -euo pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lm_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lm.log 2>&1 || { tail -30 gpurun_out/pytest_lm.log; exit 1; }
tail -1 gpurun_out/pytest_lm.log
scripts/gpu_lm_all.sh
