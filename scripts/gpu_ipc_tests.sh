set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ipc_gpu.py > gpurun_out/t_ipc.log 2>&1
