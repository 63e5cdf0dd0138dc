#!/bin/bash
# The FSDP first-claim regression test on the fixed code, then (box copy only) with the claim
# added before the buffer creation again -- expected to FAIL.
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
T="tests/test_lm_ops_gpu.py -k first_claim"
timeout -k 10 300 python -u -m pytest $T -q --timeout 120 --timeout-method thread > gpurun_out/claim_fixed.log 2>&1; echo "fixed rc=$?"; tail -1 gpurun_out/claim_fixed.log
python - <<'PY'
p = "distributed_training_amd/parallel/fsdp.py"
s = open(p).read()
old = "        buf = self.grad_buffer()  # (first call of the backward: creates the buffer and resets the claims,\n        self._claimed.add(e)"
assert old in s
s = s.replace(old, "        self._claimed.add(e)\n        buf = self.grad_buffer()")
open(p, "w").write(s)
PY
timeout -k 10 300 python -u -m pytest $T -q --timeout 120 --timeout-method thread > gpurun_out/claim_old.log 2>&1; echo "old rc=$?"; grep -E "assert [0-9]|passed|failed" gpurun_out/claim_old.log | head -3
