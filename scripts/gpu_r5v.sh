#!/bin/bash
# round 5, call V: PyTorch TunableOp for the GEMMs that stay on the library (hipBLASLt / rocBLAS solution search
# per shape, instead of the library heuristic's first pick): tune inside one GPT-2 and one Llama-3 8B bench (the
# eager warm-up steps make every library call of the step once), then a same-box A/B of each model with the
# tuned results loaded (tuning off) against the default heuristic.  Also re-runs the stream-K tests (binding
# changed: workspace size from the kernel's tile dimensions).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S tests tests/test_gemm64_gpu.py -k stream_k || exit 1
G="--model gpt2 --strategy ddp --steps 30 --warmup 5"
L="--model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2"
TUNE="PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1"
env $TUNE PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_g2.csv bash $S lm v_tune_g2 --model gpt2 --strategy ddp --steps 5 --warmup 3 &&
env $TUNE PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_ll.csv bash $S lm v_tune_ll --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 2 --warmup 2 || exit 1
ls -la gpurun_out/tunableop_*.csv
: > gpurun_out/ab_tunableop_r5v.jsonl
run() {  # run <tag> <env> <model args...>
  local tag=$1 ev=$2; shift 2
  env $ev bash $S lm v_$tag "$@" > /dev/null || return 1
  python3 -c "import json; j=json.loads(open('gpurun_out/lm_v_$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag':'$tag','ms':j['ms_per_step']}))" | tee -a gpurun_out/ab_tunableop_r5v.jsonl
}
USEG="PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_g2.csv"
USEL="PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_ll.csv"
for r in 1 2; do
  run g_base_$r "DTA_X=0" $G && run g_tuned_$r "$USEG" $G || exit 1
done
for r in 1 2; do
  run l_base_$r "DTA_X=0" $L && run l_tuned_$r "$USEL" $L || exit 1
done
