#!/bin/bash
# round 5, call H: the SwiGLU-backward GEMM epilogue -- kernel / op / model tests, its tracked-table entry
# (measured here and merged into the table the benches below use), Llama A/B fused vs hipBLASLt + kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
T=distributed_training_amd/ops/gemm_table_mi355x.json
bash $S tests tests/test_gemm64_gpu.py tests/test_lm_ops_gpu.py tests/test_engine_gpu.py -k "swiglu or fused_model or staged or epilogues or cross_entropy or chunked or rope or attention" &&
bash $S table --only dswiglu --merge $T --out gpurun_out/gemm_table_mi355x.json &&
cp gpurun_out/gemm_table_mi355x.json $T &&
bash $S lm llh_fused --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
DTA_GEMM_CACHE=scripts/gemm_override_dswiglu_lib.json bash $S lm llh_lib --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S lm llh_fused2 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S prof llh bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2
