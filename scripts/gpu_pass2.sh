set -euo pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/prof_llama gpurun_out/prof_mlp
timeout -k 10 300 python -u -m pytest tests/test_p2p_gpu.py tests/test_fused_ddp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_p2p.log 2>&1
timeout -k 10 200 python scripts/bench_attn.py > gpurun_out/attn.jsonl 2> gpurun_out/attn.err
cat gpurun_out/attn.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp -o run -- python3 bench.py --steps 4096 --warmup 256 > gpurun_out/prof_mlp/bench.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama -o run -- python3 bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --ckpt --steps 2 --warmup 1 > gpurun_out/prof_llama/bench.log 2>&1
