set -euo pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --impl torch > gpurun_out/lm_gpt2_ddp_torch.json 2> gpurun_out/lm_t1.err
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy fsdp --impl torch > gpurun_out/lm_gpt2_fsdp_torch.json 2> gpurun_out/lm_t2.err
cat gpurun_out/lm_gpt2_*torch.json
timeout -k 10 600 python bench_lm.py --model llama3_8b --strategy fsdp --impl torch --batch 1 --seq 8192 --ckpt --steps 3 --warmup 2 > gpurun_out/lm_llama8b_fsdp_torch.json 2> gpurun_out/lm_t3.err
cat gpurun_out/lm_llama8b_fsdp_torch.json
