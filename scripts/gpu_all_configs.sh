# Bench every BASELINE config at the bench.py defaults (B=16 per GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 8 --warmup 3 --profile > gpurun_out/cfg_llama3_8b.log 2>&1 && \
timeout -k 10 300 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 --profile > gpurun_out/cfg_gpt2_774m.log 2>&1 && \
timeout -k 10 300 python bench.py --model llama3_2 --num_params 1B --lora_rank 16 --steps 10 --warmup 3 --profile > gpurun_out/cfg_lora_1b.log 2>&1 && \
timeout -k 10 300 python bench.py --model llama2 --num_params 7B --parallel zero1 --steps 8 --warmup 3 --profile > gpurun_out/cfg_llama2_7b.log 2>&1
