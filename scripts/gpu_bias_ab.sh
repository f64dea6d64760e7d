# Same-box GPT-2 A/B of the bias-gradient band count (256 = previous, 1024 = new default).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 > gpurun_out/gpt2_new.log 2>&1 && \
BLLM_COLSUM_BANDS=256 timeout -k 10 300 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 > gpurun_out/gpt2_old.log 2>&1 && \
timeout -k 10 300 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 > gpurun_out/gpt2_new2.log 2>&1 && \
BLLM_COLSUM_BANDS=256 timeout -k 10 300 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 > gpurun_out/gpt2_old2.log 2>&1
