# hipBLASLt residual GEMM (C != D): GPU tests, then same-box bench A/B against torch.addmm.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/lt_on.log 2>&1 && \
BLLM_LT_RESIDUAL=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/lt_off.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/lt_on2.log 2>&1 && \
timeout -k 10 300 python bench.py --model llama3_2 --num_params 1B --lora_rank 16 --steps 10 --warmup 3 > gpurun_out/lora.log 2>&1 && \
timeout -k 10 300 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 > gpurun_out/gpt2.log 2>&1
