# Round-2: LoRA kernels at arbitrary token counts; LoRA Alpaca bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lora" > gpurun_out/lora_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --preset llama32_1b_lora_alpaca --steps 20 --warmup 5 > gpurun_out/r2_lora_alpaca_v4.log 2>&1
