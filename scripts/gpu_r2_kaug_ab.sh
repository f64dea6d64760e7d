# K-augmented grouped LoRA (gate/up) A/B: BLLM_LORA_KAUG=1 vs 0, alternating processes; LoRA GPU tests first
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/kaug
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_cli_gpu.py -k "lora" -x -q --timeout 200 --timeout-method thread > gpurun_out/kaug/tests.log 2>&1 || exit 1
for i in 1 2; do
  BLLM_LORA_KAUG=1 timeout -k 10 300 python bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/kaug/on_$i.log 2>&1 && \
  BLLM_LORA_KAUG=0 timeout -k 10 300 python bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/kaug/off_$i.log 2>&1 || exit 1
done
