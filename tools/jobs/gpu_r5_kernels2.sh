# rcp-based SiLU in every SwiGLU kernel + the fused LoRA SwiGLU/wgrad kernel at 2 waves/SIMD:
# numerics, LoRA preset A/B, headline bench + kernel-trace breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/k2
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_model_gpu.py -k "swiglu or lora or layernorm or gemm_nt or fused" \
  > gpurun_out/k2/tests.log 2>&1 || { tail -40 gpurun_out/k2/tests.log; exit 3; }
tail -2 gpurun_out/k2/tests.log
for r in 1 2; do
  for f in 0 1; do
    BLLM_LORA_SWIGLU_WGRAD=$f timeout -k 10 300 python -u bench.py --preset llama32_1b_lora_alpaca --steps 20 --warmup 5 > gpurun_out/k2/lora_${f}_$r.log 2>&1 || { tail -20 gpurun_out/k2/lora_${f}_$r.log; exit 4; }
    echo "lora fused=$f round=$r $(tail -1 gpurun_out/k2/lora_${f}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/k2/headline.log 2>&1 || { tail -20 gpurun_out/k2/headline.log; exit 5; }
echo "headline $(tail -1 gpurun_out/k2/headline.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
timeout -k 10 600 python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --tag k2/prof_lora > /dev/null 2>&1 || exit 6
timeout -k 10 600 python tools/gpu_job.py prof --tag k2/prof_llama > /dev/null 2>&1 || exit 7
grep -i "swiglu\|lora_wgrad" gpurun_out/k2/prof_lora/kstats.log gpurun_out/k2/prof_llama/kstats.log
head -14 gpurun_out/k2/prof_llama/breakdown.log
