# LoRA MLP: gate/up dB + down dA inside the SwiGLU backward -- numerics, then the Llama-3.2-1B
# LoRA preset A/B (interleaved, one box), then a kernel-trace breakdown of the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/loraswi
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "swiglu or lora or layernorm" tests/test_model_gpu.py -k "lora or layernorm_dropout or swiglu" \
  > gpurun_out/loraswi/tests.log 2>&1 || { tail -40 gpurun_out/loraswi/tests.log; exit 3; }
tail -2 gpurun_out/loraswi/tests.log
for r in 1 2; do
  for f in 0 1; do
    BLLM_LORA_SWIGLU_WGRAD=$f timeout -k 10 300 python -u bench.py --preset llama32_1b_lora_alpaca --steps 20 --warmup 5 > gpurun_out/loraswi/b_${f}_$r.log 2>&1 || { tail -20 gpurun_out/loraswi/b_${f}_$r.log; exit 4; }
    echo "fused=$f round=$r $(tail -1 gpurun_out/loraswi/b_${f}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
timeout -k 10 900 python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --tag loraswi/prof > /dev/null 2>&1 || exit 5
grep -i "lora\|swiglu" gpurun_out/loraswi/prof/kstats.log
head -20 gpurun_out/loraswi/prof/breakdown.log
