# LoRA down (64-row, 4-wave K split) / up (base rows one tile ahead): micro A/B, numerics, preset A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/lorak
timeout -k 10 240 python -u tools/bench_lora.py --tokens 39424 --only up_,down_fwd_kaug --env_ab "BLLM_LORA_DOWN=16|BLLM_LORA_DOWN=64" > gpurun_out/lorak/micro.jsonl 2>&1 || { tail -5 gpurun_out/lorak/micro.jsonl; exit 2; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_model_gpu.py -k "lora" > gpurun_out/lorak/tests.log 2>&1 || { tail -40 gpurun_out/lorak/tests.log; exit 3; }
tail -1 gpurun_out/lorak/tests.log
for r in 1 2; do
  for f in 16 64; do
    BLLM_LORA_DOWN=$f timeout -k 10 300 python -u bench.py --preset llama32_1b_lora_alpaca --steps 20 --warmup 5 > gpurun_out/lorak/lora_${f}_$r.log 2>&1 || { tail -20 gpurun_out/lorak/lora_${f}_$r.log; exit 4; }
    echo "down=$f round=$r $(tail -1 gpurun_out/lorak/lora_${f}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
timeout -k 10 600 python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --tag lorak/prof > /dev/null 2>&1 || exit 6
head -8 gpurun_out/lorak/prof/breakdown.log
cat gpurun_out/lorak/micro.jsonl
