# GPT-2 fused LayerNorm + dropout passes: numerics tests, then GPT2-774M preset A/B (interleaved,
# same box), then a kernel-trace breakdown of the fused default
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/lndrop
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "layernorm or bwd_bias_grad_fused or dropout" tests/test_model_gpu.py::test_fused_layernorm_dropout_in_model \
  > gpurun_out/lndrop/tests.log 2>&1 || { tail -40 gpurun_out/lndrop/tests.log; exit 3; }
tail -2 gpurun_out/lndrop/tests.log
for r in 1 2; do
  for f in 0 fwd 1; do
    BLLM_FUSED_LN_DROPOUT=$f timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 20 --warmup 5 > gpurun_out/lndrop/b_${f}_$r.log 2>&1 || { tail -20 gpurun_out/lndrop/b_${f}_$r.log; exit 4; }
    echo "fused=$f round=$r $(tail -1 gpurun_out/lndrop/b_${f}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
timeout -k 10 900 python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --tag lndrop/prof > /dev/null 2>&1 || exit 5
grep -i "norm_\|colsum\|dropout" gpurun_out/lndrop/prof/kstats.log
head -25 gpurun_out/lndrop/prof/breakdown.log
