# GELU forward on the A&S erf form for 16-bit outputs: numerics, then GPT2-774M with the c_fc +
# bias + GELU GEMM epilogue (BLLM_FUSED_GELU=1) vs the separate pass, interleaved on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/geluab
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_training_parity_gpu.py -k "gelu or bias or gpt2 or parity" > gpurun_out/geluab/tests.log 2>&1 || { tail -40 gpurun_out/geluab/tests.log; exit 3; }
tail -1 gpurun_out/geluab/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/geluab/smoke.log 2>&1 || { tail -20 gpurun_out/geluab/smoke.log; exit 4; }
grep -c "smoke ok" gpurun_out/geluab/smoke.log
for r in 1 2; do
  for f in 0 1; do
    BLLM_FUSED_GELU=$f timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 20 --warmup 5 > gpurun_out/geluab/g${f}_$r.log 2>&1 || { tail -20 gpurun_out/geluab/g${f}_$r.log; exit 5; }
    echo "gelu_fused=$f round=$r $(tail -1 gpurun_out/geluab/g${f}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
