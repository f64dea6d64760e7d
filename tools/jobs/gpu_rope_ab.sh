# QKV GEMM + RoPE epilogue on our forward-layout kernel (BLLM_FUSED_ROPE=1) vs hipBLASLt + rope_:
# three interleaved pairs on one box, headline settings
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ropeab
for r in 1 2 3; do
  for f in 0 1; do
    BLLM_FUSED_ROPE=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ropeab/rope${f}_$r.log 2>&1 || { tail -20 gpurun_out/ropeab/rope${f}_$r.log; exit 3; }
    echo "rope=$f round=$r $(tail -1 gpurun_out/ropeab/rope${f}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*\|"power_w_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
