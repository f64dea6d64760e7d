# Headline end to end: QKV + RoPE epilogue on csrc/gemm_nt.hip vs TunableOp GEMM + rope_, ABAB
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6rope
for arm in base rope base rope; do
  extra=""; [ "$arm" = rope ] && extra="--gemm_epilogues rope"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $extra > gpurun_out/r6rope/$arm.log 2>&1 || { tail -20 gpurun_out/r6rope/$arm.log; exit 5; }
  echo "$arm $(tail -1 gpurun_out/r6rope/$arm.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
done
