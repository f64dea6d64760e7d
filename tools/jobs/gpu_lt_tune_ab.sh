# Residual GEMMs (o / down projections, hipBLASLt C != D): heuristic top-1 (default) vs timing the
# top-16 candidates (BLLM_LT_TUNE=1) vs torch.addmm through the TunableOp table (BLLM_LT_RESIDUAL=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/lttune
for r in 1 2; do
  for arm in base tune addmm; do
    case $arm in base) E="";; tune) E="BLLM_LT_TUNE=1";; addmm) E="BLLM_LT_RESIDUAL=0";; esac
    env $E timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/lttune/${arm}_$r.log 2>&1 || { tail -20 gpurun_out/lttune/${arm}_$r.log; exit 3; }
    echo "$arm round=$r $(tail -1 gpurun_out/lttune/${arm}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
