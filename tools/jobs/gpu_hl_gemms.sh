# Headline per-kernel hipBLASLt stats (which GEMM solutions run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
python tools/gpu_job.py prof --set kgrep=Cijk --tag hlg > /dev/null 2>&1 || exit 5
cat gpurun_out/hlg/kstats.log; head -8 gpurun_out/hlg/breakdown.log
