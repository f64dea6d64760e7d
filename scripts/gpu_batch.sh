# Per-GPU micro-batch sweep for the headline config (throughput + peak memory).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for B in 24 32; do
  timeout -k 10 300 python bench.py --batch_size $B --steps 5 --warmup 2 > gpurun_out/batch_$B.log 2>&1 || exit 1
done
