# Round-2: per-GPU micro-batch sweep for the full-ckpt headline (memory is ~131 GiB at B=24).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for B in 24 32 40; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 3 --batch_size $B > gpurun_out/r2_bsweep_b$B.log 2>&1 || exit 1
done
