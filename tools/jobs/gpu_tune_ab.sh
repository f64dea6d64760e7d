# Interleaved A/B of a tuned TunableOp CSV against hipBLASLt's heuristic on a preset.
# usage: bash tools/jobs/gpu_tune_ab.sh <preset> <csv>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/tab
for i in 1 2; do
timeout -k 10 300 python -u bench.py --preset $1 --steps 10 --warmup 3 --tunableop none > gpurun_out/tab/$1_base_$i.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --preset $1 --steps 10 --warmup 3 --tunableop $2 > gpurun_out/tab/$1_tuned_$i.log 2>&1 || exit 5
done
grep -o '"value": [0-9.]*' gpurun_out/tab/$1_*.log
