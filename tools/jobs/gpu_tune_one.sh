# TunableOp tuning run for one preset (progress to a log under gpurun_out so it never looks idle),
# then an interleaved A/B of the tuned CSV against the heuristic.
# usage: bash tools/jobs/gpu_tune_one.sh <preset> <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/tune gpurun_out/tab
PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 900 python -u bench.py --preset $1 --steps 1 --warmup 1 --tunableop none --tunableop_tune gpurun_out/tune/$2.csv > gpurun_out/tune/tune_$2.log 2>&1 || exit 3
ls gpurun_out/tune
for i in 1 2; do
timeout -k 10 300 python -u bench.py --preset $1 --steps 10 --warmup 3 --tunableop none > gpurun_out/tab/$1_base_$i.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --preset $1 --steps 10 --warmup 3 --tunableop gpurun_out/tune/${2}0.csv > gpurun_out/tab/$1_tuned_$i.log 2>&1 || exit 5
done
grep -o '"value": [0-9.]*' gpurun_out/tab/$1_*.log
