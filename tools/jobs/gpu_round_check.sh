# Full GPU validation of the tree: GPU tests, smoke, headline bench.  Each step has its own time
# limit; the first failing step ends the script (nothing else runs on the GPU after a failure).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/check
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/check/gpu_tests.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/check/gpu_tests.log; exit 3; }
tail -3 gpurun_out/check/gpu_tests.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/check/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/check/smoke.log; exit 4; }
tail -2 gpurun_out/check/smoke.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/check/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/check/bench.log; exit 5; }
tail -1 gpurun_out/check/bench.log
