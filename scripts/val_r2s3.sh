set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r2s3.log 2>&1 \
 && echo "gpu tests ok" && tail -2 gpurun_out/gpu_tests_r2s3.log \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2s3.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r2s3.log 2>&1 \
 && tail -2 gpurun_out/bench_r2s3.log
