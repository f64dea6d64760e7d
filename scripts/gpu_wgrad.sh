# dW MFMA kernel: numerics tests, then the micro-benchmark vs hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad or split_k" -x -v --timeout 120 --timeout-method thread > gpurun_out/wgrad_tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_wgrad.py > gpurun_out/wgrad_bench.log 2>&1
