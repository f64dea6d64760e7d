# dX MFMA GEMM: numerics tests, micro-benchmark vs hipBLASLt, headline bench with it on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_nn or dgrad or wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/dgrad_tests.log 2>&1 && \
timeout -k 10 400 python tools/bench_dgrad.py > gpurun_out/dgrad_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_dgrad_on.log 2>&1 && \
BLLM_DGRAD_GEMM=0 timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_dgrad_off.log 2>&1
