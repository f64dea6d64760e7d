# dW MFMA kernel: numerics tests (every schedule variant), the variant/hipBLASLt micro-benchmark
# (interleaved in one process), then the headline bench with the per-shape dispatch.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad or split_k" -x -q --timeout 120 --timeout-method thread > gpurun_out/wgrad_tests.log 2>&1 && \
timeout -k 10 400 python tools/bench_wgrad.py --variants 1,2 --rounds 3 > gpurun_out/wgrad_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 8 --warmup 3 --profile > gpurun_out/bench_wgrad_v1.log 2>&1 && BLLM_WGRAD_VARIANT=2 timeout -k 10 300 python bench.py --steps 8 --warmup 3 --profile > gpurun_out/bench_wgrad_v2.log 2>&1
