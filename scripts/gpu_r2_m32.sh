# dW kernel 32x32x16 MFMA variant (3): numerics (all variants + unaligned epilogue), then the
# interleaved variant-2/3 micro-benchmark on the benchmark models' dW shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/m32_tests.log 2>&1 && \
BLLM_WGRAD_VARIANT=3 timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -k "unaligned or weight_grad_path" -x -q --timeout 60 --timeout-method thread >> gpurun_out/m32_tests.log 2>&1 && \
timeout -k 10 400 python tools/bench_wgrad.py --variants 2,3 --rounds 3 > gpurun_out/m32_bench.log 2>&1
