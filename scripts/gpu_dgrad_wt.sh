# Transposed-weight dX path: numerics, transpose/GEMM layout timings, headline bench on/off.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "transpose or dgrad or model" -x -q --timeout 120 --timeout-method thread > gpurun_out/wt_tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_gemm.py --tokens 24576 --iters 10 > gpurun_out/wt_gemm.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_wt_on.log 2>&1 && \
BLLM_DGRAD_WT=0 timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_wt_off.log 2>&1
