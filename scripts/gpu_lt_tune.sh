# Same-box A/B: hipBLASLt heuristic top-1 vs timed candidate search for the residual GEMMs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BLLM_LT_TUNE=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k linear_residual -x -q --timeout 120 --timeout-method thread > gpurun_out/lt_tune_test.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/lt_top1.log 2>&1 && \
BLLM_LT_TUNE=1 BLLM_LT_VERBOSE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/lt_tuned.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/lt_top1_b.log 2>&1
