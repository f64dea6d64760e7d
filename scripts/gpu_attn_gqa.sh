# Fused-GQA dK/dV heuristic (fused when the grid has >= 1024 workgroups): numerics, kernel
# timings, headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attn or flash or model or decode or determin" -x -q --timeout 120 --timeout-method thread > gpurun_out/gqa_tests.log 2>&1 && \
timeout -k 10 200 python tools/bench_attn.py > gpurun_out/attn_auto.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_gqa_auto.log 2>&1
