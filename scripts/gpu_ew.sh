# A/B of the SwiGLU row kernels and the RMSNorm backward grid, then the GPU kernel tests and the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ew.jsonl
BLLM_SWIGLU_ROWS=0 BLLM_NORM_BWD_WG=512 timeout -k 10 120 python tools/bench_ew.py >> gpurun_out/ew.jsonl 2> gpurun_out/ew.err && \
timeout -k 10 120 python tools/bench_ew.py >> gpurun_out/ew.jsonl 2>> gpurun_out/ew.err && \
BLLM_NORM_BWD_WG=2048 timeout -k 10 120 python tools/bench_ew.py >> gpurun_out/ew.jsonl 2>> gpurun_out/ew.err && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --profile > gpurun_out/llama.log 2>&1
