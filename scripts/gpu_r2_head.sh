# Round-2: fused chunked LM head + CE validation, headline bench + rocprof.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --profile > gpurun_out/r2_llama_full_v3.log 2>&1 && \
timeout -k 10 300 python bench.py --preset llama32_1b_lora_alpaca --steps 20 --warmup 5 > gpurun_out/r2_lora_alpaca_v3.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2v3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_r2v3.log 2>&1
