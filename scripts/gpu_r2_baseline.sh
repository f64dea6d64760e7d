# Round-2 baseline: GPU tests, smoke, headline bench with none/full actv ckpt.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --actv_ckpt full > gpurun_out/llama_full.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --actv_ckpt none > gpurun_out/llama_none.log 2>&1
