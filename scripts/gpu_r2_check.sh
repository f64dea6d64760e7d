# Round-2: kernel tests (fp32 attention, long context), smoke, headline bench after recompute change.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/attn_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --profile > gpurun_out/r2_llama_full_v2.log 2>&1 && \
timeout -k 10 300 python bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 --actv_ckpt full > gpurun_out/r2_gpt2_full.log 2>&1
