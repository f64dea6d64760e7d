set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_attn.py > gpurun_out/attn.log 2>&1 && \
timeout -k 10 400 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 > gpurun_out/gpt2.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/llama.log 2>&1
