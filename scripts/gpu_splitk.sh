set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "split_k or lora" -x -v --timeout 120 --timeout-method thread > gpurun_out/splitk_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 --profile > gpurun_out/cfg_gpt2_774m.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/model_gpu_tests.log 2>&1
