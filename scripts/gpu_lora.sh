set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k lora -x -v --timeout 120 --timeout-method thread > gpurun_out/lora_tests.log 2>&1 && \
timeout -k 10 200 python tools/bench_lora.py > gpurun_out/bench_lora.log 2>&1 && \
timeout -k 10 300 python bench.py --model llama3_2 --num_params 1B --lora_rank 16 --batch_size 4 --steps 10 --warmup 3 --profile > gpurun_out/lora.log 2>&1
