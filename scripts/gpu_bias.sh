# Bias-gradient column sums: GPU kernel tests, micro-bench, GPT-2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kernel_tests.log 2>&1 && \
timeout -k 10 120 python tools/bench_ew.py > gpurun_out/ew2.jsonl 2> gpurun_out/ew2.err && \
timeout -k 10 300 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 > gpurun_out/gpt2.log 2>&1
