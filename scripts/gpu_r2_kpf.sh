# forward K-fragment prefetch: attention tests + attention bench (all shapes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "attn or flash or keep_mask" -x -q --timeout 120 --timeout-method thread > gpurun_out/kpf_tests.log 2>&1 && \
timeout -k 10 200 python3 tools/bench_attn.py --iters 30 > gpurun_out/kpf_bench.log 2>&1 && \
timeout -k 10 200 python3 tools/bench_attn.py --iters 30 --shapes llama3-8B-B24,gpt2-774M-B24,gpt2-774M-B24-nodrop,llama3.2-1B-B24 >> gpurun_out/kpf_bench.log 2>&1
