# hd-64 forward: 32-key tiles at 3 workgroups per CU for every hd-64 grid of >= 2048 workgroups
# (dropout or not); attention GPU tests, then the forward at the hd-64 shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6small2
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash_attention or attn or llama" > gpurun_out/r6small2/tests.log 2>&1 || { tail -40 gpurun_out/r6small2/tests.log; exit 5; }
tail -1 gpurun_out/r6small2/tests.log
timeout -k 10 300 python -u tools/bench_attn.py --iters 20 --shapes llama3.2-1B-B24,gpt2-774M-B64,gpt2-774M-B64-nodrop > gpurun_out/r6small2/bench.jsonl 2>&1 || { tail -20 gpurun_out/r6small2/bench.jsonl; exit 6; }
grep '"fwd_ms"' gpurun_out/r6small2/bench.jsonl | cut -c1-250
