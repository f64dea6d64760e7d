# attention workgroup order in the forward, dQ and dK/dV kernels: shipped (0) / q-block-major XCD
# order (1) / group-major XCD order (2); numerics under 2, then forward and backward timings
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6xcd3
BLLM_ATT_XCD=2 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash_attention and not fp32_is_flash" > gpurun_out/r6xcd3/tests.log 2>&1 || { tail -40 gpurun_out/r6xcd3/tests.log; exit 5; }
tail -1 gpurun_out/r6xcd3/tests.log
SH=llama3-8B-B40,llama3.2-1B-B24,gpt2-774M-B64,gpt2-774M-B64-nodrop
timeout -k 10 300 python -u tools/bench_attn.py --iters 20 --variants "x1:BLLM_ATT_XCD=1;x2:BLLM_ATT_XCD=2;sp1:BLLM_ATT_PP=3+BLLM_ATT_XCD=1" \
  --shapes $SH > gpurun_out/r6xcd3/fwd.jsonl 2>&1 || { tail -20 gpurun_out/r6xcd3/fwd.jsonl; exit 6; }
grep fwd_tflops gpurun_out/r6xcd3/fwd.jsonl | grep -v bwd_ms | cut -c1-300
timeout -k 10 400 python -u tools/bench_attn.py --iters 20 --bwd_env_ab BLLM_ATT_XCD=0,1,2 \
  --shapes $SH > gpurun_out/r6xcd3/bwd.jsonl 2>&1 || { tail -20 gpurun_out/r6xcd3/bwd.jsonl; exit 7; }
grep '"ab"' gpurun_out/r6xcd3/bwd.jsonl | cut -c1-300
