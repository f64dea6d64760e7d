# attention forward workgroup order: shipped / q-block-major XCD order (=1) / group-major XCD order (=2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6xcd2
BLLM_ATT_XCD=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash_attention and not bwd_fused_rope and not fp32_is_flash" > gpurun_out/r6xcd2/tests.log 2>&1 || { tail -40 gpurun_out/r6xcd2/tests.log; exit 5; }
tail -1 gpurun_out/r6xcd2/tests.log
timeout -k 10 300 python -u tools/bench_attn.py --iters 20 --variants "xq:BLLM_ATT_XCD=1;xg:BLLM_ATT_XCD=2" \
  --shapes llama3-8B-B40,llama3.2-1B-B24,gpt2-774M-B64,gpt2-774M-B64-nodrop,llama3-8B-B24 > gpurun_out/r6xcd2/ab.jsonl 2>&1 || { tail -20 gpurun_out/r6xcd2/ab.jsonl; exit 6; }
grep fwd_tflops gpurun_out/r6xcd2/ab.jsonl | grep -v bwd_ms | cut -c1-300
