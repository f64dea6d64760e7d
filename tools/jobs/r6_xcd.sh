# XCD-aware workgroup order for the attention forward (BLLM_ATT_XCD=1, temporary A/B switch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6xcd
BLLM_ATT_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash_attention and not bwd_fused_rope and not fp32_is_flash" > gpurun_out/r6xcd/tests.log 2>&1 || { tail -40 gpurun_out/r6xcd/tests.log; exit 5; }
tail -1 gpurun_out/r6xcd/tests.log
timeout -k 10 300 python -u tools/bench_attn.py --iters 20 --env_ab BLLM_ATT_XCD \
  --shapes llama3-8B-B40,llama3.2-1B-B24,gpt2-774M-B64,gpt2-774M-B64-nodrop > gpurun_out/r6xcd/ab.jsonl 2>&1 || { tail -20 gpurun_out/r6xcd/ab.jsonl; exit 6; }
grep '"ab"' gpurun_out/r6xcd/ab.jsonl | cut -c1-250
