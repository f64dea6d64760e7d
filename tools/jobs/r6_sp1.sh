# software-pipelined forward (BLLM_ATT_PP=3, temporary A/B switch) and the ping-pong one (=1):
# numerics of the pipelined kernel, then forward TF/s of all three interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6sp
BLLM_ATT_PP=3 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash_attention and not bwd_fused_rope and not fp32_is_flash" > gpurun_out/r6sp/tests.log 2>&1 || { tail -40 gpurun_out/r6sp/tests.log; exit 5; }
tail -1 gpurun_out/r6sp/tests.log
timeout -k 10 300 python -u tools/bench_attn.py --iters 20 --variants "pp:BLLM_ATT_PP=1;sp:BLLM_ATT_PP=3" \
  --shapes llama3-8B-B40,llama3.2-1B-B24,gpt2-774M-B64,gpt2-774M-B64-nodrop > gpurun_out/r6sp/ab.jsonl 2>&1 || { tail -20 gpurun_out/r6sp/ab.jsonl; exit 6; }
grep fwd_tflops gpurun_out/r6sp/ab.jsonl | grep -v bwd_ms | cut -c1-300
