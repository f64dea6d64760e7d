# dK/dV kernel workgroup order: shipped (1 == block-major) vs group-major (2: a unit's key blocks
# back to back, its Q / dO stream re-read through one L2); BLLM_KV_ORDER is a temporary A/B switch
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6kvorder
BLLM_KV_ORDER=2 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash_attention and not fp32_is_flash" > gpurun_out/r6kvorder/tests.log 2>&1 || { tail -40 gpurun_out/r6kvorder/tests.log; exit 5; }
tail -1 gpurun_out/r6kvorder/tests.log
timeout -k 10 400 python -u tools/bench_attn.py --iters 20 --bwd_env_ab BLLM_KV_ORDER=1,2 \
  --shapes llama3-8B-B40,llama3-8B-B24,llama3.2-1B-B24,gpt2-774M-B64,gpt2-774M-B64-nodrop > gpurun_out/r6kvorder/bwd.jsonl 2>&1 || { tail -20 gpurun_out/r6kvorder/bwd.jsonl; exit 6; }
grep '"ab"' gpurun_out/r6kvorder/bwd.jsonl | cut -c1-250
