# hd-64 no-dropout forward at 3 workgroups per CU (139 VGPRs fit 3 waves / SIMD) vs 2:
# BLLM_FWD_OCC3 is a temporary A/B switch
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6fwdocc3
BLLM_FWD_OCC3=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash_attention and not fp32_is_flash" > gpurun_out/r6fwdocc3/tests.log 2>&1 || { tail -40 gpurun_out/r6fwdocc3/tests.log; exit 5; }
tail -1 gpurun_out/r6fwdocc3/tests.log
timeout -k 10 300 python -u tools/bench_attn.py --iters 20 --env_ab BLLM_FWD_OCC3 \
  --shapes llama3.2-1B-B24,gpt2-774M-B64-nodrop,gpt2-774M-B24-nodrop,gpt2-124M > gpurun_out/r6fwdocc3/ab.jsonl 2>&1 || { tail -20 gpurun_out/r6fwdocc3/ab.jsonl; exit 6; }
grep '"ab"' gpurun_out/r6fwdocc3/ab.jsonl | cut -c1-250
