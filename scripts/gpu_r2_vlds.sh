#!/bin/bash
# A/B of the V-in-LDS dK/dV kernels (BLLM_ATTN_KV_VLDS) + numerics
set -o pipefail
mkdir -p gpurun_out
BLLM_ATTN_KV_VLDS=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or flash" > gpurun_out/vlds_tests.log 2>&1 || { tail -30 gpurun_out/vlds_tests.log; exit 1; }
tail -1 gpurun_out/vlds_tests.log
for v in 0 1; do
  BLLM_ATTN_KV_VLDS=$v timeout -k 10 200 python -u tools/bench_attn.py --iters 30 --shapes llama3-8B,llama3-8B-B24 > gpurun_out/vlds_$v.log 2>&1 || exit 1
  echo "== vlds=$v"; grep shape gpurun_out/vlds_$v.log
done
BLLM_ATTN_KV_VLDS=1 BLLM_ATTN_KV_VARIANT=0 timeout -k 10 200 python -u tools/bench_attn.py --iters 30 --shapes llama3-8B-B24 > gpurun_out/vlds_1_unfused.log 2>&1 || exit 1
echo "== vlds=1 unfused"; grep shape gpurun_out/vlds_1_unfused.log
