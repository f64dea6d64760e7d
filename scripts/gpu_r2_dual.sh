#!/bin/bash
# A/B of the dual-image 4-slot dK/dV kernel: numerics under BLLM_ATTN_KV_DUAL=1, then kernel timings
set -o pipefail
mkdir -p gpurun_out
export BLLM_ATTN_KV_DUAL=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or flash" > gpurun_out/dual_tests.log 2>&1 || { tail -30 gpurun_out/dual_tests.log; exit 1; }
tail -3 gpurun_out/dual_tests.log
for v in 0 1; do
  BLLM_ATTN_KV_DUAL=$v timeout -k 10 200 python -u tools/bench_attn.py --iters 30 > gpurun_out/dual_bench_$v.log 2>&1 || exit 1
  echo "== dual=$v"; cat gpurun_out/dual_bench_$v.log
done
