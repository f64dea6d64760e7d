#!/bin/bash
# A/B of attention forward variants (BLLM_ATTN_FWD_VARIANT) + numerics of the candidate
set -o pipefail
mkdir -p gpurun_out
V=${1:-3}
BLLM_ATTN_FWD_VARIANT=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or flash" > gpurun_out/fwd_tests.log 2>&1 || { tail -30 gpurun_out/fwd_tests.log; exit 1; }
tail -2 gpurun_out/fwd_tests.log
for v in 0 $V; do
  BLLM_ATTN_FWD_VARIANT=$v timeout -k 10 200 python -u tools/bench_attn.py --iters 30 > gpurun_out/fwd_bench_$v.log 2>&1 || exit 1
  echo "== fwd variant $v"; grep shape gpurun_out/fwd_bench_$v.log
done
