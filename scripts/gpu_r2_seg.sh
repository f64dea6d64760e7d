#!/bin/bash
# headline after the dual dK/dV default + checkpoint_sequential last-block semantics; segments=2 data point
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or flash" > gpurun_out/seg_tests.log 2>&1 || { tail -30 gpurun_out/seg_tests.log; exit 1; }
tail -2 gpurun_out/seg_tests.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/seg_bench_default.log 2>&1 || { tail -20 gpurun_out/seg_bench_default.log; exit 1; }
tail -1 gpurun_out/seg_bench_default.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --ckpt_segments 2 > gpurun_out/seg_bench_s2.log 2>&1 || { tail -20 gpurun_out/seg_bench_s2.log; exit 1; }
tail -1 gpurun_out/seg_bench_s2.log
