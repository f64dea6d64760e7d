# One-GPU rehearsal of the multi-GPU engine path: RCCL world 1 with BLLM_FORCE_COMM=1 (real
# all-gather / reduce-scatter / all-reduce issue, waits and shard frees), numerics vs the local
# engine, then the headline bench with and without the forced collective path.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engines_gpu.py -x -v --timeout 360 --timeout-method thread > gpurun_out/rehearse_tests.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --force_comm > gpurun_out/rehearse_bench_forced.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/rehearse_bench_noshard.log 2>&1
