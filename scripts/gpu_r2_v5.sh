# Round-2 v5: GPU tests, smoke, default bench (B=40), rocprof summary.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 8 --warmup 3 --profile > gpurun_out/r2_llama_full_v5.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_v5 -o run -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/prof_v5.log 2>&1 && \
python3 $R/tools/step_breakdown.py /tmp/prof_v5/run_results.db > $R/gpurun_out/prof_v5_breakdown.md 2>&1
