# Round-2 v8: GPU tests, smoke, default bench (B=40, 31/32 blocks recomputed), rocprof breakdown + top kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 180 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r2_llama_full_v8.log 2>&1 || { tail -30 gpurun_out/r2_llama_full_v8.log; exit 1; }
tail -1 gpurun_out/r2_llama_full_v8.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_v8 -o run -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/prof_v8.log 2>&1 || { tail -20 $R/gpurun_out/prof_v8.log; exit 1; }
python3 $R/tools/step_breakdown.py /tmp/prof_v8/run_results.db > $R/gpurun_out/prof_v8_breakdown.md 2>&1
python3 $R/tools/rocpd_summary.py /tmp/prof_v8/run_results.db --top 30 --md $R/gpurun_out/prof_v8_top.md > /dev/null 2>&1
head -30 $R/gpurun_out/prof_v8_breakdown.md
