set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_gpt2 -o run -- python3 $R/bench.py --model GPT2 --num_params 774M --parallel ddp --steps 3 --warmup 2 > $R/gpurun_out/prof_gpt2.log 2>&1 && \
python3 $R/tools/step_breakdown.py /tmp/prof_gpt2/run_results.db > $R/gpurun_out/gpt2_breakdown.md 2>&1 && \
python3 $R/tools/rocpd_summary.py /tmp/prof_gpt2/run_results.db --top 40 > $R/gpurun_out/gpt2_kernels.md 2>&1
