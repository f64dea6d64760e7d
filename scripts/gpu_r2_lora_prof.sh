# LoRA Alpaca preset (BASELINE #4): bench + rocprof per-kernel breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/lora_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_lora -o run -- python3 $R/bench.py --preset llama32_1b_lora_alpaca --steps 3 --warmup 2 > $R/gpurun_out/prof_lora.log 2>&1 && \
python3 $R/tools/step_breakdown.py /tmp/prof_lora/run_results.db > $R/gpurun_out/lora_breakdown.md 2>&1 && \
python3 $R/tools/rocpd_summary.py /tmp/prof_lora/run_results.db --top 40 > $R/gpurun_out/lora_kernels.md 2>&1
