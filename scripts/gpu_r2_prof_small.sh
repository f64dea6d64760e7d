# Round-2: rocprof of the LoRA Alpaca (#4) and GPT2-774M DDP (#2) presets (summaries only).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_lora -o run -- python3 $R/bench.py --preset llama32_1b_lora_alpaca --steps 5 --warmup 3 > $R/gpurun_out/prof_lora.log 2>&1 && \
python3 $R/tools/step_breakdown.py /tmp/prof_lora/run_results.db > $R/gpurun_out/prof_lora_breakdown.md 2>&1 && \
python3 $R/tools/rocpd_summary.py /tmp/prof_lora/run_results.db --top 40 > $R/gpurun_out/prof_lora_top.md 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_gpt2 -o run -- python3 $R/bench.py --preset gpt2_774m_ddp --steps 3 --warmup 2 > $R/gpurun_out/prof_gpt2.log 2>&1 && \
python3 $R/tools/step_breakdown.py /tmp/prof_gpt2/run_results.db > $R/gpurun_out/prof_gpt2_breakdown.md 2>&1 && \
python3 $R/tools/rocpd_summary.py /tmp/prof_gpt2/run_results.db --top 40 > $R/gpurun_out/prof_gpt2_top.md 2>&1
