# Bench + kernel profile of the secondary BASELINE configs (GPT2-774M DDP, Llama-3.2-1B LoRA, Llama-2-7B).
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model llama3_2 --num_params 1B --lora_rank 16 --steps 10 --warmup 3 --profile > gpurun_out/lora.log 2>&1 && \
timeout -k 10 300 python bench.py --model llama2 --num_params 7B --steps 8 --warmup 3 --profile > gpurun_out/llama2.log 2>&1 && \
timeout -k 10 300 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 --profile > gpurun_out/gpt2.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_gpt2 -o run -- python3 $R/bench.py --model GPT2 --num_params 774M --parallel ddp --steps 3 --warmup 2 > $R/gpurun_out/prof_gpt2.log 2>&1 && \
python3 $R/tools/step_breakdown.py /tmp/prof_gpt2/run_results.db > $R/gpurun_out/gpt2_breakdown.md 2>&1 && \
python3 $R/tools/rocpd_summary.py /tmp/prof_gpt2/run_results.db --top 60 > $R/gpurun_out/gpt2_kernels.md 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_lora -o run -- python3 $R/bench.py --model llama3_2 --num_params 1B --lora_rank 16 --steps 3 --warmup 2 > $R/gpurun_out/prof_lora.log 2>&1 && \
python3 $R/tools/step_breakdown.py /tmp/prof_lora/run_results.db > $R/gpurun_out/lora_breakdown.md 2>&1 && \
python3 $R/tools/rocpd_summary.py /tmp/prof_lora/run_results.db --top 60 > $R/gpurun_out/lora_kernels.md 2>&1
