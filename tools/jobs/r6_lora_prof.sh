# LoRA preset (Llama-3.2-1B Alpaca, r=16) kernel-trace breakdown of the final round-6 tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/v17
timeout -k 10 900 python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --tag v17/lora > gpurun_out/v17/lora_prof.log 2>&1 || { tail -30 gpurun_out/v17/lora_prof.log; exit 5; }
head -40 gpurun_out/v17/lora/breakdown.log
