# Final-tree v12 breakdowns of the headline, GPT-2 and LoRA presets.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
python tools/gpu_job.py prof --tag v12_llama > /dev/null 2>&1 || exit 3
python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --tag v12_gpt2 > /dev/null 2>&1 || exit 4
python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --tag v12_lora > /dev/null 2>&1 || exit 5
head -3 gpurun_out/v12_llama/breakdown.log gpurun_out/v12_gpt2/breakdown.log gpurun_out/v12_lora/breakdown.log
