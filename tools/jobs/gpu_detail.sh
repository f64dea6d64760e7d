# Per-kernel detail (avg us / call) of the LoRA and GPT-2 presets' LoRA / embedding kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --set kgrep=lora --tag dt_lora > /dev/null 2>&1 || exit 5
python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --set kgrep=emb --tag dt_gpt2 > /dev/null 2>&1 || exit 6
cat gpurun_out/dt_lora/kstats.log gpurun_out/dt_gpt2/kstats.log
