# v17 kernel-trace breakdowns final round-6 tree (XCD order, 16-B backward stores, dropout fold) (headline Llama-3-8B, GPT2-774M),
# plus the LoRA preset bench on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/v17
timeout -k 10 900 python tools/gpu_job.py prof --tag v17/headline > gpurun_out/v17/headline.log 2>&1 || { tail -30 gpurun_out/v17/headline.log; exit 5; }
head -22 gpurun_out/v17/headline/breakdown.log
timeout -k 10 900 python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --tag v17/gpt2 > gpurun_out/v17/gpt2.log 2>&1 || { tail -30 gpurun_out/v17/gpt2.log; exit 6; }
head -22 gpurun_out/v17/gpt2/breakdown.log
timeout -k 10 400 python -u bench.py --preset llama32_1b_lora_alpaca --steps 20 --warmup 5 > gpurun_out/v17/lora.log 2>&1 || { tail -20 gpurun_out/v17/lora.log; exit 7; }
echo "lora $(tail -1 gpurun_out/v17/lora.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')"
