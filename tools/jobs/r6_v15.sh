# v15 kernel-trace breakdowns of the round-6 tree (headline Llama-3-8B, GPT2-774M) and the
# GPT-2 / LoRA presets on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/v15
timeout -k 10 900 python tools/gpu_job.py prof --tag v15/headline > gpurun_out/v15/headline.log 2>&1 || { tail -30 gpurun_out/v15/headline.log; exit 5; }
head -22 gpurun_out/v15/headline/breakdown.log
timeout -k 10 900 python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --tag v15/gpt2 > gpurun_out/v15/gpt2.log 2>&1 || { tail -30 gpurun_out/v15/gpt2.log; exit 6; }
head -22 gpurun_out/v15/gpt2/breakdown.log
for p in gpt2_774m_ddp llama32_1b_lora_alpaca; do
  timeout -k 10 400 python -u bench.py --preset $p --steps 20 --warmup 5 > gpurun_out/v15/$p.log 2>&1 || { tail -20 gpurun_out/v15/$p.log; exit 7; }
  echo "$p $(tail -1 gpurun_out/v15/$p.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' ')"
done
