# Same-box A/B of the LoRA K-augmentation (BLLM_LORA_KAUG=0 = no augmented groups) and v11
# breakdowns of the LoRA and GPT-2 presets.  Each step has its own limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
for i in 1 2; do
timeout -k 10 300 python -u bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/ab/lora_kaug_$i.log 2>&1 || exit 3
BLLM_LORA_KAUG=0 timeout -k 10 300 python -u bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/ab/lora_nokaug_$i.log 2>&1 || exit 4
done
grep -o '"value": [0-9.]*' gpurun_out/ab/lora_*.log
python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --tag ab_prof_lora > /dev/null 2>&1 || exit 5
python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --tag ab_prof_gpt2 > /dev/null 2>&1 || exit 6
head -24 gpurun_out/ab_prof_lora/breakdown.log
head -24 gpurun_out/ab_prof_gpt2/breakdown.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ab/hl_base_$i.log 2>&1 || exit 7
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --tunableop configs/tunableop_llama3_8b_b40_mi355x.csv > gpurun_out/ab/hl_tuned_$i.log 2>&1 || exit 8
done
grep -o '"value": [0-9.]*' gpurun_out/ab/hl_*.log
