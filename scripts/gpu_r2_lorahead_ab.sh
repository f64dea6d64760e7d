# K-augmented LoRA head A/B: BLLM_LORA_HEAD_FUSED=1 vs 0, alternating processes on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/loraab
for i in 1 2; do
  BLLM_LORA_HEAD_FUSED=1 timeout -k 10 300 python bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/loraab/on_$i.log 2>&1 && \
  BLLM_LORA_HEAD_FUSED=0 timeout -k 10 300 python bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/loraab/off_$i.log 2>&1 || exit 1
done
