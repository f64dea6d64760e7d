# v14 kernel-trace breakdown of the Llama-3.2-1B LoRA preset (with lora_head_bwd_k)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/lorahead
timeout -k 10 900 python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --tag lorahead/prof14 > gpurun_out/lorahead/prof14.log 2>&1 || { tail -30 gpurun_out/lorahead/prof14.log; exit 5; }
head -24 gpurun_out/lorahead/prof14/breakdown.log
grep -i "lora\|lhb" gpurun_out/lorahead/prof14/kstats.log
