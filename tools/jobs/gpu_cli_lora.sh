# Llama-3.2-1B Alpaca LoRA finetune through the user-facing CLI (main.py) on one MI355X: the fused
# LoRA kernels (K-augmented groups, SwiGLU-backward dB/dA, one-pass head backward) on the user path
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/cli_lora; mkdir -p $O
timeout -k 10 600 python -u main.py --model llama3_2 --num_params 1B --finetune --dataset alpaca --use_lora \
  --lora_rank 16 --lora_alpha 32 --data_type bf16 --batch_size 32 --n_epochs 20 --synthetic_data --data_dir /tmp/cli_lora_data \
  --output_dir /tmp/cli_lora_ckpt --max_steps 41 --eval_freq 20 --print_sample_iter 1000 --save_ckpt_freq 1000 \
  --metrics_file $O/metrics.jsonl > $O/main.log 2>&1 || { tail -30 $O/main.log; exit 3; }
grep -i "tok/s\|loss" $O/main.log | tail -8
