#!/bin/bash
# convergence through the reference CLI with activation checkpointing on (the fused recompute paths):
# GPT-2 124M bf16 (GELU recompute + fused bias sums) and Llama-3.2-1B bf16 (SwiGLU recompute + RoPE-bwd epilogues)
set -o pipefail
mkdir -p gpurun_out/conv3
timeout -k 10 500 python -u main.py --model GPT2 --num_params 124M --data_type bf16 --data_dir /tmp/conv_data \
  --synthetic_data --synthetic_mb 8 --output_dir /tmp/conv_gpt2 --n_epochs 1 --max_steps 400 --eval_freq 50 --save_ckpt_freq 100000 \
  --print_sample_iter 200 --batch_size 16 --lr 6e-4 --warmup_steps 40 --sample_tokens 20 --no_plot --use_actv_ckpt \
  --metrics_file gpurun_out/conv3/gpt2_124m_ckpt.jsonl > gpurun_out/conv3/gpt2_124m_ckpt.log 2>&1 || { tail -30 gpurun_out/conv3/gpt2_124m_ckpt.log; exit 1; }
tail -3 gpurun_out/conv3/gpt2_124m_ckpt.log
timeout -k 10 600 python -u main.py --model llama3_2 --num_params 1B --data_type bf16 --data_dir /tmp/conv_data \
  --synthetic_data --synthetic_mb 8 --output_dir /tmp/conv_llama --n_epochs 1 --max_steps 300 --eval_freq 50 --save_ckpt_freq 100000 \
  --print_sample_iter 150 --batch_size 8 --lr 3e-4 --warmup_steps 30 --sample_tokens 20 --no_plot --use_actv_ckpt \
  --metrics_file gpurun_out/conv3/llama32_1b_ckpt.jsonl > gpurun_out/conv3/llama32_1b_ckpt.log 2>&1 || { tail -30 gpurun_out/conv3/llama32_1b_ckpt.log; exit 1; }
tail -3 gpurun_out/conv3/llama32_1b_ckpt.log
