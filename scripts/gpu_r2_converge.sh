#!/bin/bash
# convergence evidence on the GPU through the reference CLI: GPT-2 124M (full size, bf16) and
# Llama-3.2-1B (bf16, FSDP engine via multi_gpu world 1) on synthetic Gutenberg-shaped text
set -o pipefail
mkdir -p gpurun_out/conv
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29611
timeout -k 10 500 python -u main.py --model GPT2 --num_params 124M --data_type bf16 --data_dir /tmp/conv_data \
  --synthetic_data --synthetic_mb 8 --output_dir /tmp/conv_gpt2 --n_epochs 1 --max_steps 400 --eval_freq 50 --save_ckpt_freq 100000 \
  --print_sample_iter 200 --batch_size 16 --lr 6e-4 --warmup_steps 40 --sample_tokens 20 --no_plot \
  --metrics_file gpurun_out/conv/gpt2_124m.jsonl > gpurun_out/conv/gpt2_124m.log 2>&1 || { tail -30 gpurun_out/conv/gpt2_124m.log; exit 1; }
tail -5 gpurun_out/conv/gpt2_124m.log
