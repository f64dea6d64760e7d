#!/bin/bash
# GPU validation pass (run via gpurun). Each GPU step has its own time limit; steps are
# chained with && so the first failure / fault / timeout ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 \
 && echo "gpu tests ok" \
 && timeout -k 10 400 torchrun --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
      bench.py --gpus 1 --steps 3 --warmup 1 --parallel fsdp > gpurun_out/bench_fsdp1.log 2>&1 \
 && echo "fsdp1 bench ok" \
 && timeout -k 10 400 python main.py --model llama3_2 --num_params 1B --finetune --dataset alpaca \
      --data_dir /tmp/alpaca --synthetic_data --use_lora --lora_rank 16 --data_type bf16 --batch_size 8 \
      --output_dir /tmp/ckpt --max_steps 30 --eval_freq 10 --print_sample_iter 1000 --save_ckpt_freq 1000 \
      --metrics_file gpurun_out/lora_metrics.jsonl > gpurun_out/lora_run.log 2>&1 \
 && echo "lora finetune ok"
rc=$?
tail -3 gpurun_out/gpu_tests.log
tail -2 gpurun_out/bench_fsdp1.log 2>/dev/null
tail -4 gpurun_out/lora_run.log 2>/dev/null
exit $rc
