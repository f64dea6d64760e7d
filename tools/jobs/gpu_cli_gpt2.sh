# GPT2-774M DDP through the CLI (main.py -> Trainer.train_model) vs bench.py's preset on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/cligpt2
ARGS="--model GPT2 --num_params 774M --run_type multi_gpu --data_type bf16 --batch_size 64 --synthetic_data --synthetic_mb 8 --n_epochs 1 --data_dir /tmp/bllm_cli_gpt2 --output_dir /tmp/bllm_cli_gpt2_ckpt --print_sample_iter 1000 --save_ckpt_freq 0 --skip_final_save --no_plot --sample_tokens 20"
timeout -k 10 600 python -u main.py $ARGS --max_steps 61 --eval_freq 20 --metrics_file gpurun_out/cligpt2/metrics.jsonl > gpurun_out/cligpt2/main.log 2>&1 || { tail -20 gpurun_out/cligpt2/main.log; exit 3; }
grep -E "Step|GEMM selection|DDP|engine" gpurun_out/cligpt2/main.log | tail -8
timeout -k 10 400 python -u bench.py --preset gpt2_774m_ddp --steps 20 --warmup 5 > gpurun_out/cligpt2/bench.log 2>&1 || { tail -20 gpurun_out/cligpt2/bench.log; exit 4; }
tail -1 gpurun_out/cligpt2/bench.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*'
