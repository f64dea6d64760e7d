# CLI headline on the final round-5 tree (61 steps, eval every 20), then bench.py on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/cli3; mkdir -p $O
ARGS="--model llama3 --num_params 8B --run_type multi_gpu --use_fsdp --use_actv_ckpt --actv_ckpt_mode auto --data_type bf16 --batch_size 40 --synthetic_data --synthetic_mb 4 --n_epochs 1 --data_dir /tmp/bllm_cli_gutenberg --output_dir /tmp/bllm_cli_ckpt --print_sample_iter 1000 --save_ckpt_freq 0 --skip_final_save --no_plot --sample_tokens 50"
timeout -k 10 700 python -u main.py $ARGS --max_steps 61 --eval_freq 20 --metrics_file $O/metrics.jsonl > $O/main.log 2>&1 || { tail -20 $O/main.log; exit 3; }
grep -E "Step" $O/main.log | tail -4
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 5; }
tail -1 $O/bench.log > $O/bench.json
grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' $O/bench.json
