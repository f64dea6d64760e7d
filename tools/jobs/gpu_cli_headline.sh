# The headline configuration through the user-facing CLI (main.py -> Trainer), then bench.py on
# the same box; the steady-state tok/s of the CLI comes from its metrics JSONL (eval / sample /
# checkpoint phases excluded by the trainer's clock).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/cli
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py -x -q --timeout 280 --timeout-method thread > gpurun_out/cli/engines_gpu.log 2>&1 || { tail -30 gpurun_out/cli/engines_gpu.log; exit 3; }
tail -2 gpurun_out/cli/engines_gpu.log
timeout -k 10 700 python -u main.py --model llama3 --num_params 8B --run_type multi_gpu --use_fsdp --use_actv_ckpt \
  --actv_ckpt_mode auto --data_type bf16 --batch_size 40 --synthetic_data --synthetic_mb 4 --n_epochs 1 \
  --data_dir /tmp/bllm_cli_gutenberg --output_dir /tmp/bllm_cli_ckpt --max_steps 61 --eval_freq 20 \
  --print_sample_iter 1000 --save_ckpt_freq 0 --skip_final_save --no_plot --sample_tokens 50 \
  --metrics_file gpurun_out/cli/metrics.jsonl > gpurun_out/cli/main.log 2>&1 || { tail -30 gpurun_out/cli/main.log; exit 4; }
grep -E "Step|auto|adaptation|tok/s" gpurun_out/cli/main.log | tail -12
cat gpurun_out/cli/metrics.jsonl
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/cli/bench.log 2>&1 || { tail -20 gpurun_out/cli/bench.log; exit 5; }
tail -1 gpurun_out/cli/bench.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*'
