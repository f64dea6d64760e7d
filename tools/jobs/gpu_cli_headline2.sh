# CLI headline after the tok/s window fix (eval excluded): 61 steps, eval every 20; then a traced
# 12-step run for the GPU idle gaps with forward-pass indices; then bench.py on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/cli2
ARGS="--model llama3 --num_params 8B --run_type multi_gpu --use_fsdp --use_actv_ckpt --actv_ckpt_mode auto --data_type bf16 --batch_size 40 --synthetic_data --synthetic_mb 4 --n_epochs 1 --data_dir /tmp/bllm_cli_gutenberg --output_dir /tmp/bllm_cli_ckpt --print_sample_iter 1000 --save_ckpt_freq 0 --skip_final_save --no_plot --sample_tokens 50"
timeout -k 10 700 python -u main.py $ARGS --max_steps 61 --eval_freq 20 --metrics_file gpurun_out/cli2/metrics.jsonl > gpurun_out/cli2/main.log 2>&1 || { tail -20 gpurun_out/cli2/main.log; exit 3; }
grep -E "Step|auto" gpurun_out/cli2/main.log | tail -6
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/cli2/tr -o run -- python3 -u main.py $ARGS --max_steps 12 --eval_freq 5 > gpurun_out/cli2/traced.log 2>&1 || { tail -20 gpurun_out/cli2/traced.log; exit 4; }
timeout -k 10 120 python tools/gaps.py "$(find gpurun_out/cli2/tr -name '*.db' -print -quit)" --top 30 > gpurun_out/cli2/gaps.txt 2>&1
cat gpurun_out/cli2/gaps.txt
rm -rf gpurun_out/cli2/tr
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/cli2/bench.log 2>&1 || { tail -20 gpurun_out/cli2/bench.log; exit 5; }
tail -1 gpurun_out/cli2/bench.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*'
bash tools/jobs/gpu_gemm_pmc.sh
