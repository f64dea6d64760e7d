# torch.profiler trace of two CLI training steps (host ops + runtime calls + kernels), summarised
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/clitrace
timeout -k 10 400 python -u main.py --model llama3 --num_params 8B --run_type multi_gpu --use_fsdp --use_actv_ckpt \
  --actv_ckpt_mode auto --data_type bf16 --batch_size 40 --synthetic_data --synthetic_mb 2 --n_epochs 1 \
  --data_dir /tmp/bllm_cli_gutenberg --output_dir /tmp/bllm_cli_trace --max_steps 10 --eval_freq 100 \
  --print_sample_iter 1000 --save_ckpt_freq 0 --skip_final_save --no_plot --sample_tokens 20 \
  --profile_steps 6:7 > gpurun_out/clitrace/main.log 2>&1 || { tail -20 gpurun_out/clitrace/main.log; exit 3; }
timeout -k 10 200 python tools/trace_top.py /tmp/bllm_cli_trace/trace_steps6-7_rank0.json --top 40 > gpurun_out/clitrace/top.txt 2>&1 || { tail gpurun_out/clitrace/top.txt; exit 4; }
cat gpurun_out/clitrace/top.txt
bash tools/jobs/gpu_wgrad_map_ab.sh
bash tools/jobs/gpu_attn_cfg_ab.sh
