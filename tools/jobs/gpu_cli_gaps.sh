# GPU idle gaps of the CLI headline run vs bench.py under a kernel trace (where the CLI's extra
# time per step goes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/cligaps
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/cligaps/cli -o run -- python3 -u main.py --model llama3 --num_params 8B --run_type multi_gpu --use_fsdp --use_actv_ckpt \
  --actv_ckpt_mode auto --data_type bf16 --batch_size 40 --synthetic_data --synthetic_mb 2 --n_epochs 1 \
  --data_dir /tmp/bllm_cli_gutenberg --output_dir /tmp/bllm_cli_ckpt --max_steps 8 --eval_freq 100 \
  --print_sample_iter 1000 --save_ckpt_freq 0 --skip_final_save --no_plot --sample_tokens 20 --num_workers 0 > gpurun_out/cligaps/cli.log 2>&1 || { tail -20 gpurun_out/cligaps/cli.log; exit 3; }
timeout -k 10 120 python tools/gaps.py "$(find gpurun_out/cligaps/cli -name '*.db' -print -quit)" --top 40 > gpurun_out/cligaps/cli_gaps.txt 2>&1
cat gpurun_out/cligaps/cli_gaps.txt
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/cligaps/bench -o run -- python3 -u bench.py --steps 4 --warmup 3 > gpurun_out/cligaps/bench.log 2>&1 || { tail -20 gpurun_out/cligaps/bench.log; exit 4; }
timeout -k 10 120 python tools/gaps.py "$(find gpurun_out/cligaps/bench -name '*.db' -print -quit)" --top 25 > gpurun_out/cligaps/bench_gaps.txt 2>&1
cat gpurun_out/cligaps/bench_gaps.txt
rm -rf gpurun_out/cligaps/cli gpurun_out/cligaps/bench
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/cligaps/smoke.log 2>&1 || { tail -20 gpurun_out/cligaps/smoke.log; exit 5; }
grep "smoke ok" gpurun_out/cligaps/smoke.log
