# CLI throughput by launch mode: mp.spawn (reference main.py path) vs torchrun with one rank,
# and the loader in-process; same box, same config (tok/s from the metrics JSONL)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/clilaunch
ARGS="--model llama3 --num_params 8B --run_type multi_gpu --use_fsdp --use_actv_ckpt --actv_ckpt_mode auto --data_type bf16 --batch_size 40 --synthetic_data --synthetic_mb 2 --n_epochs 1 --data_dir /tmp/bllm_cli_gutenberg --output_dir /tmp/bllm_cli_ckpt --max_steps 31 --eval_freq 15 --print_sample_iter 1000 --save_ckpt_freq 0 --skip_final_save --no_plot --sample_tokens 20"
summ() { python3 -c "import sys,json; [print('   ', r['step'], r['tokens_per_s'], r.get('data_wait_s')) for r in map(json.loads, open(sys.argv[1]))]" "$1"; }
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 main.py $ARGS --metrics_file gpurun_out/clilaunch/torchrun.jsonl > gpurun_out/clilaunch/torchrun.log 2>&1 || { tail -20 gpurun_out/clilaunch/torchrun.log; exit 3; }
echo "== torchrun"; summ gpurun_out/clilaunch/torchrun.jsonl
timeout -k 10 400 python -u main.py $ARGS --metrics_file gpurun_out/clilaunch/spawn.jsonl > gpurun_out/clilaunch/spawn.log 2>&1 || { tail -20 gpurun_out/clilaunch/spawn.log; exit 4; }
echo "== spawn"; summ gpurun_out/clilaunch/spawn.jsonl
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29562 main.py $ARGS --num_workers 0 --metrics_file gpurun_out/clilaunch/torchrun_w0.jsonl > gpurun_out/clilaunch/torchrun_w0.log 2>&1 || { tail -20 gpurun_out/clilaunch/torchrun_w0.log; exit 5; }
echo "== torchrun workers0"; summ gpurun_out/clilaunch/torchrun_w0.jsonl
bash tools/jobs/gpu_attn_cfg_ab.sh
