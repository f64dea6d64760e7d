# Where the CLI's extra ~0.4 s/step goes (the kernels per step equal bench.py's): loader wait and
# allocator retries in the metrics JSONL, with the loader in-process and the sampler without
# HIP-graph capture as variants.  Then the attention PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/clidiag
cli() {  # name, extra args...
  local name=$1; shift
  timeout -k 10 400 python -u main.py --model llama3 --num_params 8B --run_type multi_gpu --use_fsdp --use_actv_ckpt \
    --actv_ckpt_mode auto --data_type bf16 --batch_size 40 --synthetic_data --synthetic_mb 2.5 --n_epochs 1 \
    --data_dir /tmp/bllm_cli_gutenberg --output_dir /tmp/bllm_cli_ckpt --max_steps 41 --eval_freq 20 \
    --print_sample_iter 1000 --save_ckpt_freq 0 --skip_final_save --no_plot --sample_tokens 20 \
    --metrics_file gpurun_out/clidiag/$name.jsonl "$@" > gpurun_out/clidiag/$name.log 2>&1 || { tail -20 gpurun_out/clidiag/$name.log; exit 3; }
  echo "== $name"; cat gpurun_out/clidiag/$name.jsonl | python3 -c "import sys,json; [print(r['step'], r['tokens_per_s'], r.get('data_wait_s'), r.get('alloc_retries')) for r in map(json.loads, sys.stdin)]"
}
cli default
cli workers0 --num_workers 0
BLLM_DECODE_GRAPH=0 cli nograph
bash tools/jobs/gpu_attn_pmc.sh
