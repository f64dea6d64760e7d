# Pipelined attention forward: numerics tests, then same-process A/B of the forward at the
# headline / GPT-2 / Llama-3.2-1B shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/attnpipe
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "pipelined or deferred or (test_flash_attention and not keep and not long and not fp32 and not gqa and not rope and not small)" --timeout 280 --timeout-method thread > gpurun_out/attnpipe/tests.log 2>&1 || { tail -30 gpurun_out/attnpipe/tests.log; exit 3; }
tail -2 gpurun_out/attnpipe/tests.log
timeout -k 10 200 python -u tools/bench_attn.py --shapes llama3-8B-B40,llama3.2-1B-B24,gpt2-774M-B64-nodrop --env_ab BLLM_ATTN_PIPE > gpurun_out/attnpipe/ab.jsonl 2>&1 || { tail -5 gpurun_out/attnpipe/ab.jsonl; exit 4; }
grep '"ab"' gpurun_out/attnpipe/ab.jsonl
# the CLI headline run under a kernel trace: one training step's kernel classes + span (host gaps)
mkdir -p gpurun_out/cliprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/cliprof/rocprof -o run -- python3 -u main.py --model llama3 --num_params 8B --run_type multi_gpu --use_fsdp --use_actv_ckpt \
  --actv_ckpt_mode auto --data_type bf16 --batch_size 40 --synthetic_data --synthetic_mb 2 --n_epochs 1 \
  --data_dir /tmp/bllm_cli_gutenberg --output_dir /tmp/bllm_cli_ckpt --max_steps 8 --eval_freq 4 \
  --print_sample_iter 1000 --save_ckpt_freq 0 --skip_final_save --no_plot --sample_tokens 20 > gpurun_out/cliprof/main.log 2>&1 || { tail -20 gpurun_out/cliprof/main.log; exit 5; }
timeout -k 10 120 python tools/step_breakdown.py "$(find gpurun_out/cliprof/rocprof -name '*.db' -print -quit)" > gpurun_out/cliprof/breakdown.log 2>&1 || { tail gpurun_out/cliprof/breakdown.log; exit 6; }
head -30 gpurun_out/cliprof/breakdown.log
rm -rf gpurun_out/cliprof/rocprof
