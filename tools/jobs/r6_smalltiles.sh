# GPT-2 (hd 64, dropout) forward tiling after the round's changes: 32-key tiles at 3 workgroups
# per CU (shipped for >= 2048 workgroups) vs 64-key tiles at 2; BLLM_FWD_SMALL is a temporary switch
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6small
timeout -k 10 300 python -u tools/bench_attn.py --iters 20 --env_ab BLLM_FWD_SMALL \
  --shapes gpt2-774M-B64,gpt2-774M-B24,gpt2-774M-B64-nodrop,llama3.2-1B-B24 > gpurun_out/r6small/ab.jsonl 2>&1 || { tail -20 gpurun_out/r6small/ab.jsonl; exit 6; }
grep '"ab"' gpurun_out/r6small/ab.jsonl | cut -c1-250
