# A/B: non-temporal output stores in the dW kernel epilogue (BLLM_EXP_NT=1) vs plain stores.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/nt
timeout -k 10 300 python tools/bench_wgrad.py --models llama3_8b,gpt2_774m --tokens 40960 --rounds 3 > gpurun_out/nt/wgrad_off.jsonl 2>&1 || exit 3
BLLM_EXP_NT=1 timeout -k 10 300 python tools/bench_wgrad.py --models llama3_8b,gpt2_774m --tokens 40960 --rounds 3 > gpurun_out/nt/wgrad_on.jsonl 2>&1 || exit 4
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/nt/hl_off_$i.log 2>&1 || exit 5
BLLM_EXP_NT=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/nt/hl_on_$i.log 2>&1 || exit 6
done
grep -o '"value": [0-9.]*' gpurun_out/nt/hl_*.log
