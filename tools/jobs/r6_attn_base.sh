# Round-6 attention baseline: kernel times at the headline / GPT-2 shapes on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6base
timeout -k 10 300 python -u tools/bench_attn.py --shapes llama3-8B-B40,gpt2-774M-B64,gpt2-774M-B64-nodrop,llama3.2-1B-B24 > gpurun_out/r6base/attn.jsonl 2>&1 || { tail -5 gpurun_out/r6base/attn.jsonl; exit 3; }
cat gpurun_out/r6base/attn.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6base/prof -o run -- python3 -u tools/bench_attn.py --shapes llama3-8B-B40,gpt2-774M-B64 --iters 5 > gpurun_out/r6base/prof.log 2>&1 || { tail -5 gpurun_out/r6base/prof.log; exit 4; }
find gpurun_out/r6base/prof -name '*kernel_stats.csv' -exec cat {} \; | head -20
