# hd-64 dK/dV: separate vs dual LDS images, GPT-2 774M B=24 with and without dropout, alternated
# in separate processes (the staging choice is read once per process).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hd64b
S=gpt2-774M-B24,gpt2-774M-B24-nodrop,llama3.2-1B-B24
for i in 1 2 3; do
  timeout -k 10 120 python3 tools/bench_attn.py --shapes $S --iters 30 > gpurun_out/hd64b/sep_$i.log 2>&1 && \
  BLLM_ATTN_KV_DUAL=1 timeout -k 10 120 python3 tools/bench_attn.py --shapes $S --iters 30 > gpurun_out/hd64b/dual_$i.log 2>&1 || exit 1
done
