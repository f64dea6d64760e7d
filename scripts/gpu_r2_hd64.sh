# hd-64 attention backward (GPT-2 774M B=24 with dropout, Llama-3.2-1B B=24): per-kernel times of
# the dK/dV staging variants (env read once per process, so one process per variant).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hd64
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/hd64/$n -o run -- python3 tools/bench_attn.py --shapes gpt2-774M-B24,llama3.2-1B-B24 --iters 20 > gpurun_out/hd64/$n.log 2>&1
}
run default && run dual BLLM_ATTN_KV_DUAL=1 && run vlds BLLM_ATTN_KV_DUAL=1 BLLM_ATTN_KV_VLDS=1 && run v1 BLLM_ATTN_KV_VARIANT=1 && run q1 BLLM_ATTN_Q_VARIANT=1
