# Forward-layout GEMM: tile->XCD map, group depth and L2-prefetch distance A/B (each run has
# hipBLASLt interleaved in the same process as the control).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ntmap
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u tools/bench_gemm_nt.py --rounds 3 --models llama,gpt2 > gpurun_out/ntmap/$name.jsonl 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/ntmap/$name.jsonl; exit 3; }
  echo "== $name"; grep -o '"gemm": "[a-z_0-9]*".*tflops": [0-9.]*, "gemm_nt_us[^,]*, "gemm_nt_tflops": [0-9.]*' gpurun_out/ntmap/$name.jsonl | sed 's/"M_N_K[^]]*], //'
}
run base BLLM_X=0
run pf3 BLLM_NT_PF=3
run pf4 BLLM_NT_PF=4
run pf6 BLLM_NT_PF=6
run map1 BLLM_NT_MAP=1
run map2 BLLM_NT_MAP=2
run gm2 BLLM_NT_GM=2
run gm8 BLLM_NT_GM=8
run map1gm8 BLLM_NT_MAP=1 BLLM_NT_GM=8
run map2gm8 BLLM_NT_MAP=2 BLLM_NT_GM=8
