# Attention forward tiling A/B: keys per tile x ring slots x workgroups per CU (read per launch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/attncfg
V="t32r3w2:BLLM_ATTN_FWD_CFG=32,3,2;t32r4w2:BLLM_ATTN_FWD_CFG=32,4,2;t32r2w3:BLLM_ATTN_FWD_CFG=32,2,3;t64r3w2:BLLM_ATTN_FWD_CFG=64,3,2;pipe:BLLM_ATTN_PIPE=1"
timeout -k 10 300 python -u tools/bench_attn.py --shapes llama3-8B-B40,llama3.2-1B-B24,gpt2-774M-B64,gpt2-774M-B64-nodrop --variants "$V" > gpurun_out/attncfg/ab.jsonl 2>&1 || { tail -5 gpurun_out/attncfg/ab.jsonl; exit 3; }
grep fwd_tflops gpurun_out/attncfg/ab.jsonl
