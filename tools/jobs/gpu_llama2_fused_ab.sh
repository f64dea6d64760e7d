# Llama-2-7B preset (no TunableOp table): fused SwiGLU / RoPE GEMM epilogues vs the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/l2fused; mkdir -p $O
for r in 1 2; do
  for v in base swiglu swiglu_rope; do
    case $v in base) E="";; swiglu) E="BLLM_FUSED_SWIGLU=1";; swiglu_rope) E="BLLM_FUSED_SWIGLU=1 BLLM_FUSED_ROPE=1";; esac
    env $E timeout -k 10 400 python -u bench.py --preset llama2_7b_fsdp_mp --steps 10 --warmup 3 > $O/${v}_$r.log 2>&1 || { tail -20 $O/${v}_$r.log; exit 5; }
    echo "$v round=$r $(tail -1 $O/${v}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
