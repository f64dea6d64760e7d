# End-to-end A/B of the forward epilogue fusions on csrc/gemm_nt.hip (SwiGLU, RoPE on the
# headline; bias + GELU on GPT-2), each arm run twice, interleaved; plus the micro A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/fused
timeout -k 10 200 python -u tools/bench_gemm_nt.py --swiglu --rounds 3 > gpurun_out/fused/micro.jsonl 2>&1 || { tail -5 gpurun_out/fused/micro.jsonl; exit 3; }
cat gpurun_out/fused/micro.jsonl
hl() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/fused/$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/fused/$name.log; exit 4; }
  echo "$name $(grep -o '"value": [0-9.]*' gpurun_out/fused/$name.log) $(grep -o '"sclk_mhz_avg": [0-9.]*' gpurun_out/fused/$name.log)"
}
for i in 1 2; do
hl base_$i BLLM_X=0
hl swiglu_rope_$i BLLM_FUSED_SWIGLU=1 BLLM_FUSED_ROPE=1
done
hl swiglu_1 BLLM_FUSED_SWIGLU=1
hl rope_1 BLLM_FUSED_ROPE=1
g2() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 20 --warmup 5 > gpurun_out/fused/$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/fused/$name.log; exit 5; }
  echo "$name $(grep -o '"value": [0-9.]*' gpurun_out/fused/$name.log) $(grep -o '"sclk_mhz_avg": [0-9.]*' gpurun_out/fused/$name.log)"
}
for i in 1 2; do
g2 gpt2_base_$i BLLM_X=0
g2 gpt2_gelu_$i BLLM_FUSED_GELU=1
done
