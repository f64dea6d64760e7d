# attention fwd / bwd at T = 4096 and 8192 (Llama-3-8B heads, GPT-2 heads): final tree vs the
# extension built from commit 621bfe1 (before the round's XCD order / store changes), ABAB
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6longctx
P=building_llm_from_scratch_amd
cp $P/_C.so /tmp/_C_after.so
for arm in after before after before; do
  if [ "$arm" = before ]; then cp $P/_C_before.so $P/_C.so; else cp /tmp/_C_after.so $P/_C.so; fi
  for T in 4096 8192; do
    timeout -k 10 200 python -u tools/bench_attn.py --iters 10 --T $T --shapes llama3-8B-B40,gpt2-774M-B64 > gpurun_out/r6longctx/${arm}_$T.jsonl 2>&1 || { tail -20 gpurun_out/r6longctx/${arm}_$T.jsonl; exit 5; }
    echo "$arm T=$T $(grep '"fwd_ms"' gpurun_out/r6longctx/${arm}_$T.jsonl | grep -o '"shape": "[^"]*"\|"fwd_tflops": [0-9.]*\|"bwd_ms": [0-9.]*' | tr '\n' ' ')"
  done
done
cp /tmp/_C_after.so $P/_C.so
