# Llama-3.2-1B (hd 64, no dropout) forward: 32-key tiles (this build) vs 64-key tiles (_C_ref.so), ABAB x2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6small3
P=building_llm_from_scratch_amd
cp $P/_C.so /tmp/_C_new.so
for arm in new ref new ref new ref; do
  if [ "$arm" = ref ]; then cp $P/_C_ref.so $P/_C.so; else cp /tmp/_C_new.so $P/_C.so; fi
  timeout -k 10 120 python -u tools/bench_attn.py --iters 30 --shapes gpt2-124M,llama3.2-1B-B24 > gpurun_out/r6small3/$arm.jsonl 2>&1 || { tail -20 gpurun_out/r6small3/$arm.jsonl; exit 6; }
  echo "$arm $(grep '"fwd_ms"' gpurun_out/r6small3/$arm.jsonl | grep -o '"shape": "[^"]*"\|"fwd_tflops": [0-9.]*' | tr '\n' ' ')"
done
cp /tmp/_C_new.so $P/_C.so
