# attention forward: dropout 1/keep folded into the epilogue (this build) vs per-element (_C_ref.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6dropfold
P=building_llm_from_scratch_amd
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash_attention and not fp32_is_flash" > gpurun_out/r6dropfold/tests.log 2>&1 || { tail -40 gpurun_out/r6dropfold/tests.log; exit 5; }
tail -1 gpurun_out/r6dropfold/tests.log
SH=gpt2-774M-B64,gpt2-774M-B24,gpt2-774M-B64-nodrop
cp $P/_C.so /tmp/_C_new.so
for arm in new ref new ref; do
  if [ "$arm" = ref ]; then cp $P/_C_ref.so $P/_C.so; else cp /tmp/_C_new.so $P/_C.so; fi
  timeout -k 10 200 python -u tools/bench_attn.py --iters 20 --shapes $SH > gpurun_out/r6dropfold/$arm.jsonl 2>&1 || { tail -20 gpurun_out/r6dropfold/$arm.jsonl; exit 6; }
  echo "$arm $(grep '"fwd_ms"' gpurun_out/r6dropfold/$arm.jsonl | grep -o '"shape": "[^"]*"\|"fwd_tflops": [0-9.]*' | tr '\n' ' ')"
done
cp /tmp/_C_new.so $P/_C.so
