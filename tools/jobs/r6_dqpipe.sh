# dQ kernel: K / V fragments one step ahead + 16-B dQ stores (this build) vs the previous build
# (_C_ref.so), ABAB on one box; attention GPU tests on this build first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6dqpipe
P=building_llm_from_scratch_amd
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash_attention and not fp32_is_flash" > gpurun_out/r6dqpipe/tests.log 2>&1 || { tail -40 gpurun_out/r6dqpipe/tests.log; exit 5; }
tail -1 gpurun_out/r6dqpipe/tests.log
SH=llama3-8B-B40,llama3.2-1B-B24,gpt2-774M-B64,gpt2-774M-B64-nodrop
cp $P/_C.so /tmp/_C_new.so
for arm in new ref new ref; do
  if [ "$arm" = ref ]; then cp $P/_C_ref.so $P/_C.so; else cp /tmp/_C_new.so $P/_C.so; fi
  timeout -k 10 200 python -u tools/bench_attn.py --iters 20 --shapes $SH > gpurun_out/r6dqpipe/$arm.jsonl 2>&1 || { tail -20 gpurun_out/r6dqpipe/$arm.jsonl; exit 6; }
  echo "$arm $(grep '"fwd_ms"' gpurun_out/r6dqpipe/$arm.jsonl | grep -o '"shape": "[^"]*"\|"bwd_ms": [0-9.]*' | tr '\n' ' ')"
done
cp /tmp/_C_new.so $P/_C.so
