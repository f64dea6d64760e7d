# norm backward with the next row's loads in flight (this build) vs the previous build (_C_ref.so):
# norm GPU tests, kernel ABAB (tools/bench_norm_bwd.py), GPT2-774M preset ABAB
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6normpf
P=building_llm_from_scratch_amd
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "norm or layernorm or gpt2" > gpurun_out/r6normpf/tests.log 2>&1 || { tail -40 gpurun_out/r6normpf/tests.log; exit 5; }
tail -1 gpurun_out/r6normpf/tests.log
cp $P/_C.so /tmp/_C_new.so
for arm in new ref new ref; do
  if [ "$arm" = ref ]; then cp $P/_C_ref.so $P/_C.so; else cp /tmp/_C_new.so $P/_C.so; fi
  timeout -k 10 120 python -u tools/bench_norm_bwd.py > gpurun_out/r6normpf/k_$arm.json 2>&1 || { tail -20 gpurun_out/r6normpf/k_$arm.json; exit 6; }
  echo "kernel $arm $(tail -1 gpurun_out/r6normpf/k_$arm.json)"
done
for arm in new ref new ref; do
  if [ "$arm" = ref ]; then cp $P/_C_ref.so $P/_C.so; else cp /tmp/_C_new.so $P/_C.so; fi
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --preset gpt2_774m_ddp > gpurun_out/r6normpf/g2_$arm.log 2>&1 || { tail -20 gpurun_out/r6normpf/g2_$arm.log; exit 7; }
  echo "gpt2 $arm $(tail -1 gpurun_out/r6normpf/g2_$arm.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
done
cp /tmp/_C_new.so $P/_C.so
