# LoRA head: u = dl B^T and dB = st^T dl in one pass over each dlogits chunk (lora_head_bwd_) --
# numerics, the one-chunk microbench, then the Llama-3.2-1B LoRA preset A/B (interleaved, one box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/lorahead; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "lora" tests/test_model_gpu.py -k "lora" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 120 python -u tools/bench_head_u.py > $O/micro.json 2>&1 || { tail -20 $O/micro.json; exit 4; }
cat $O/micro.json
for r in 1 2; do
  for f in 0 1; do
    BLLM_LORA_HEAD_FUSED=$f timeout -k 10 300 python -u bench.py --preset llama32_1b_lora_alpaca --steps 20 --warmup 5 > $O/b_${f}_$r.log 2>&1 || { tail -20 $O/b_${f}_$r.log; exit 5; }
    echo "fused=$f round=$r $(tail -1 $O/b_${f}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
