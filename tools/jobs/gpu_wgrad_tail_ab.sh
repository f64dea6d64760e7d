# dW split tail: numerics, micro A/B at the headline shapes, headline A/B (BLLM_WGRAD_TAIL=0/1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/wgtail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/wgtail/tests.log 2>&1 || { tail -40 gpurun_out/wgtail/tests.log; exit 3; }
tail -1 gpurun_out/wgtail/tests.log
timeout -k 10 200 python -u tools/bench_wgrad_tail.py > gpurun_out/wgtail/micro.jsonl 2>&1 || { tail -5 gpurun_out/wgtail/micro.jsonl; exit 4; }
cat gpurun_out/wgtail/micro.jsonl
for r in 1 2; do
  for f in 0 1; do
    BLLM_WGRAD_TAIL=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/wgtail/h${f}_$r.log 2>&1 || { tail -20 gpurun_out/wgtail/h${f}_$r.log; exit 5; }
    echo "tail=$f round=$r $(tail -1 gpurun_out/wgtail/h${f}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
