# norm backward row pipelining A/B (BLLM_NORM_BWD_PIPE, round 5; the switch and the pipelined
# kernel were removed after this measurement: profiles/r5/norm_bwd_pipe/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/normbwd; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "norm" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for p in 0 1 0 1; do
  echo "pipe=$p $(BLLM_NORM_BWD_PIPE=$p timeout -k 10 120 python -u tools/bench_norm_bwd.py 2>/dev/null | tail -1)" || exit 4
done | tee $O/micro.txt
for r in 1 2; do
  for p in 0 1; do
    BLLM_NORM_BWD_PIPE=$p timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 20 --warmup 5 > $O/g_${p}_$r.log 2>&1 || { tail -20 $O/g_${p}_$r.log; exit 5; }
    echo "gpt2 pipe=$p round=$r $(tail -1 $O/g_${p}_$r.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  done
done
