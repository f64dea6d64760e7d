# lora_head_bwd_ numerics, then per-kernel time (main kernel + the two fixed-order partial sums)
# (historical: the BLLM_LHB_DEPTH / BLLM_LHB_WG knobs this sweeps were removed after it; depth 4 and
# 512 workgroups are fixed in csrc/lora.hip -- the script documents how profiles/r5/lora_head/sweep*.txt were made)
# and the one-chunk microbench per prefetch depth
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/lorahead/prof; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "lora_head" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O -o run -- python3 tools/prof_lora_head.py > $O/log.txt 2>&1 || { tail -20 $O/log.txt; exit 4; }
for d in 2 4; do for wg in 512 768; do
  echo "depth=$d wg=$wg $(BLLM_LHB_DEPTH=$d BLLM_LHB_WG=$wg timeout -k 10 120 python -u tools/bench_head_u.py 2>/dev/null | tail -1)" || exit 5
done; done | tee $O/sweep.txt
