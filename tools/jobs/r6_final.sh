# Round 6 tree on one box: headline bench (driver settings) with and
# without TORCH_NCCL_ENABLE_TIMING on the forced-comm path, presets, v15 breakdowns
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6final
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6final/headline.log 2>&1 || { tail -20 gpurun_out/r6final/headline.log; exit 5; }
echo "headline $(tail -1 gpurun_out/r6final/headline.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
# RCCL per-collective event timing cost on the forced-comm (N>1 code path) run, ABAB
for arm in 1 0 1 0; do
  TORCH_NCCL_ENABLE_TIMING=$arm timeout -k 10 300 python -u bench.py --force_comm --layers 8 --steps 10 --warmup 3 > gpurun_out/r6final/forced_timing$arm.log 2>&1 || { tail -20 gpurun_out/r6final/forced_timing$arm.log; exit 6; }
  echo "timing=$arm $(tail -1 gpurun_out/r6final/forced_timing$arm.log | grep -o '"ms_per_step": [0-9.]*')"
done
tail -1 gpurun_out/r6final/forced_timing1.log > gpurun_out/r6final/forced_timing1.json
timeout -k 10 300 python -u tools/bench_attn.py --shapes llama3-8B-B40,gpt2-774M-B64,gpt2-774M-B64-nodrop,llama3.2-1B-B24 > gpurun_out/r6final/attn.jsonl 2>&1 || { tail -5 gpurun_out/r6final/attn.jsonl; exit 7; }
cat gpurun_out/r6final/attn.jsonl | grep shape
# hd-64 dK/dV (forward keep mask) at 3 waves per SIMD vs 2
BLLM_ATT_OCC3=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "keep_mask" --timeout 200 --timeout-method thread > gpurun_out/r6final/occ_tests.log 2>&1 || { tail -30 gpurun_out/r6final/occ_tests.log; exit 8; }
tail -1 gpurun_out/r6final/occ_tests.log
timeout -k 10 300 python -u tools/bench_attn.py --shapes gpt2-774M-B64,gpt2-774M-B24,gpt2-774M --bwd_env_ab BLLM_ATT_OCC3=0,2 > gpurun_out/r6final/occ_ab.jsonl 2>&1 || { tail -5 gpurun_out/r6final/occ_ab.jsonl; exit 9; }
grep '"ab"' gpurun_out/r6final/occ_ab.jsonl
