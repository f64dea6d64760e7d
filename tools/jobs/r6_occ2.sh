# hd-64 dQ (keep mask) and dropout forward at 4 waves per SIMD vs the shipped occupancy
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6occ2
BLLM_ATT_OCC=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "keep_mask or small_tiles" --timeout 200 --timeout-method thread > gpurun_out/r6occ2/tests.log 2>&1 || { tail -30 gpurun_out/r6occ2/tests.log; exit 3; }
tail -1 gpurun_out/r6occ2/tests.log
timeout -k 10 300 python -u tools/bench_attn.py --shapes gpt2-774M-B64,gpt2-774M-B24 --bwd_env_ab BLLM_ATT_OCC=0,3,4 --variants "occ4:BLLM_ATT_OCC=4" > gpurun_out/r6occ2/ab.jsonl 2>&1 || { tail -5 gpurun_out/r6occ2/ab.jsonl; exit 4; }
grep '"ab"\|fwd_tflops"' gpurun_out/r6occ2/ab.jsonl
