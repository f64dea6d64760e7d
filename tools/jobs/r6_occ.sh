# hd-64 dK/dV (forward keep mask) at 3 waves per SIMD (launch bound 3, 168 VGPRs) vs 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6occ
BLLM_ATT_OCC3=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "keep_mask" --timeout 200 --timeout-method thread > gpurun_out/r6occ/tests.log 2>&1 || { tail -30 gpurun_out/r6occ/tests.log; exit 3; }
tail -1 gpurun_out/r6occ/tests.log
timeout -k 10 300 python -u tools/bench_attn.py --shapes gpt2-774M-B64,gpt2-774M-B24,gpt2-774M --bwd_env_ab BLLM_ATT_OCC3=0,2 > gpurun_out/r6occ/ab.jsonl 2>&1 || { tail -5 gpurun_out/r6occ/ab.jsonl; exit 4; }
grep '"ab"' gpurun_out/r6occ/ab.jsonl
