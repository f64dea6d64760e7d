# TEMPORARY A/B of the hd-64 dQ tilings (BLLM_EXP_DQ) on the GPT-2 attention shapes, plus numerics.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/dq
for v in 0 1 2 3 4 0; do
BLLM_EXP_DQ=$v timeout -k 10 120 python tools/bench_attn.py --shapes gpt2-774M-B64,gpt2-774M-B64-nodrop,llama3.2-1B-B24 > gpurun_out/dq/v$v.jsonl 2>&1 || exit 3
echo "v$v $(grep -o '"shape": "[^"]*"\|"bwd_ms": [0-9.]*' gpurun_out/dq/v$v.jsonl | tr '\n' ' ')"
done
for v in 1 2 3 4; do
BLLM_EXP_DQ=$v timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "attn and 64" > gpurun_out/dq/t$v.log 2>&1 || { echo "tests v$v failed"; tail -5 gpurun_out/dq/t$v.log; exit 4; }
echo "tests v$v $(tail -1 gpurun_out/dq/t$v.log)"
done
