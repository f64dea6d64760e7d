# forward K-fragment prefetch A/B: variant 0 (prefetch) vs 3 (no prefetch), alternating processes
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pks
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "attn or flash or keep_mask" -x -q --timeout 120 --timeout-method thread > gpurun_out/pks/tests.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pks
S=llama3-8B-B24,llama3.2-1B-B24,gpt2-774M-B24,gpt2-774M-B24-nodrop
for i in 1 2 3; do
  BLLM_ATTN_FWD_VARIANT=0 timeout -k 10 120 python3 tools/bench_attn.py --shapes $S --iters 30 > gpurun_out/pks/v0_$i.log 2>&1 && \
  BLLM_ATTN_FWD_VARIANT=3 timeout -k 10 120 python3 tools/bench_attn.py --shapes $S --iters 30 > gpurun_out/pks/v3_$i.log 2>&1 || exit 1
done
