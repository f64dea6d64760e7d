set -o pipefail
mkdir -p gpurun_out
for u in 4 2 8 4; do
  BLLM_SWIGLU_U=$u timeout -k 10 200 python -u tools/bench_ew.py >> gpurun_out/swu.jsonl 2>&1 || exit 1
done
cat gpurun_out/swu.jsonl | grep env
