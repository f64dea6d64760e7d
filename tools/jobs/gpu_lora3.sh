# LoRA kernel tuning check: tests, micro-bench, preset bench, per-kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/l3
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "kaug or lora" > gpurun_out/l3/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/l3/tests.log; exit 3; }
tail -2 gpurun_out/l3/tests.log
timeout -k 10 200 python tools/bench_lora.py --iters 20 > gpurun_out/l3/bench_lora.jsonl 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/l3/lora_1.log 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/l3/lora_2.log 2>&1 || exit 6
grep -o '"value": [0-9.]*' gpurun_out/l3/lora_*.log
python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --set kgrep=lora --tag l3_prof > /dev/null 2>&1 || exit 7
cat gpurun_out/l3_prof/kstats.log; head -8 gpurun_out/l3_prof/breakdown.log
