# LoRA K-augmentation + embedding backward check: targeted GPU tests, then LoRA / GPT-2 / headline
# benches, then a TunableOp tune + A/B on GPT-2.  Each step has its own limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/lk
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "kaug or lora or embedding" > gpurun_out/lk/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/lk/tests.log; exit 3; }
tail -2 gpurun_out/lk/tests.log
timeout -k 10 300 python -u bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/lk/lora.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/lk/gpt2.log 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/lk/headline.log 2>&1 || exit 6
grep -ho '"metric": "[^"]*", "value": [0-9.]*' gpurun_out/lk/*.log
timeout -k 10 600 python -u bench.py --preset gpt2_774m_ddp --steps 2 --warmup 1 --tunableop_tune gpurun_out/lk/gpt2.csv > gpurun_out/lk/tune_gpt2.log 2>&1 || exit 7
for i in 1 2; do
timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/lk/gpt2_base_$i.log 2>&1 || exit 8
timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 --tunableop gpurun_out/lk/gpt20.csv > gpurun_out/lk/gpt2_tuned_$i.log 2>&1 || exit 9
done
grep -o '"value": [0-9.]*' gpurun_out/lk/gpt2_*.log
python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --tag lk_prof_lora > /dev/null 2>&1 || exit 10
python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --tag lk_prof_gpt2 > /dev/null 2>&1 || exit 11
head -30 gpurun_out/lk_prof_lora/breakdown.log
