# TunableOp tuning runs for the GPT-2 and Llama-2-7B presets (progress printed so the run never
# looks idle), then interleaved A/B of each tuned CSV against the heuristic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/tune
export PYTORCH_TUNABLEOP_VERBOSE=1
timeout -k 10 900 python -u bench.py --preset gpt2_774m_ddp --steps 1 --warmup 1 --tunableop_tune gpurun_out/tune/gpt2.csv 2>&1 | tee gpurun_out/tune/tune_gpt2.log | grep --line-buffered -c "" > /dev/null || exit 3
unset PYTORCH_TUNABLEOP_VERBOSE
ls gpurun_out/tune
for i in 1 2; do
timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 --tunableop none > gpurun_out/tune/gpt2_base_$i.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 --tunableop gpurun_out/tune/gpt20.csv > gpurun_out/tune/gpt2_tuned_$i.log 2>&1 || exit 5
done
grep -o '"value": [0-9.]*' gpurun_out/tune/gpt2_*.log
