# Padded-vocabulary fused head: model / CE GPU tests, GPT-2 bench, hipBLASLt per-kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/head
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_training_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "model or ce or head or parity or determin" > gpurun_out/head/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/head/tests.log; exit 3; }
tail -2 gpurun_out/head/tests.log
timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/head/gpt2_1.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/head/gpt2_2.log 2>&1 || exit 5
grep -o '"value": [0-9.]*' gpurun_out/head/gpt2_*.log
python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --set kgrep=Cijk --tag head_prof > /dev/null 2>&1 || exit 6
cat gpurun_out/head_prof/kstats.log; head -12 gpurun_out/head_prof/breakdown.log
