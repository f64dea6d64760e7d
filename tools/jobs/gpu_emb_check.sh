# Embedding backward (two-pass) check: GPU tests, GPT-2 + headline benches, per-kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/emb
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "embedding or determinis or gpt2" > gpurun_out/emb/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/emb/tests.log; exit 3; }
tail -2 gpurun_out/emb/tests.log
timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/emb/gpt2.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/emb/headline.log 2>&1 || exit 5
grep -ho '"metric": "[^"]*", "value": [0-9.]*' gpurun_out/emb/*.log
python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --set kgrep=emb --tag emb_prof > /dev/null 2>&1 || exit 6
cat gpurun_out/emb_prof/kstats.log; head -16 gpurun_out/emb_prof/breakdown.log
