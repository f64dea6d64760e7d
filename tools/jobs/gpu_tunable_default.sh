# Headline with the TunableOp CSV on by default vs --tunableop none (interleaved), plus the bench
# world-2 rehearsal test on the preset path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/tod
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/tod/default_$i.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --tunableop none > gpurun_out/tod/none_$i.log 2>&1 || exit 4
done
grep -o '"value": [0-9.]*\|"gemm_tuning": [^,]*' gpurun_out/tod/*.log
timeout -k 10 500 python -u -m pytest tests/test_engines_gpu.py tests/test_kernels_gpu.py -k "engines or bench or lora_model" -x -q --timeout 450 --timeout-method thread -p no:cacheprovider > gpurun_out/tod/engines.log 2>&1 || { tail -20 gpurun_out/tod/engines.log; exit 5; }
tail -1 gpurun_out/tod/engines.log
