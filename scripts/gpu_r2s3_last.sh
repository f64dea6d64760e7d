set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/last_gpu_tests.log 2>&1 || { tail -30 gpurun_out/last_gpu_tests.log; exit 1; }
tail -1 gpurun_out/last_gpu_tests.log
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/last_smoke.log 2>&1 || { tail -30 gpurun_out/last_smoke.log; exit 1; }
grep smoke gpurun_out/last_smoke.log
