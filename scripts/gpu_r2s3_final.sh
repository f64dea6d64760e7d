# Round-2 session-3 final validation: whole GPU suite, smoke, default bench, Llama-2 preset
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final_gpu_tests.log 2>&1 || { tail -30 gpurun_out/final_gpu_tests.log; exit 1; }
tail -2 gpurun_out/final_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -30 gpurun_out/final_smoke.log; exit 1; }
cat gpurun_out/final_smoke.log | grep smoke
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/final_bench.log 2>&1 || { tail -30 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log | cut -c1-300
timeout -k 10 600 python -u bench.py --preset llama2_7b_fsdp_mp --steps 10 --warmup 3 > gpurun_out/final_bench_llama2.log 2>&1 || { tail -30 gpurun_out/final_bench_llama2.log; exit 1; }
tail -1 gpurun_out/final_bench_llama2.log | cut -c1-300
