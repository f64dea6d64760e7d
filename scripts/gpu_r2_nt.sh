# NT (both K-contiguous) GEMM on the MFMA kernel: numerics, then forward-layout bench vs hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_nt or gemm_nn" -x -q --timeout 120 --timeout-method thread > gpurun_out/nt_tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_dgrad.py --forward --tokens 40960 --models llama3_8b > gpurun_out/nt_bench.log 2>&1 && \
timeout -k 10 300 python tools/bench_dgrad.py --forward --tokens 24576 --models gpt2_774m >> gpurun_out/nt_bench.log 2>&1
