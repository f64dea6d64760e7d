# Forward-layout and dX-layout GEMMs: hipBLASLt (both weight storage orders) vs the MFMA kernel
# (csrc/gemm_wgrad.hip, K-contiguous A) — decides whether epilogue-fused GEMMs can pay.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_dgrad.py --forward --tokens 40960 --models llama3_8b > gpurun_out/fwdgemm.log 2>&1 && \
timeout -k 10 300 python tools/bench_dgrad.py --tokens 40960 --models llama3_8b >> gpurun_out/fwdgemm.log 2>&1 && \
timeout -k 10 300 python tools/bench_dgrad.py --forward --tokens 24576 --models gpt2_774m >> gpurun_out/fwdgemm.log 2>&1 && \
timeout -k 10 300 python tools/bench_dgrad.py --tokens 24576 --models gpt2_774m >> gpurun_out/fwdgemm.log 2>&1
