# GEMM layout bench at the bench's token count: default hipBLASLt heuristics vs TunableOp-tuned solutions.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
timeout -k 10 200 python tools/bench_gemm.py --tokens 16384 --iters 10 > gpurun_out/gemm_default.log 2>&1 && \
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/gemm%d.csv \
timeout -k 10 700 python tools/bench_gemm.py --tokens 16384 --iters 10 > gpurun_out/gemm_tuned.log 2>&1
