# Round-2: PyTorch TunableOp (all hipBLASLt + rocBLAS solutions timed per GEMM shape) for the headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTORCH_TUNABLEOP_ENABLED=1
export PYTORCH_TUNABLEOP_TUNING=1
export PYTORCH_TUNABLEOP_FILENAME=$GRAFT_REPO_ROOT/gpurun_out/tunableop_llama3_8b_b40.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40
export PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=10
timeout -k 10 900 python bench.py --steps 3 --warmup 2 > gpurun_out/r2_tunable_tune.log 2>&1 && \
export PYTORCH_TUNABLEOP_TUNING=0 && \
timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/r2_tunable_use.log 2>&1 && \
unset PYTORCH_TUNABLEOP_ENABLED && \
timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/r2_tunable_off.log 2>&1
