# K-augmented LoRA head: model-level GPU tests, LoRA preset bench, per-dispatch trace
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/lorahead
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_cli_gpu.py -k "lora or model" -x -q --timeout 200 --timeout-method thread > gpurun_out/lorahead/tests.log 2>&1 && \
timeout -k 10 300 python bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/lorahead/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/lorahead -o run -- python3 $R/bench.py --preset llama32_1b_lora_alpaca --steps 2 --warmup 2 > $R/gpurun_out/lorahead/prof.log 2>&1
