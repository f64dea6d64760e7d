# tall-block lora_down: LoRA kernel tests, then the LoRA Alpaca preset bench + per-dispatch trace
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/lora3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lora" -x -q --timeout 120 --timeout-method thread > gpurun_out/lora3/tests.log 2>&1 && \
timeout -k 10 300 python bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/lora3/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/lora3 -o run -- python3 $R/bench.py --preset llama32_1b_lora_alpaca --steps 2 --warmup 2 > $R/gpurun_out/lora3/prof.log 2>&1
