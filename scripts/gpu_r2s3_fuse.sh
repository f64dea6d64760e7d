set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "swiglu or rope or flash_attention_bwd_fused or model or deterministic or lora" > gpurun_out/fuse_tests.log 2>&1 \
 && tail -2 gpurun_out/fuse_tests.log \
 && timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_fuse.log 2>&1 \
 && tail -1 gpurun_out/bench_fuse.log \
 && timeout -k 10 600 python -u bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/bench_fuse_lora.log 2>&1 \
 && tail -1 gpurun_out/bench_fuse_lora.log
