set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "bias or gelu or model or deterministic or gpt2" > gpurun_out/gelu_tests.log 2>&1 || { tail -30 gpurun_out/gelu_tests.log; exit 1; }
tail -2 gpurun_out/gelu_tests.log
timeout -k 10 600 python -u bench.py --preset gpt2_774m_ddp --actv_ckpt full --steps 8 --warmup 3 > gpurun_out/bench_gpt2_full.log 2>&1 || { tail -20 gpurun_out/bench_gpt2_full.log; exit 1; }
tail -1 gpurun_out/bench_gpt2_full.log | cut -c1-250
BLLM_RECOMPUTE_FUSED=0 timeout -k 10 600 python -u bench.py --preset gpt2_774m_ddp --actv_ckpt full --steps 8 --warmup 3 > gpurun_out/bench_gpt2_full_off.log 2>&1 || exit 1
tail -1 gpurun_out/bench_gpt2_full_off.log | cut -c1-250
timeout -k 10 600 python -u bench.py --preset gpt2_774m_ddp --actv_ckpt full --steps 8 --warmup 3 > gpurun_out/bench_gpt2_full_b.log 2>&1 || exit 1
tail -1 gpurun_out/bench_gpt2_full_b.log | cut -c1-250
