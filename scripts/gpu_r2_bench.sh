# Round-2: GPU tests + new bench (FSDP engine at world 1, full ckpt) + presets + rocprof of the headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --profile > gpurun_out/r2_llama_full.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --actv_ckpt selective > gpurun_out/r2_llama_selective.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --actv_ckpt none > gpurun_out/r2_llama_none.log 2>&1 && \
timeout -k 10 300 python bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/r2_gpt2.log 2>&1 && \
timeout -k 10 300 python bench.py --preset llama32_1b_lora_alpaca --steps 20 --warmup 5 > gpurun_out/r2_lora_alpaca.log 2>&1 && \
timeout -k 10 300 python bench.py --preset llama2_7b_fsdp_mp --steps 10 --warmup 3 > gpurun_out/r2_llama2.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_r2.log 2>&1
