# Round-end validation: GPU tests, smoke, headline bench (local + torchrun/RCCL FSDP engine), GPT-2, LoRA, rocprof stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --profile > gpurun_out/llama.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/llama_torchrun.log 2>&1 && \
timeout -k 10 300 python bench.py --model GPT2 --num_params 774M --parallel ddp --steps 10 --warmup 3 > gpurun_out/gpt2.log 2>&1 && \
timeout -k 10 300 python bench.py --model llama3_2 --num_params 1B --lora_rank 16 --steps 10 --warmup 3 > gpurun_out/lora.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
