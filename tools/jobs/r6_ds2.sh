# Stored-dS backward v2 (stores left in flight by counted waits; dq_ds ring variants) and the
# pipelined forward body: numerics, then same-process A/Bs
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6ds2
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "stored_ds or test_flash_attention" --timeout 300 --timeout-method thread > gpurun_out/r6ds2/tests.log 2>&1 || { tail -40 gpurun_out/r6ds2/tests.log; exit 3; }
tail -2 gpurun_out/r6ds2/tests.log
BLLM_FWD_PIPE=1 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "test_flash_attention and not stored_ds" --timeout 300 --timeout-method thread > gpurun_out/r6ds2/tests_pipe.log 2>&1 || { tail -40 gpurun_out/r6ds2/tests_pipe.log; exit 4; }
tail -2 gpurun_out/r6ds2/tests_pipe.log
S=llama3-8B-B40,gpt2-774M-B64,gpt2-774M-B64-nodrop,llama3.2-1B-B24
timeout -k 10 300 python -u tools/bench_attn.py --shapes $S --env_ab BLLM_FWD_PIPE > gpurun_out/r6ds2/fwd_pipe.jsonl 2>&1 || { tail -5 gpurun_out/r6ds2/fwd_pipe.jsonl; exit 5; }
grep '"ab"' gpurun_out/r6ds2/fwd_pipe.jsonl
timeout -k 10 300 python -u tools/bench_attn.py --shapes $S --bwd_env_ab BLLM_DQDS=0,1,2 --store_ds > gpurun_out/r6ds2/dqds.jsonl 2>&1 || { tail -5 gpurun_out/r6ds2/dqds.jsonl; exit 6; }
grep '"ab"' gpurun_out/r6ds2/dqds.jsonl
timeout -k 10 300 python -u tools/bench_attn.py --shapes $S --ds_ab > gpurun_out/r6ds2/ds_ab.jsonl 2>&1 || { tail -5 gpurun_out/r6ds2/ds_ab.jsonl; exit 7; }
grep store_ds gpurun_out/r6ds2/ds_ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6ds2/prof -o run -- python3 -u tools/bench_attn.py --shapes llama3-8B-B40,gpt2-774M-B64 --iters 5 > gpurun_out/r6ds2/prof.log 2>&1 || { tail -5 gpurun_out/r6ds2/prof.log; exit 8; }
timeout -k 10 300 python -u tools/bench_attn.py --shapes llama3-8B-B40,gpt2-774M-B64,llama3.2-1B-B24 --bwd_env_ab BLLM_BWD_PIPE=0,1 > gpurun_out/r6ds2/bpipe.jsonl 2>&1 || { tail -5 gpurun_out/r6ds2/bpipe.jsonl; exit 9; }
grep '"ab"' gpurun_out/r6ds2/bpipe.jsonl
BLLM_BWD_PIPE=1 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "test_flash_attention" --timeout 300 --timeout-method thread > gpurun_out/r6ds2/tests_bpipe.log 2>&1 || { tail -40 gpurun_out/r6ds2/tests_bpipe.log; exit 10; }
tail -2 gpurun_out/r6ds2/tests_bpipe.log
