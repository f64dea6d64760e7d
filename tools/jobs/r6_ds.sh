# Stored-dS backward: numerics tests, then A/B vs the recomputing dQ kernel (+ deferred-store arm)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6ds
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "stored_ds" --timeout 300 --timeout-method thread > gpurun_out/r6ds/tests.log 2>&1 || { tail -40 gpurun_out/r6ds/tests.log; exit 3; }
tail -2 gpurun_out/r6ds/tests.log
timeout -k 10 300 python -u tools/bench_attn.py --shapes llama3-8B-B40,gpt2-774M-B64,gpt2-774M-B64-nodrop,llama3.2-1B-B24 --ds_ab > gpurun_out/r6ds/ab.jsonl 2>&1 || { tail -5 gpurun_out/r6ds/ab.jsonl; exit 4; }
grep store_ds gpurun_out/r6ds/ab.jsonl
BLLM_DS_DEFER=1 timeout -k 10 300 python -u tools/bench_attn.py --shapes llama3-8B-B40,gpt2-774M-B64 --ds_ab > gpurun_out/r6ds/ab_defer.jsonl 2>&1 || { tail -5 gpurun_out/r6ds/ab_defer.jsonl; exit 5; }
grep store_ds gpurun_out/r6ds/ab_defer.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6ds/prof -o run -- python3 -u tools/bench_attn.py --shapes llama3-8B-B40,gpt2-774M-B64 --iters 5 > gpurun_out/r6ds/prof.log 2>&1 || { tail -5 gpurun_out/r6ds/prof.log; exit 6; }
