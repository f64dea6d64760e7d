# attention GPU tests after the hd-64 dual default change, then the GPT-2 774M preset bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "attn or flash or keep_mask" -x -q --timeout 120 --timeout-method thread > gpurun_out/hd64c_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/hd64c_gpt2.log 2>&1
