# ping-pong forward: numerics, A/B against the shipped kernel, per-phase s_memtime stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6pp
BLLM_ATT_PP=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash_attention and not bwd_fused_rope and not fp32_is_flash" > gpurun_out/r6pp/tests.log 2>&1 || { tail -40 gpurun_out/r6pp/tests.log; exit 5; }
tail -2 gpurun_out/r6pp/tests.log
timeout -k 10 300 python -u tools/bench_attn.py --iters 20 --env_ab BLLM_ATT_PP \
  --shapes llama3-8B-B40,llama3.2-1B-B24,gpt2-774M-B64,gpt2-774M-B64-nodrop > gpurun_out/r6pp/ab.jsonl 2>&1 || { tail -20 gpurun_out/r6pp/ab.jsonl; exit 6; }
grep '"ab"' gpurun_out/r6pp/ab.jsonl
BLLM_ATT_PP=2 timeout -k 10 120 python -u -c "
import torch, sys; sys.path.insert(0, '.')
from building_llm_from_scratch_amd import ops
ops.load_ext(required=True)
for B, H, G, hd in ((40, 32, 8, 128), (64, 20, 20, 64)):
    T = 1024
    qkv = torch.randn(B * T, (H + 2 * G) * hd, device='cuda', dtype=torch.bfloat16)
    for _ in range(2):
        ops.flash_attn_fwd(qkv, B, T, H, G, hd, True, 0.0, 1, 0)
    torch.cuda.synchronize()
    print('shape', B, H, G, hd, file=sys.stderr, flush=True)
" > gpurun_out/r6pp/stamps.log 2>&1 || { tail -20 gpurun_out/r6pp/stamps.log; exit 7; }
cat gpurun_out/r6pp/stamps.log | cut -c1-600
