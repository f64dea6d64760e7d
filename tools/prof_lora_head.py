#!/usr/bin/env python3
"""lora_head_bwd_ alone on one LoRA-head dlogits chunk (8192 x 128,256), for rocprofv3 --kernel-trace."""
import sys
import torch
sys.path.insert(0, '.')
from building_llm_from_scratch_amd import ops
ops.load_ext(required=True)
rows, V, r = 8192, 128256, 16
dl = (torch.rand(rows, V, device='cuda') * 2 - 1).to(torch.bfloat16)
B = (torch.rand(r, V, device='cuda') * 2 - 1).to(torch.bfloat16)
st = (torch.rand(rows, r, device='cuda') * 2 - 1).to(torch.bfloat16)
ub = torch.empty(rows, r, device='cuda', dtype=torch.bfloat16)
gB = torch.empty(r, V, device='cuda', dtype=torch.float32)
for _ in range(20):
    ops.lora_head_bwd_(dl, st, B, ub, gB, True)
torch.cuda.synchronize()
print("ok")
