#!/usr/bin/env python3
"""u = dl B^T over one LoRA-head dlogits chunk (8192 x 128,256): lora_down vs a hipBLASLt mm; and
u plus dB = st^T dl: hipBLASLt mm + lora_wgrad vs the one-pass lora_head_bwd_."""
import torch, json
def timeit(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3
import sys; sys.path.insert(0, '.')
from building_llm_from_scratch_amd import ops
ops.load_ext(required=True)
rows, V, r = 8192, 128256, 16
dl = (torch.rand(rows, V, device='cuda')*2-1).to(torch.bfloat16)
B = (torch.rand(r, V, device='cuda')*2-1).to(torch.bfloat16)
ub = torch.empty(rows, r, device='cuda', dtype=torch.bfloat16)
t1 = timeit(lambda: ops.lora_down_into(dl, [B], [0], [V], [0], r, 1.0, ub))
t2 = timeit(lambda: torch.mm(dl, B.t(), out=ub))
st = (torch.rand(rows, r, device='cuda')*2-1).to(torch.bfloat16)
gB = torch.empty(r, V, device='cuda', dtype=torch.float32)
def pair():
    torch.mm(dl, B.t(), out=ub)
    ops.lora_wgrad(st, dl, [gB], [0], [0], 1.0, accumulate=True)
t3 = timeit(pair)
t4 = timeit(lambda: ops.lora_wgrad(st, dl, [gB], [0], [0], 1.0, accumulate=True))
t5 = timeit(lambda: ops.lora_head_bwd_(dl, st, B, ub, gB, True))
print(json.dumps({"lora_down_us": round(t1,1), "hipblaslt_mm_us": round(t2,1), "lora_wgrad_us": round(t4,1),
                  "mm_plus_wgrad_us": round(t3,1), "lora_head_bwd_us": round(t5,1), "GB": rows*V*2/1e9}))
