#!/usr/bin/env python3
"""Norm backward (with the residual-gradient dx_acc) at the headline and GPT-2 shapes: us per call
and achieved HBM bandwidth (dy, x, dx_acc read + dx written)."""
import json
import sys
import torch
sys.path.insert(0, '.')
from building_llm_from_scratch_amd import ops
ops.load_ext(required=True)


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


out = {}
for name, N, d, ln in (("rms_llama3_8b", 40960, 4096, False), ("ln_gpt2_774m", 65536, 1280, True)):
    x = torch.randn(N, d, device="cuda").to(torch.bfloat16)
    dy = torch.randn(N, d, device="cuda").to(torch.bfloat16)
    acc = torch.randn(N, d, device="cuda").to(torch.bfloat16)
    w = torch.randn(d, device="cuda").to(torch.bfloat16)
    if ln:
        b = torch.randn(d, device="cuda").to(torch.bfloat16)
        _, mean, rstd = ops.layernorm_fwd(x, w, b, 1e-5)
        fn = lambda: ops.layernorm_bwd(dy, x, w, mean, rstd, dx_acc=acc)  # noqa: E731
    else:
        _, rstd = ops.rmsnorm_fwd(x, w, 1e-5)
        fn = lambda: ops.rmsnorm_bwd(dy, x, w, rstd, dx_acc=acc)  # noqa: E731
    t = timeit(fn)
    out[name] = {"us": round(t, 1), "TBps": round(4 * N * d * 2 / t / 1e6, 2)}
print(json.dumps(out))
