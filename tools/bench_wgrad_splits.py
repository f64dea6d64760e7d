#!/usr/bin/env python3
"""dW kernel split-K sweep at the GPT2-774M shapes (65,536 tokens): us per call for each split
count vs the one ``ops.wgrad_plan`` picks.  One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402

ops.load_ext(required=True)
TOK = 65536
SHAPES = [("qkv", 3840, 1280), ("o", 1280, 1280), ("fc1", 5120, 1280), ("fc2", 1280, 5120)]


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for name, O, I in SHAPES:
    dy = (torch.rand(TOK, O, device="cuda") * 2 - 1).to(torch.bfloat16)
    x = (torch.rand(TOK, I, device="cuda") * 2 - 1).to(torch.bfloat16)
    c = torch.empty(O, I, device="cuda", dtype=torch.bfloat16)
    row = {"shape": name, "plan": list(ops.wgrad_plan(O, I, TOK))}
    row["plan_us"] = round(timeit(lambda: ops.wgrad_gemm_(dy, x, c)), 1)
    for S in (1, 2, 3, 4, 5, 6, 8, 10, 12, 16):
        row[f"S{S}"] = round(timeit(lambda: ops.wgrad_gemm_(dy, x, c, splits=S)), 1)
    print(json.dumps(row), flush=True)
