#!/usr/bin/env python3
"""t = x A_cat (LoRA down projection) on lora_down vs a skinny hipBLASLt mm, at the Llama-3.2-1B
LoRA block shapes (38,400 tokens).  One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402


def timeit(fn, iters=20):
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


def main():
    ops.load_ext(required=True)
    N = 38400
    for name, K, R in (("qkv", 2048, 48), ("gate_up", 2048, 32), ("down", 8192, 16), ("o", 2048, 16)):
        x = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        P = (torch.rand(R, K, device="cuda") * 0.1).to(torch.bfloat16)
        out = torch.empty(N, R, device="cuda", dtype=torch.bfloat16)
        t1 = timeit(lambda: ops.lora_down_into(x, [P], [0], [K], [0], R, 1.0, out))
        t2 = timeit(lambda: torch.mm(x, P.t(), out=out))
        print(json.dumps({"group": name, "K": K, "R": R, "lora_down_us": round(t1, 1), "mm_us": round(t2, 1),
                          "roof_us": round(N * K * 2 / 5e12 * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
