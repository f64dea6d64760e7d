#!/usr/bin/env python3
"""LoRA weight gradients (dA = s x^T u, dB = s t^T dy) on lora_wgrad vs hipBLASLt GEMMs, at the
Llama-3.2-1B LoRA block shapes (38,400 tokens).  One JSON line per case."""
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
    N, bf = 38400, torch.bfloat16
    for name, K, r in (("dA_o", 2048, 16), ("dA_down", 8192, 16)):
        x = (torch.rand(N, K, device="cuda") * 2 - 1).to(bf)
        u = (torch.rand(N, r, device="cuda") * 2 - 1).to(bf)
        g = torch.empty(K, r, device="cuda", dtype=bf)
        t1 = timeit(lambda: ops.lora_wgrad(u, x, [g.t()], [0], [0], 0.5))
        t2 = timeit(lambda: torch.mm(x.t(), u, out=g))
        print(json.dumps({"case": name, "lora_wgrad_us": round(t1, 1), "mm_us": round(t2, 1)}), flush=True)
    for name, M, r in (("dB_o", 2048, 16), ("dB_gu_member", 8192, 16), ("dB_q", 2048, 16)):
        dy = (torch.rand(N, M, device="cuda") * 2 - 1).to(bf)
        t = (torch.rand(N, r, device="cuda") * 2 - 1).to(bf)
        g = torch.empty(r, M, device="cuda", dtype=bf)
        t1 = timeit(lambda: ops.lora_wgrad(t, dy, [g], [0], [0], 0.5))
        t2 = timeit(lambda: torch.mm(t.t(), dy, out=g))
        print(json.dumps({"case": name, "lora_wgrad_us": round(t1, 1), "mm_us": round(t2, 1)}), flush=True)


if __name__ == "__main__":
    main()
