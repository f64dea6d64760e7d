#!/usr/bin/env python3
"""Head-GEMM K sweep (GPU): logits = [h | s t | 0] . [W | B^T | 0]^T for the Llama-3.2-1B LoRA head
(8192-row chunk, V = 128,256) at augmented K = 2048 + pad: hipBLASLt's kernel choice depends on
K, so the pad is picked by measurement.  Prints one JSON line per K."""
import json
import sys

import torch


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    rows, V = 8192, 128256
    for K in [int(k) for k in (sys.argv[1] if len(sys.argv) > 1 else "2048,2064,2112,2176,2240,2304").split(",")]:
        a = (torch.rand(rows, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(V, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        out = torch.empty(rows, V, device="cuda", dtype=torch.bfloat16)
        ms = timeit(lambda: torch.mm(a, w.t(), out=out))
        dl = (torch.rand(rows, V, device="cuda") * 2 - 1).to(torch.bfloat16)
        wt = w.t().contiguous().t()          # the dX operand as the fused head passes it (W^T copy)
        dha = torch.empty(rows, K, device="cuda", dtype=torch.bfloat16)
        ms_dx = timeit(lambda: torch.mm(dl, wt, out=dha))
        print(json.dumps({"K": K, "logits_ms": round(ms, 3), "logits_tflops": round(2 * rows * V * K / ms / 1e9, 1),
                          "dx_ms": round(ms_dx, 3), "dx_tflops": round(2 * rows * V * K / ms_dx / 1e9, 1)}), flush=True)
        del a, w, out, dl, wt, dha
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
