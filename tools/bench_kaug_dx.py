#!/usr/bin/env python3
"""K-augmented LoRA dX GEMMs (GPU): [dx_W | u | 0] = dy . [W^T ; Bd ; 0]^T at the Llama-3.2-1B
block shapes (38,400 tokens) vs the base width alone, to catch hipBLASLt kernel-selection cliffs
on the augmented output width (as the LM head showed).  One JSON line per group."""
import json

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
    M = 38400
    for name, K_out, n_in, pad in (("qkv", 3072, 2048, 64), ("gate_up", 16384, 2048, 64), ("down", 2048, 8192, 64),
                                   ("qkv_fwd", 2112, 3072, 0), ("gate_up_fwd", 2112, 16384, 0), ("down_fwd", 8256, 2048, 0)):
        r = {"group": name, "M": M, "K": K_out}
        dy = (torch.rand(M, K_out, device="cuda") * 2 - 1).to(torch.bfloat16)
        for tag, n in (("base", n_in), ("aug", n_in + pad)):
            if pad == 0 and tag == "aug":
                continue
            wt = (torch.rand(n, K_out, device="cuda") * 2 - 1).to(torch.bfloat16)
            out = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
            ms = timeit(lambda: torch.mm(dy, wt.t(), out=out))
            r[f"{tag}_N"] = n
            r[f"{tag}_ms"] = round(ms, 3)
            r[f"{tag}_tflops"] = round(2 * M * n * K_out / ms / 1e9, 1)
            del wt, out
        print(json.dumps(r), flush=True)
        del dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
