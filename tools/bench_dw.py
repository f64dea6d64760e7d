#!/usr/bin/env python3
"""Weight-gradient GEMM micro-benchmark (GPU): dW[out, in] = dY^T X with K = N tokens.

With N = 16384 tokens and small projections (GPT-2 d=1280, Llama-3.2-1B d=2048) the output has
only ~100-200 tiles of 256x256 for 256 CUs, each with a 16k-deep K loop, and hipBLASLt's default
kernel leaves the chip half idle.  This compares the single GEMM against explicit split-K
(batched GEMM over token chunks with fp32 partial outputs, then a fixed-order sum).
Usage: python tools/bench_dw.py [--tokens 16384]"""
import argparse
import json

import torch


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    a = ap.parse_args()
    N = a.tokens
    shapes = {"gpt2_qkv": (3840, 1280), "gpt2_o": (1280, 1280), "gpt2_fc1": (5120, 1280), "gpt2_fc2": (1280, 5120),
              "l1b_qkv": (3072, 2048), "l1b_o": (2048, 2048), "l1b_gu": (16384, 2048), "l1b_down": (2048, 8192),
              "l8b_o": (4096, 4096), "l8b_gu": (28672, 4096)}
    dt = torch.bfloat16
    for name, (o, i) in shapes.items():
        x = torch.randn(N, i, device="cuda", dtype=dt)
        dy = torch.randn(N, o, device="cuda", dtype=dt)
        gW = torch.empty(o, i, device="cuda", dtype=dt)
        fl = 2.0 * N * o * i
        r = {"shape": name, "out_in": [o, i]}
        r["mm_xT_dy_outT"] = timeit(lambda: torch.mm(x.t(), dy, out=gW.t()))
        r["mm_dyT_x"] = timeit(lambda: torch.mm(dy.t(), x, out=gW))
        for S in (2, 4, 8):
            xs, dys = x.view(S, N // S, i), dy.view(S, N // S, o)
            part = torch.empty(S, i, o, device="cuda", dtype=torch.float32)

            def f32(xs=xs, dys=dys, part=part):
                torch.bmm(xs.transpose(1, 2), dys, out_dtype=torch.float32, out=part)
                torch.sum(part, 0, out=gW.t())
            try:
                r[f"splitk{S}_f32"] = timeit(f32)
            except Exception as ex:  # noqa: BLE001
                r[f"splitk{S}_f32"] = str(ex)[:80]
            partb = torch.empty(S, i, o, device="cuda", dtype=dt)

            def b16(xs=xs, dys=dys, partb=partb):
                torch.bmm(xs.transpose(1, 2), dys, out=partb)
                torch.sum(partb, 0, dtype=torch.float32).to(dt)
            r[f"splitk{S}_bf16"] = timeit(b16)
        for k in list(r):
            if isinstance(r[k], float):
                r[k] = f"{r[k]:.0f}us/{fl / r[k] / 1e9:.0f}TF"
        print(json.dumps(r), flush=True)
        del x, dy, gW
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
