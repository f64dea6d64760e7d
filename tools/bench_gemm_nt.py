#!/usr/bin/env python3
"""Forward-layout GEMM A/B (GPU): y[M, N] = x[M, K] . W[N, K]^T, bf16, random operands.

hipBLASLt (torch.mm) vs the persistent kernel of csrc/gemm_nt.hip (ops.gemm_nt_), interleaved
in ONE process over --rounds, median per shape; the kernel's output checked against
hipBLASLt's (relative Frobenius).  Shapes: the Llama-3-8B projections at the bench's 40 x 1024
tokens and GPT2-774M's at 24 x 1024.  ``--swiglu``: gate/up + SwiGLU and QKV + RoPE, hipBLASLt +
the separate pass vs the fused epilogues.
Usage: python tools/bench_gemm_nt.py [--rounds 3 --iters 10 --models llama,gpt2 --only down]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402

SHAPES = {
    "llama": (40960, {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 28672), "down": (14336, 4096),
                      "head_chunk": (4096, 128256)}),
    "gpt2": (24576, {"qkv": (1280, 3840), "o": (1280, 1280), "fc1": (1280, 5120), "fc2": (5120, 1280)}),
}


def timeit(fn, iters):
    for _ in range(2):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--models", default="llama,gpt2")
    ap.add_argument("--arms", default="hipblaslt,gemm_nt")
    ap.add_argument("--only", default="", help="comma list of gemm names to run (e.g. gate_up)")
    ap.add_argument("--swiglu", action="store_true",
                    help="gate/up + SwiGLU and QKV + RoPE: hipBLASLt + separate pass vs the fused kernels")
    a = ap.parse_args()
    ops.load_ext(required=True)
    dt = torch.bfloat16
    if a.swiglu:
        return bench_fused(a)
    want = a.arms.split(",")
    for model in a.models.split(","):
        tokens, shapes = SHAPES[model]
        for name, (k, n) in shapes.items():
            if a.only and name not in a.only.split(","):
                continue
            m = 8192 if name == "head_chunk" else tokens   # the fused head runs 8192-row chunks
            x = torch.rand(m, k, device="cuda", dtype=dt) * 2 - 1
            w = (torch.rand(n, k, device="cuda", dtype=dt) * 2 - 1) * 0.05
            ref = torch.mm(x, w.t())
            y = torch.empty(m, n, device="cuda", dtype=dt)
            out = torch.empty(m, n, device="cuda", dtype=dt)
            fns = {"hipblaslt": lambda: torch.mm(x, w.t(), out=y), "gemm_nt": lambda: ops.gemm_nt_(x, w, out)}
            fns = {k_: f for k_, f in fns.items() if k_ in want}
            times = {kk: [] for kk in fns}
            for _ in range(a.rounds):
                for kk, fn in fns.items():
                    times[kk].append(timeit(fn, a.iters))
            fl = 2.0 * m * n * k
            r = {"model": model, "gemm": name, "M_N_K": [m, n, k]}
            for kk, ts in times.items():
                med = sorted(ts)[len(ts) // 2]
                r[kk + "_us"] = round(med * 1e3, 1)
                r[kk + "_tflops"] = round(fl / med / 1e9, 1)
            if "gemm_nt" in fns:
                r["rel_err_gemm_nt"] = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
            print(json.dumps(r), flush=True)
            del x, w, ref, out, y
            torch.cuda.empty_cache()


def bench_fused(a):
    dt = torch.bfloat16
    for model, (tokens, K, F) in {"llama": (40960, 4096, 14336), "llama32_1b": (40960, 2048, 8192)}.items():
        x = torch.rand(tokens, K, device="cuda", dtype=dt) * 2 - 1
        w = (torch.rand(2 * F, K, device="cuda", dtype=dt) * 2 - 1) * 0.05
        gu = torch.empty(tokens, 2 * F, device="cuda", dtype=dt)

        def sep():
            torch.mm(x, w.t(), out=gu)
            return ops.swiglu_fwd(gu)
        fns = {"hipblaslt+swiglu_fwd": sep, "fused": lambda: ops.gemm_nt_swiglu(x, w)}
        times = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, fn in fns.items():
                times[k].append(timeit(fn, a.iters))
        ref = sep()
        r = {"model": model, "M_K_F": [tokens, K, F]}
        for k, ts in times.items():
            r[k + "_us"] = round(sorted(ts)[len(ts) // 2] * 1e3, 1)
        _, act = fns["fused"]()
        r["act_equal"] = bool(torch.equal(act, ref))
        print(json.dumps(r), flush=True)
        del x, w, gu
        torch.cuda.empty_cache()
    # QKV + RoPE: hipBLASLt GEMM + rope_ vs the fused persistent kernel (Llama-3-8B at 40 x 1024)
    tokens, K, H, G, hd, T = 40960, 4096, 32, 8, 128, 1024
    x = torch.rand(tokens, K, device="cuda", dtype=dt) * 2 - 1
    w = (torch.rand((H + 2 * G) * hd, K, device="cuda", dtype=dt) * 2 - 1) * 0.05
    cos, sin = ops.rope_tables(hd, T, 500000.0, None, device="cuda")
    q = torch.empty(tokens, w.shape[0], device="cuda", dtype=dt)

    def sep_r():
        torch.mm(x, w.t(), out=q)
        ops.rope_(q, cos, sin, T, H, G, hd)
    fns = {"hipblaslt+rope": sep_r, "fused_rope": lambda: ops.gemm_nt_rope(x, w, cos, sin, T, H, G, hd)}
    times = {k: [] for k in fns}
    for _ in range(a.rounds):
        for k, fn in fns.items():
            times[k].append(timeit(fn, a.iters))
    print(json.dumps({"model": "llama", "op": "qkv+rope", **{k + "_us": round(sorted(v)[len(v) // 2] * 1e3, 1)
                                                              for k, v in times.items()}}), flush=True)


if __name__ == "__main__":
    main()
