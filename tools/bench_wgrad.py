#!/usr/bin/env python3
"""dW GEMM micro-benchmark (GPU): the token-major MFMA kernel (csrc/gemm_wgrad.hip,
``ops.wgrad_gemm_``) vs hipBLASLt (``torch.mm(x^T, dy)`` into the transposed view, the previous
path) on the weight-gradient shapes of the benchmark models at 16,384 tokens.
Random [-1, 1) operands (zero-filled data inflates MFMA clocks).  Prints one JSON line per shape.
Usage: python tools/bench_wgrad.py [--tokens 16384] [--iters 10]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402

SHAPES = {
    "llama3_8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
                  ("head", 128256, 4096)],
    "llama32_1b": [("qkv", 3072, 2048), ("o", 2048, 2048), ("gate_up", 16384, 2048), ("down", 2048, 8192)],
    "gpt2_774m": [("qkv", 3840, 1280), ("o", 1280, 1280), ("fc1", 5120, 1280), ("fc2", 1280, 5120),
                  ("head_padded", 50432, 1280)],
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
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--models", default="llama3_8b,gpt2_774m,llama32_1b")
    ap.add_argument("--rounds", type=int, default=3, help="interleaved rounds (median reported)")
    ap.add_argument("--only", default="", help="comma list of gemm names to run")
    ap.add_argument("--no_hipblaslt", action="store_true", help="time only our kernel (profiling runs)")
    ap.add_argument("--variants", default="",
                    help="extra MFMA arms 'name:VAR=v,VAR2=v;name2:...' timed interleaved with the default "
                         "(kernel knobs read per launch)")
    a = ap.parse_args()
    ops.load_ext(required=True)
    Nt = a.tokens
    for model in a.models.split(","):
        for name, out_f, in_f in SHAPES[model]:
            if a.only and name not in a.only.split(","):
                continue
            dy = (torch.rand(Nt, out_f, device="cuda") * 2 - 1).to(torch.bfloat16)
            x = (torch.rand(Nt, in_f, device="cuda") * 2 - 1).to(torch.bfloat16)
            g0 = torch.empty(out_f, in_f, device="cuda", dtype=torch.bfloat16)
            g1 = torch.empty_like(g0)
            fl = 2.0 * Nt * out_f * in_f
            r = {"model": model, "gemm": name, "out_in": [out_f, in_f], "tokens": Nt}
            auto = ops.wgrad_splits(out_f, in_f, Nt)
            r["auto_splits"] = auto
            r["preferred"] = ops.wgrad_gemm_preferred(out_f, in_f)
            times = {}
            for _ in range(a.rounds):  # interleaved rounds in one process (variance correlated)
                if not a.no_hipblaslt:
                    times.setdefault("hipblaslt_us", []).append(
                        timeit(lambda: torch.mm(x.t(), dy, out=g0.t()), a.iters))
                times.setdefault("mfma_us", []).append(
                    timeit(lambda: ops.wgrad_gemm_(dy, x, g1, False, auto), a.iters))
                for vd in filter(None, a.variants.split(";")):
                    vname, kv = vd.split(":", 1)
                    env = dict(e.split("=") for e in kv.split(",") if e)
                    os.environ.update(env)
                    times.setdefault(f"{vname}_us", []).append(
                        timeit(lambda: ops.wgrad_gemm_(dy, x, g1, False, auto), a.iters))
                    for k_ in env:
                        os.environ.pop(k_)
            for k, ts in times.items():
                r[k] = sorted(ts)[len(ts) // 2]
            g1.zero_()
            ops.wgrad_gemm_(dy, x, g1, False, auto)
            torch.cuda.synchronize()
            if not a.no_hipblaslt:
                r["max_rel_err_vs_hipblaslt"] = round(((g1.float() - g0.float()).abs().max()
                                                       / g0.float().abs().max()).item(), 5)
            for k in list(r):
                if k.endswith("_us"):
                    r[k.replace("_us", "_tflops")] = round(fl / r[k] / 1e6, 1)
                    r[k] = round(r[k], 1)
            print(json.dumps(r), flush=True)
            del dy, x, g0, g1
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
