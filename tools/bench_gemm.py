#!/usr/bin/env python3
"""GEMM layout micro-benchmark (GPU) for the Llama-3-8B training shapes (N = 4096 tokens).

For every projection it times the three training GEMMs in the layouts the block compute uses
(forward y = x W^T, input-grad dX = dY W, weight-grad dW = dY^T X) plus the alternative
input-grad layout with a pre-transposed weight copy (dX = dY (W^T)^T, both operands
K-contiguous), so the choice of layout is measured rather than guessed.
Usage: python tools/bench_gemm.py [--iters 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402


def timeit(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--backend", choices=["default", "hipblaslt", "rocblas"], default="default")
    a = ap.parse_args()
    ops.load_ext(required=True)
    if a.backend != "default":
        torch.backends.cuda.preferred_blas_library("cublaslt" if a.backend == "hipblaslt" else "cublas")
    N = a.tokens
    shapes = {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 28672), "down": (14336, 4096),
              "head": (4096, 128256)}
    dt = torch.bfloat16
    out = []
    for name, (k_in, n_out) in shapes.items():
        x = torch.randn(N, k_in, device="cuda", dtype=dt)
        w = torch.randn(n_out, k_in, device="cuda", dtype=dt) * 0.02
        wt = w.t().contiguous()
        dy = torch.randn(N, n_out, device="cuda", dtype=dt)
        y = torch.empty(N, n_out, device="cuda", dtype=dt)
        dx = torch.empty(N, k_in, device="cuda", dtype=dt)
        dw = torch.empty(n_out, k_in, device="cuda", dtype=dt)
        fl = 2.0 * N * k_in * n_out
        r = {"gemm": name, "M_N_K": [N, n_out, k_in]}
        r["fwd_xWt"] = timeit(lambda: torch.mm(x, w.t(), out=y), a.iters)
        r["dx_dyW"] = timeit(lambda: torch.mm(dy, w, out=dx), a.iters)
        r["dx_dyWt_T"] = timeit(lambda: torch.mm(dy, wt.t(), out=dx), a.iters)
        r["dw_dyTx"] = timeit(lambda: torch.mm(dy.t(), x, out=dw), a.iters)
        r["dw_xTdy_outT"] = timeit(lambda: torch.mm(x.t(), dy, out=dw.t()), a.iters)
        dwt = torch.empty(k_in, n_out, device="cuda", dtype=dt)
        r["dwT_xTdy"] = timeit(lambda: torch.mm(x.t(), dy, out=dwt), a.iters)
        r["transpose_w"] = timeit(lambda: wt.copy_(w.t()), a.iters)
        r["transpose_w_hip"] = timeit(lambda: ops.transpose2d(w), a.iters)
        assert torch.equal(ops.transpose2d(w), wt)
        r["transpose_w_hip_TBps"] = round(4 * w.numel() / r["transpose_w_hip"] / 1e9, 2)
        for k in ("fwd_xWt", "dx_dyW", "dx_dyWt_T", "dw_dyTx", "dw_xTdy_outT", "dwT_xTdy"):
            r[k + "_tflops"] = round(fl / r[k] / 1e9, 1)
        for k in list(r):
            if isinstance(r[k], float) and not k.endswith(("tflops", "TBps")):
                r[k] = round(r[k] * 1e3, 1)  # us
        print(json.dumps(r), flush=True)
        out.append(r)
        del x, w, wt, dy, y, dx, dw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
