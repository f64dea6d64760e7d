#!/usr/bin/env python3
"""dX GEMM micro-benchmark (GPU): dx[N, in] = dy[N, out] @ W[out, in] on the MFMA kernel with a
K-contiguous A (csrc/gemm_wgrad.hip, ``ops.gemm_nn_``) vs hipBLASLt (``torch.mm``), on the
input-gradient shapes of the benchmark models.  Interleaved rounds in one process, median.
``--forward``: the forward layout instead, y[N, out] = x[N, in] @ W^T, hipBLASLt on W vs the
kernel on a [in, out] copy of W^T (the shapes an epilogue-fused forward GEMM would run).
``hipblaslt_wt_us``: hipBLASLt on the K-contiguous W^T copy (the default dX path).
Usage: python tools/bench_dgrad.py [--tokens 24576] [--iters 10] [--rounds 3] [--forward]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402
from tools.bench_wgrad import SHAPES, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--models", default="llama3_8b,gpt2_774m,llama32_1b")
    ap.add_argument("--forward", action="store_true")
    a = ap.parse_args()
    ops.load_ext(required=True)
    Nt = a.tokens
    for model in a.models.split(","):
        for name, out_f, in_f in SHAPES[model]:
            if a.forward:  # y = x W^T: "dy" is x [N, in], the B operand W^T [in, out]
                out_f, in_f = in_f, out_f
            dy = (torch.rand(Nt, out_f, device="cuda") * 2 - 1).to(torch.bfloat16)
            W = ((torch.rand(out_f, in_f, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
            Wt = W.t().contiguous()   # the other storage order of the same operand
            d0 = torch.empty(Nt, in_f, device="cuda", dtype=torch.bfloat16)
            d1 = torch.empty_like(d0)
            d2 = torch.empty_like(d0)
            fl = 2.0 * Nt * out_f * in_f
            r = {"model": model, "gemm": name, "layout": "fwd" if a.forward else "dx",
                 "k_n": [out_f, in_f], "tokens": Nt}
            times = {"hipblaslt_us": [], "hipblaslt_wt_us": [], "mfma_us": []}
            if a.forward:
                times["mfma_nt_us"] = []
                d3 = torch.empty_like(d0)
            # forward: the model's hipBLASLt call is x @ W^T on the [out, in] weight (= Wt.t());
            # the kernel needs B row-major [K, N] = W here
            lt_main, lt_alt = (Wt.t(), W) if a.forward else (W, Wt.t())
            for _ in range(a.rounds):
                times["hipblaslt_us"].append(timeit(lambda: torch.mm(dy, lt_main, out=d0), a.iters))
                times["hipblaslt_wt_us"].append(timeit(lambda: torch.mm(dy, lt_alt, out=d2), a.iters))
                times["mfma_us"].append(timeit(lambda: ops.gemm_nn_(dy, W, d1, False), a.iters))
                if a.forward:  # both operands K-contiguous: x [N, in] . Wlin[out, in]^T
                    times["mfma_nt_us"].append(timeit(lambda: ops.gemm_nt_(dy, Wt, d3, False), a.iters))
            for k, ts in times.items():
                r[k] = sorted(ts)[len(ts) // 2]
            torch.cuda.synchronize()
            r["max_rel_err_vs_hipblaslt"] = round(((d1.float() - d0.float()).abs().max() / d0.float().abs().max()).item(), 5)
            if a.forward:
                r["nt_max_rel_err"] = round(((d3.float() - d0.float()).abs().max() / d0.float().abs().max()).item(), 5)
            for k in list(r):
                if k.endswith("_us"):
                    r[k.replace("_us", "_tflops")] = round(fl / r[k] / 1e6, 1)
                    r[k] = round(r[k], 1)
            print(json.dumps(r), flush=True)
            del dy, W, Wt, d0, d1, d2
            if a.forward:
                del d3
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
