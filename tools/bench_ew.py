"""Micro-benchmark of the HBM-bound Llama-3-8B elementwise/norm kernels at the bench shape
(24 x 1024 tokens): SwiGLU fwd/bwd on [N, 2*14336] and RMSNorm bwd (with the residual-gradient
add) on [N, 4096], bf16; plus the GPT2-774M bias-gradient column sums ([N, 1280], [N, 5120]).  Prints one JSON line with us/call and achieved GB/s per op.
Compare kernel changes by running this once per build.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402


def _time(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ops.load_ext(required=True)
    N, F, d = 24 * 1024, 14336, 4096
    dev, dt = "cuda:0", torch.bfloat16
    gu = torch.randn(N, 2 * F, device=dev).to(dt)
    da = torch.randn(N, F, device=dev).to(dt)
    x = torch.randn(N, d, device=dev).to(dt)
    dy = torch.randn(N, d, device=dev).to(dt)
    acc = torch.randn(N, d, device=dev).to(dt)
    w = torch.randn(d, device=dev).to(dt)
    dw = torch.zeros(d, device=dev, dtype=dt)
    _, rstd = ops.rmsnorm_fwd(x, w, 1e-5)
    g1 = torch.randn(N, 1280, device=dev).to(dt)     # GPT2-774M out/fc2 bias grads
    g5 = torch.randn(N, 5120, device=dev).to(dt)     # GPT2-774M fc1 bias grad
    db1 = torch.zeros(1280, device=dev, dtype=dt)
    db5 = torch.zeros(5120, device=dev, dtype=dt)
    res = {}
    # GPT2-774M at the preset's micro-batch 64 x 1024: the fused backward + bias column sums
    N64 = 64 * 1024
    f64 = torch.randn(N64, 5120, device=dev).to(dt)
    dg64 = torch.randn(N64, 5120, device=dev).to(dt)
    dm64 = torch.randn(N64, 1280, device=dev).to(dt)
    for name, fn, nbytes in (
        ("gpt2_b64_gelu_bwd_bias_5120", lambda: ops.gelu_bwd_bias(f64, dg64, db5, True), 3 * N64 * 5120 * 2),
        ("gpt2_b64_dropout_bwd_bias_1280", lambda: ops.dropout_bwd_bias(dm64, 0.1, 7, 0, db1, True), 2 * N64 * 1280 * 2),
        ("gpt2_b64_gelu_bwd_5120", lambda: ops.gelu_bwd(f64, dg64), 3 * N64 * 5120 * 2),
    ):
        us = _time(fn)
        res[name] = {"us": round(us, 1), "GBps": round(nbytes / us / 1e3, 1)}
    x64 = torch.randn(N64, 1280, device=dev).to(dt)
    w1 = torch.randn(1280, device=dev).to(dt)
    b1 = torch.randn(1280, device=dev).to(dt)
    _, m64, r64 = ops.layernorm_fwd(x64, w1, b1, 1e-5)
    dw1 = torch.zeros(1280, device=dev, dtype=dt)
    for name, fn, nbytes in (
        ("gpt2_b64_layernorm_bwd_1280", lambda: ops.layernorm_bwd(dm64, x64, w1, m64, r64, dm64, dw1, db1, True),
         4 * N64 * 1280 * 2),
        ("gpt2_b64_layernorm_fwd_1280", lambda: ops.layernorm_fwd(x64, w1, b1, 1e-5), 2 * N64 * 1280 * 2),
    ):
        us = _time(fn)
        res[name] = {"us": round(us, 1), "GBps": round(nbytes / us / 1e3, 1)}
    del f64, dg64, dm64, x64
    for name, fn, nbytes in (
        ("swiglu_fwd", lambda: ops.swiglu_fwd(gu), 3 * N * F * 2),
        ("swiglu_bwd", lambda: ops.swiglu_bwd(gu, da), 5 * N * F * 2),
        ("swiglu_bwd_act", lambda: ops.swiglu_bwd_act(gu, da), 6 * N * F * 2),
        ("rmsnorm_fwd", lambda: ops.rmsnorm_fwd(x, w, 1e-5), 2 * N * d * 2),
        ("rmsnorm_bwd", lambda: ops.rmsnorm_bwd(dy, x, w, rstd, acc, dw, True), 4 * N * d * 2),
        ("bias_grad_1280", lambda: ops.bias_grad_(g1, db1, True), N * 1280 * 2),
        ("bias_grad_5120", lambda: ops.bias_grad_(g5, db5, True), N * 5120 * 2),
    ):
        us = _time(fn)
        res[name] = {"us": round(us, 1), "GBps": round(nbytes / us / 1e3, 1)}
    del gu, da
    # fused AdamW on a 1 G-parameter slot (bf16 param + grad, fp32 master / m / v): 28 B per parameter
    n = 1 << 30
    p_ = torch.zeros(n, device=dev, dtype=dt)
    g_ = torch.full((n,), 1e-3, device=dev, dtype=dt)
    mst = torch.zeros(n, device=dev, dtype=torch.float32)
    m1, m2 = torch.zeros_like(mst), torch.zeros_like(mst)
    us = _time(lambda: ops.adamw_step_(p_, mst, g_, m1, m2, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1), iters=5)
    res["adamw_1g_params"] = {"us": round(us, 1), "GBps": round(28 * n / us / 1e3, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
