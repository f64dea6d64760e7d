#!/usr/bin/env python3
"""LoRA kernel micro-benchmark (GPU): csrc/lora.hip ops at the Llama-3.2-1B LoRA shapes
(N = 38,400 tokens, rank 16) with their HBM-roofline time, so each kernel's efficiency is read
off directly.  Usage: python tools/bench_lora.py [--tokens 4096] [--rank 16] [--iters 50]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402

HBM = 5.0e12  # B/s achievable


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
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=38400, help="default: the LoRA preset's ~38k tokens per step")
    ap.add_argument("--rank", type=int, default=16)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default=None, help="comma-separated case-name prefixes")
    ap.add_argument("--env_ab", default=None,
                    help="'|'-separated arms of KEY=VALUE[+KEY=VALUE] environment settings read per launch "
                         "(e.g. 'BLLM_LORA_DOWN=16|'), each case timed under every arm")
    a = ap.parse_args()
    ops.load_ext(required=True)
    N, r, dt = a.tokens, a.rank, torch.bfloat16
    groups = {"qkv": (2048, [2048, 512, 512]), "o": (2048, [2048]), "gate_up": (2048, [8192, 8192]),
              "down": (8192, [2048]), "head": (2048, [128256])}
    for name, (K, outs) in groups.items():
        M = sum(outs)
        c0 = [sum(outs[:i]) for i in range(len(outs))]
        offs = [i * r for i in range(len(outs))]
        R = r * len(outs)
        x = torch.randn(N, K, device="cuda", dtype=dt)
        dy = torch.randn(N, M, device="cuda", dtype=dt)
        As = [torch.randn(K, r, device="cuda", dtype=dt) * 0.05 for _ in outs]
        Bs = [torch.randn(r, o, device="cuda", dtype=dt) * 0.05 for o in outs]
        P = ops.lora_pack_t(As)
        t = ops.lora_down(x, [P], [0], [K], [0], R)
        u = ops.lora_down(dy, Bs, c0, outs, offs, R)
        y = torch.empty(N, M, device="cuda", dtype=dt)
        dx = torch.empty(N, K, device="cuda", dtype=dt)
        gB = [torch.empty(r, o, device="cuda", dtype=dt) for o in outs]
        gA = [torch.empty(K, r, device="cuda", dtype=dt) for _ in outs]
        Rp = -(-(K + R) // 64) * 64 - K                        # rows padded to 128-B lines (FusedLinear._kaug_pad)
        xa = torch.randn(N, K + Rp, device="cuda", dtype=dt)    # K-augmented [x | s t | 0] / [dx_W | u | 0]
        res = {"group": name, "N_K_M": [N, K, M]}
        cases = {
            "down_fwd": (lambda: ops.lora_down(x, [P], [0], [K], [0], R), N * K * 2),
            "down_bwd": (lambda: ops.lora_down(dy, Bs, c0, outs, offs, R), N * M * 2),
            "up_fwd": (lambda: ops.lora_up_(y, t, Bs, c0, offs, 2.0), N * M * 2),
            "up_bwd": (lambda: ops.lora_up_(dx, u, [P], [0], [0], 2.0), N * K * 2),
            "down_fwd_kaug": (lambda: ops.lora_down_into(xa[:, :K], [P], [0], [K], [0], R, 2.0, xa[:, K:]), N * K * 2),
            "up_bwd_kaug": (lambda: ops.lora_up_(dx, xa[:, K:K + R], [P], [0], [0], 2.0, base=xa[:, :K]), 2 * N * K * 2),
            "wgrad_A_kaug": (lambda: ops.lora_wgrad(xa[:, K:K + R], xa[:, :K], [g.t() for g in gA], offs, [0] * len(outs),
                                                    2.0), N * K * 2),
            "wgrad_B": (lambda: ops.lora_wgrad(t, dy, gB, offs, c0, 2.0), N * M * 2),
            "wgrad_A": (lambda: ops.lora_wgrad(u, x, [g.t() for g in gA], offs, [0] * len(outs), 2.0), N * K * 2),
        }
        for k, (fn, nbytes) in cases.items():
            if a.only and not any(k.startswith(o) for o in a.only.split(",")):
                continue
            for env in (a.env_ab.split("|") if a.env_ab else [""]):
                for kv in env.split("+") if env else []:   # KEY=VALUE[+KEY=VALUE] set for this arm
                    key, val = kv.split("=", 1)
                    os.environ[key] = val
                us = timeit(fn, a.iters)
                for kv in env.split("+") if env else []:
                    os.environ.pop(kv.split("=", 1)[0], None)
                res[k + (f"[{env}]" if env else "")] = {"us": round(us, 1), "roofline_us": round(nbytes / HBM * 1e6, 1),
                                                        "TB/s": round(nbytes / us / 1e6, 2)}
        print(json.dumps(res), flush=True)
        del x, dy, y, dx, t, u, xa
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
