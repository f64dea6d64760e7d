#!/usr/bin/env python3
"""Attention kernel micro-benchmark (GPU): fwd / bwd time and effective TFLOP/s at the
Llama-3-8B (hd 128, GQA 32/8) and GPT-2 (hd 64) training shapes, causal.
Usage: python tools/bench_attn.py [--iters 20] [--shapes llama3-8B-B40,gpt2-774M-B64]"""
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
    ap.add_argument("--shapes", default="", help="comma-separated shape names (default: all)")
    ap.add_argument("--noncausal", action="store_true", help="full (non-causal) attention")
    ap.add_argument("--T", type=int, default=None, help="override the sequence length")
    ap.add_argument("--env_ab", default="",
                    help="NAME: time the forward with env NAME=0 and NAME=1 in this process (A/B of a "
                         "kernel variant read per launch) and report the outputs' max difference")
    ap.add_argument("--variants", default="",
                    help="forward A/B arms 'name:VAR=v+VAR2=v;name2:...' (kernel knobs read per launch), "
                         "timed interleaved with the default; outputs compared with the default's")
    ap.add_argument("--bwd_env_ab", default="",
                    help="NAME=v1,v2,...: time the backward under each value of env NAME (a kernel knob read per "
                         "launch), interleaved, and report dqkv's max difference from the first value's")
    ap.add_argument("--no_mask", action="store_true",
                    help="dropout shapes: re-hash the keep bits in backward instead of reading the forward's mask")
    a = ap.parse_args()
    ops.load_ext(required=True)
    shapes = [("llama3-8B", 4, 1024, 32, 8, 128, 0.0), ("llama3-8B-B24", 24, 1024, 32, 8, 128, 0.0),
              ("llama3-8B-B40", 40, 1024, 32, 8, 128, 0.0),
              ("llama3.2-1B-B24", 24, 1024, 32, 8, 64, 0.0), ("gpt2-774M", 4, 1024, 20, 20, 64, 0.1),
              ("gpt2-774M-nodrop", 4, 1024, 20, 20, 64, 0.0),
              ("gpt2-774M-B24", 24, 1024, 20, 20, 64, 0.1),
              ("gpt2-774M-B24-nodrop", 24, 1024, 20, 20, 64, 0.0),
              ("gpt2-774M-B64", 64, 1024, 20, 20, 64, 0.1), ("gpt2-774M-B64-nodrop", 64, 1024, 20, 20, 64, 0.0),
              ("gpt2-124M", 4, 1024, 12, 12, 64, 0.0)]
    if a.shapes:
        keep = a.shapes.split(",")
        shapes = [sh for sh in shapes if sh[0] in keep]
    causal = not a.noncausal
    res = []
    for name, B, T, H, G, hd, p in shapes:
        if a.T:
            B, T = max(1, B * T // a.T), a.T
        qkv = torch.randn(B * T, (H + 2 * G) * hd, device="cuda", dtype=torch.bfloat16)
        do = torch.randn(B * T, H * hd, device="cuda", dtype=torch.bfloat16)
        km = None if a.no_mask else ops.attn_keep_mask(qkv, B, T, H, hd, p)
        o, lse = ops.flash_attn_fwd(qkv, B, T, H, G, hd, causal, p, 1, 0, keep_mask=km)
        tf = timeit(lambda: ops.flash_attn_fwd(qkv, B, T, H, G, hd, causal, p, 1, 0, keep_mask=km), a.iters)
        tb = timeit(lambda: ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, causal, p, 1, 0, keep_mask=km), a.iters)
        flop = 2 * 2 * B * H * T * T * hd / (2 if causal else 1)  # two matmuls (causal: half the square)
        if a.variants:
            arms = [("default", {})] + [(vd.split(":", 1)[0], dict(e.split("=", 1) for e in vd.split(":", 1)[1].split("+") if e))
                                        for vd in a.variants.split(";") if vd]
            tt, outs = {}, {}
            for rnd in range(3):
                for an, env in arms:
                    os.environ.update(env)
                    tt.setdefault(an, []).append(
                        timeit(lambda: ops.flash_attn_fwd(qkv, B, T, H, G, hd, causal, p, 1, 0, keep_mask=km), a.iters))
                    outs[an] = ops.flash_attn_fwd(qkv, B, T, H, G, hd, causal, p, 1, 0, keep_mask=km)
                    for k_ in env:
                        os.environ.pop(k_)
            o_ref = outs["default"][0].float()
            print(json.dumps(dict(shape=name, fwd_tflops={an: round(flop / sorted(v)[1] / 1e9, 1) for an, v in tt.items()},
                                  max_abs_o={an: float((o[0].float() - o_ref).abs().max()) for an, o in outs.items()})),
                  flush=True)
        if a.env_ab:
            ab = {}
            outs = {}
            for rnd in range(3):
                for v in ("0", "1"):
                    os.environ[a.env_ab] = v
                    t = timeit(lambda: ops.flash_attn_fwd(qkv, B, T, H, G, hd, causal, p, 1, 0, keep_mask=km), a.iters)
                    ab.setdefault(v, []).append(t)
                    outs[v] = ops.flash_attn_fwd(qkv, B, T, H, G, hd, causal, p, 1, 0, keep_mask=km)
            os.environ.pop(a.env_ab)
            med = {v: sorted(ts)[1] for v, ts in ab.items()}
            (o0, l0), (o1, l1) = outs["0"], outs["1"]
            print(json.dumps(dict(shape=name, ab=a.env_ab, fwd_ms_0=round(med["0"], 4), fwd_ms_1=round(med["1"], 4),
                                  tflops_0=round(flop / med["0"] / 1e9, 1), tflops_1=round(flop / med["1"] / 1e9, 1),
                                  max_abs_o=float((o0.float() - o1.float()).abs().max()),
                                  max_abs_lse=float((l0 - l1).abs().max()))), flush=True)
        if a.bwd_env_ab:
            nm, vals = a.bwd_env_ab.split("=", 1)
            vals = vals.split(",")
            tt, outs = {}, {}
            for rnd in range(3):
                for v in vals:
                    os.environ[nm] = v
                    tt.setdefault(v, []).append(timeit(
                        lambda: ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, causal, p, 1, 0, keep_mask=km), a.iters))
                    outs[v] = ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, causal, p, 1, 0, keep_mask=km)
            os.environ.pop(nm)
            ref0 = outs[vals[0]].float()
            print(json.dumps(dict(shape=name, ab=nm, bwd_ms={v: round(sorted(ts)[1], 4) for v, ts in tt.items()},
                                  max_abs_dqkv={v: float((x.float() - ref0).abs().max()) for v, x in outs.items()})),
                  flush=True)
        res.append(dict(shape=name, B=B, T=T, causal=causal, keep_mask=km is not None, fwd_ms=round(tf, 4), bwd_ms=round(tb, 4),
                        fwd_tflops=round(flop / tf / 1e9, 1), bwd_tflops_5mm=round(2.5 * flop / tb / 1e9, 1)))
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
