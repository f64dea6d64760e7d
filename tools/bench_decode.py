#!/usr/bin/env python3
"""Sampling / decode benchmark (GPU): the Trainer's sample print (reference train.py:213-229:
200 new tokens, top-k 5, temperature 1) on random-init weights, KV-cache decode
(train/generate.py:generate_cached).  Prints ms per generated token and tokens/s.
Usage: python tools/bench_decode.py [--model llama3 --num_params 8B] [--tokens 200] [--graph 0|1]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402
from building_llm_from_scratch_amd.config import get_config  # noqa: E402
from building_llm_from_scratch_amd.models import build_model  # noqa: E402
from building_llm_from_scratch_amd.train import generate as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3")
    ap.add_argument("--num_params", default="8B")
    ap.add_argument("--tokens", type=int, default=200)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--prompt", type=int, default=6)
    ap.add_argument("--graph", type=int, default=None, help="force the hipGraph decode step on/off")
    a = ap.parse_args()
    ops.load_ext(required=True)
    cfg = get_config(a.model, a.num_params).replace(dtype=torch.bfloat16)
    torch.manual_seed(0)
    m = build_model(cfg, device="cuda")
    m.flatten()
    if a.graph is not None:
        os.environ["BLLM_DECODE_GRAPH"] = str(a.graph)
    idx = torch.randint(0, cfg.vocab_size, (a.batch, a.prompt), device="cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    G.generate_cached(m, idx, 8, cfg.context_length, temperature=1.0, top_k=5, generator=g)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = G.generate_cached(m, idx, a.tokens, cfg.context_length, temperature=1.0, top_k=5, generator=g)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = out.shape[1] - a.prompt
    print(json.dumps({"model": f"{a.model}-{a.num_params}", "batch": a.batch, "new_tokens": n,
                      "ms_per_token": round(1000 * dt / max(n, 1), 3), "tokens_per_s": round(a.batch * n / dt, 1),
                      "graph": os.environ.get("BLLM_DECODE_GRAPH", "default")}))


if __name__ == "__main__":
    main()
