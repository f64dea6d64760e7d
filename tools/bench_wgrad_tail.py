"""dW of the Llama-3-8B QKV / down projections at 40,960 tokens: every tile split 2 ways (round 4)
vs whole-K waves + a 2-way split tail (ops.wgrad_plan), interleaved in one process; us and PF."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402


def _time(fn, iters=10):
    for _ in range(2):
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
    K = 40960
    for name, M, N in (("qkv", 6144, 4096), ("down", 4096, 14336)):
        a = torch.randn(K, M, device="cuda").to(torch.bfloat16)
        b = torch.randn(K, N, device="cuda").to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        plan = ops.wgrad_plan(M, N, K)
        res = {"shape": name, "plan": list(plan)}
        arms = {"split2": lambda: ops.wgrad_gemm_(a, b, c, False, 2),
                "tail": lambda: torch.ops.bllm.wgrad_gemm_tail_(a, b, c, False, plan[1], plan[2]),
                "split1": lambda: ops.wgrad_gemm_(a, b, c, False, 1)}
        t = {k: [] for k in arms}
        for _ in range(3):
            for k, fn in arms.items():
                t[k].append(_time(fn))
        for k, v in t.items():
            us = sorted(v)[1]
            res[k] = {"us": round(us, 1), "PF": round(2 * M * N * K / us / 1e9, 3)}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
