#!/usr/bin/env python3
"""Headline benchmark: whole-node training tokens/s, Llama-3-8B bf16 FSDP (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Each rank runs a micro-batch of 24 sequences x ``T = 1024`` (the reference clamps every Llama
to ctx 1024, Models/Llama/config.py:115-124) of synthetic token ids through one full training
step — forward, fused CE, backward, global-norm clip 1.0,
AdamW(wd 0.1) with fp32 master weights — on random-init weights of the full Llama-3-8B
architecture.  Nothing is skipped inside the timed region.  W untimed warm-up steps, then
exactly K timed steps bracketed by barrier + device sync; the slowest rank's time is used.
Weak scaling: per-GPU work is fixed, total tokens grow with N.

Micro-batch: the reference's ``--batch_size`` default of 4 (args.py:53) was sized for a 16 GB
T4.  One MI355X holds 288 GB, so the benchmark sizes the per-GPU micro-batch for that
(measured on one GPU, profiles/r1_llama3_8b_1gpu_v4.md): B=4 20.0k tok/s, B=16 25.0k (184 GiB
peak), B=24 25.5k (217 GiB), B=32 25.7k (249 GiB).  B=24 keeps ~70 GB of headroom on the
single-GPU (unsharded) run; it also keeps FSDP's per-block all-gathers (416 MiB) and
reduce-scatters hidden under block compute at 2 GPUs, where two ranks share a single xGMI
link.  ``--batch_size 4`` reproduces the reference default.

Activation checkpointing: off by default, like the reference (``--use_actv_ckpt`` is opt-in,
args.py:76).  Same-box A/B at B=24 (profiles/r1_bench_v7_ckpt_*.log): none 26.94k tok/s at
229 GiB peak vs selective (norm outputs recomputed) 26.74k at 217 GiB.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TOKENS_PER_S = None  # the reference publishes no number


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3")
    ap.add_argument("--num_params", default="8B")
    ap.add_argument("--batch_size", type=int, default=24, help="micro-batch per GPU (reference CLI default: 4)")
    ap.add_argument("--seq_len", type=int, default=1024)
    ap.add_argument("--actv_ckpt", default="none", choices=["none", "selective", "full"],
                    help="none = the reference default (use_actv_ckpt off); selective recomputes the norms")
    ap.add_argument("--parallel", default="fsdp", choices=["fsdp", "ddp", "zero1"])
    ap.add_argument("--reshard_after_forward", type=int, default=1)
    ap.add_argument("--layers", type=int, default=None, help="(debug only) override n_layers; invalidates the metric")
    ap.add_argument("--profile", action="store_true", help="print a per-phase timing breakdown")
    ap.add_argument("--lora_rank", type=int, default=0, help="LoRA finetune benchmark (freeze base, rank r)")
    ap.add_argument("--lora_alpha", type=int, default=32)
    ap.add_argument("--overlap_optimizer", action="store_true",
                    help="run AdamW on a side HIP stream under the next forward")
    return ap.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    from building_llm_from_scratch_amd import ops
    from building_llm_from_scratch_amd.config import get_config
    from building_llm_from_scratch_amd.models import build_model
    from building_llm_from_scratch_amd.parallel import setup_engine
    from building_llm_from_scratch_amd.train.optim import FusedAdamW

    launched = "WORLD_SIZE" in os.environ and "RANK" in os.environ  # torchrun
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == a.gpus, f"--gpus {a.gpus} but WORLD_SIZE={world} (launch with torchrun for N>1)"
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = launched or world > 1
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
    ops.load_ext(required=True)

    cfg = get_config(a.model, a.num_params, context_length=a.seq_len).replace(dtype=torch.bfloat16)
    if a.layers:
        cfg = cfg.replace(n_layers=a.layers)
    torch.manual_seed(123)
    model = build_model(cfg, use_actv_ckpt=a.actv_ckpt, device=dev)
    if a.lora_rank:
        from building_llm_from_scratch_amd.models import replace_linear_with_lora
        for p in model.parameters():
            p.requires_grad = False
        replace_linear_with_lora(model, rank=a.lora_rank, alpha=a.lora_alpha)
    engine = setup_engine(model, a.parallel if distributed else "local", device=dev,
                          reshard_after_forward=bool(a.reshard_after_forward))
    opt = FusedAdamW(model, lr=3e-4, weight_decay=0.1, engine=engine, overlap=a.overlap_optimizer)
    B, T = a.batch_size, a.seq_len
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    data = [torch.randint(0, cfg.vocab_size, (B, T + 1), device=dev, generator=g) for _ in range(4)]

    def step(i):
        batch = data[i % len(data)]
        opt.zero_grad()
        loss = model(batch[:, :-1], batch[:, 1:])
        loss.backward()
        opt.clip_grad_norm_(1.0)
        opt.step()
        return loss

    for i in range(a.warmup):
        loss = step(i)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(i)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if distributed:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = el.item()
    tokens = world * B * T * a.steps
    tps = tokens / elapsed
    ms = 1000 * elapsed / a.steps
    flops_tok = cfg.train_flops_per_token(T)
    if a.actv_ckpt == "full":
        flops_tok *= 4.0 / 3.0
    mfu = tps / world * flops_tok / 2.5e15
    if a.profile and rank == 0:
        prof = profile_phases(model, opt, data[0], dev)
        print(json.dumps({"profile_ms": prof}), file=sys.stderr)
    if rank == 0:
        out = {
            "metric": ("tokens/sec (whole node) Llama-3-8B bf16 FSDP" if (a.model, a.num_params) == ("llama3", "8B")
                       else f"tokens/sec (whole node) {cfg.name}-{cfg.size} bf16 {a.parallel}"
                       + (f" LoRA r={a.lora_rank}" if a.lora_rank else "")),
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (tps / BASELINE_TOKENS_PER_S) if BASELINE_TOKENS_PER_S else None,
            "dtype": "bf16",
            "data": "synthetic token ids (Gutenberg-pretraining shape), random-init weights",
            "config": {
                "model": f"{cfg.name}-{cfg.size}" + (f" ({cfg.n_layers} layers, INVALID)" if a.layers else ""),
                "global_batch": world * B,
                "micro_batch_per_gpu": B,
                "seq_len": T,
                "parallelism": f"{a.parallel}{world}",
                "engine": type(engine).__name__,
                "actv_ckpt": a.actv_ckpt,
                "optimizer": "AdamW fp32 master, wd 0.1, clip 1.0",
            },
            "mfu_dense_bf16": round(mfu, 4),
            "peak_mem_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1),
            "final_loss": round(float(loss.item()), 4),
        }
        print(json.dumps(out))
    if distributed:
        dist.destroy_process_group()


def profile_phases(model, opt, batch, dev, n=3):
    import torch
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    res = {"fwd": 0.0, "bwd": 0.0, "clip+opt": 0.0}
    for _ in range(n):
        e = [ev() for _ in range(4)]
        e[0].record()
        loss = model(batch[:, :-1], batch[:, 1:])
        e[1].record()
        loss.backward()
        e[2].record()
        opt.clip_grad_norm_(1.0)
        opt.step()
        e[3].record()
        torch.cuda.synchronize()
        res["fwd"] += e[0].elapsed_time(e[1]) / n
        res["bwd"] += e[1].elapsed_time(e[2]) / n
        res["clip+opt"] += e[2].elapsed_time(e[3]) / n
    return {k: round(v, 2) for k, v in res.items()}


if __name__ == "__main__":
    main()
