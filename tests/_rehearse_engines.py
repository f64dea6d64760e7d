"""GPU rehearsal of the N>1 engine path on ONE MI355X (run as a subprocess by
tests/test_engines_gpu.py): RCCL process group of world 1 with ``BLLM_FORCE_COMM=1``, so DDP /
ZeRO-1 / FSDP issue their real all-gathers, reduce-scatters and all-reduces on RCCL's
high-priority stream (shards freed / re-allocated, waits on the compute stream) — the code that
runs at 2-8 GPUs, minus the cross-GPU traffic RCCL cannot rehearse with two ranks on one device.
Compares bf16 Llama training (full activation checkpointing, 3 AdamW steps) against the local
engine.  Prints one JSON line."""
import json
import os
import socket
import sys
from datetime import timedelta

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402
from building_llm_from_scratch_amd.config import get_config  # noqa: E402
from building_llm_from_scratch_amd.models import build_model  # noqa: E402
from building_llm_from_scratch_amd.parallel import nccl_pg_options, setup_engine  # noqa: E402
from building_llm_from_scratch_amd.train.optim import FusedAdamW  # noqa: E402


def run(kind, dev, batches):
    torch.manual_seed(0)
    cfg = get_config("llama3_2", "1B").replace(context_length=256, emb_dim=512, n_heads=4, n_kv_groups=2,
                                               hidden_dim=1024, n_layers=3, vocab_size=1024, dtype=torch.bfloat16)
    m = build_model(cfg, use_actv_ckpt="full", device=dev)
    eng = setup_engine(m, kind, device=dev, prefetch=1)
    opt = FusedAdamW(m, lr=1e-3, weight_decay=0.1, engine=eng)
    losses = []
    for b in batches:
        opt.zero_grad()
        loss = m(b[:, :-1], b[:, 1:])
        loss.backward()
        opt.clip_grad_norm_(1.0)
        opt.step()
        losses.append(loss.float().item())
    sd = eng.full_state_dict() if hasattr(eng, "full_state_dict") else m.state_dict()
    sd = {k: v.detach().float().cpu() for k, v in sd.items() if not k.endswith(("mask", "cos", "sin"))}
    info = {"no_shard": getattr(eng, "no_shard", None), "no_comm": getattr(eng, "no_comm", None)}
    del m, eng, opt
    torch.cuda.empty_cache()
    return losses, sd, info


def main():
    kinds = sys.argv[1].split(",")
    ops.load_ext(required=True)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            timeout=timedelta(minutes=2), device_id=dev, pg_options=nccl_pg_options())
    g = torch.Generator(device=dev).manual_seed(5)
    batches = [torch.randint(0, 1024, (4, 257), device=dev, generator=g) for _ in range(3)]
    try:
        ref_losses, ref_sd, _ = run("local", dev, batches)
        out = {"ref_losses": ref_losses}
        for kind in kinds:
            os.environ["BLLM_FORCE_COMM"] = "1"
            losses, sd, info = run(kind, dev, batches)
            os.environ["BLLM_FORCE_COMM"] = "0"
            diff = max((sd[k] - ref_sd[k]).abs().max().item() for k in ref_sd)
            out[kind] = {"losses": losses, "max_param_diff": diff, "keys_match": set(sd) == set(ref_sd), **info}
        print(json.dumps(out), flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
