"""World-2 rehearsal of the engines on ONE MI355X with real kernels: two processes share cuda:0,
joined by a gloo process group over GPU tensors (RCCL refuses two ranks on one device).  Each
rank trains bf16 Llama (full activation checkpointing, 3 AdamW steps) on its half of every batch;
the result is compared with one process training on the whole batch through the local engine.
What this exercises beyond the world-1 forced-comm rehearsal: real shards (each rank keeps 1/2
of every flat), a gather that brings back the OTHER rank's half, reduce-scatters that average two
different gradients, and the cross-rank clip norm.  Run by tests/test_engines_gpu.py; prints one
JSON line from rank 0."""
import json
import os
import socket
import sys
from datetime import timedelta

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from building_llm_from_scratch_amd import ops  # noqa: E402
from building_llm_from_scratch_amd.config import get_config  # noqa: E402
from building_llm_from_scratch_amd.models import build_model  # noqa: E402
from building_llm_from_scratch_amd.parallel import setup_engine  # noqa: E402
from building_llm_from_scratch_amd.train.optim import FusedAdamW  # noqa: E402

CFG = dict(context_length=256, emb_dim=512, n_heads=4, n_kv_groups=2, hidden_dim=1024, n_layers=3,
           vocab_size=1024, dtype=torch.bfloat16)


def train(kind, dev, batches, rank, world):
    torch.manual_seed(0)
    cfg = get_config("llama3_2", "1B").replace(**CFG)
    m = build_model(cfg, use_actv_ckpt="full", device=dev)
    eng = setup_engine(m, kind, device=dev, prefetch=1)
    opt = FusedAdamW(m, lr=1e-3, weight_decay=0.1, engine=eng)
    losses = []
    for b in batches:
        n = b.shape[0] // world
        mine = b[rank * n:(rank + 1) * n]
        opt.zero_grad()
        loss = m(mine[:, :-1], mine[:, 1:])
        loss.backward()
        opt.clip_grad_norm_(1.0)
        opt.step()
        lt = loss.detach().float().reshape(1)
        if world > 1:
            dist.all_reduce(lt)
            lt /= world
        losses.append(lt.item())
    sd = eng.full_state_dict() if hasattr(eng, "full_state_dict") else m.state_dict()
    if sd is not None:
        sd = {k: v.detach().float().cpu() for k, v in sd.items() if not k.endswith(("mask", "cos", "sin"))}
    return losses, sd


def worker(rank, kinds, port, q):
    try:
        ops.load_ext(required=True)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2,
                                timeout=timedelta(minutes=3))
        g = torch.Generator(device=dev).manual_seed(5)
        batches = [torch.randint(0, 1024, (4, 257), device=dev, generator=g) for _ in range(3)]
        out = {}
        if rank == 0:
            ref_losses, ref_sd = train("local", dev, batches, 0, 1)
            out["ref_losses"] = ref_losses
        dist.barrier()
        for kind in kinds:
            losses, sd = train(kind, dev, batches, rank, 2)
            if rank == 0:
                diff = max((sd[k] - ref_sd[k]).abs().max().item() for k in ref_sd)
                rel = max(((sd[k] - ref_sd[k]).norm() / (ref_sd[k].norm() + 1e-12)).item() for k in ref_sd)
                out[kind] = {"losses": losses, "max_param_diff": diff, "max_rel_diff": rel,
                             "keys_match": set(sd) == set(ref_sd)}
            dist.barrier()
        dist.destroy_process_group()
        if rank == 0:
            q.put(json.dumps(out))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put("ERROR " + traceback.format_exc())
        raise


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    kinds = args[0].split(",") if args else ["fsdp", "zero1", "ddp"]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, kinds, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(120)
    print(res, flush=True)
    codes = [p.exitcode for p in procs]
    print(json.dumps({"exitcodes": codes}), flush=True)
    # a Python-level error (e.g. a collective gloo does not implement for GPU tensors) is reported
    # in the JSON and exits 0 when ``--report`` is given; a crash (negative exit code) never does
    crashed = any(c is None or c < 0 for c in codes)
    ok = not res.startswith("ERROR") and codes == [0, 0]
    sys.exit(0 if ok or ("--report" in sys.argv and not crashed) else 1)


if __name__ == "__main__":
    main()
