"""FSDP auto prefetch depth and unit residency (CPU, gloo, world 2).

* The auto depth (``--fsdp_prefetch 0``) decides how many all-gathers a rank issues ahead of each
  reduce-scatter in backward, so every rank must pick the same depth even when the ranks see
  different sequence lengths (instruction batches are padded per batch).  The depth function is
  patched to depend on the token count so that a per-rank sizing WOULD disagree.
* After a training forward only the head unit stays gathered (it is the first unit of backward);
  after an eval forward nothing does."""
import os
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from building_llm_from_scratch_amd.config import get_config
from building_llm_from_scratch_amd.models import build_model
from building_llm_from_scratch_amd.parallel import setup_engine
from building_llm_from_scratch_amd.train.optim import FusedAdamW


def _cfg():
    return get_config("llama3_2", "1B").replace(context_length=32, emb_dim=64, n_heads=4, n_kv_groups=2,
                                                hidden_dim=96, n_layers=3, vocab_size=97, dtype=torch.float32)


def _worker(rank, world, out, store):
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    try:
        from building_llm_from_scratch_amd.parallel import commplan
        # rank 0 sees 2 x 16 = 32 tokens, rank 1 2 x 8 = 16: a per-rank sizing gives 1 vs 2
        commplan.fsdp_prefetch_depth = lambda nbytes, numel, tokens, world_, **kw: 1 if tokens >= 32 else 2
        torch.manual_seed(0)
        m = build_model(_cfg())
        eng = setup_engine(m, "fsdp", device="cpu", prefetch=0)
        opt = FusedAdamW(m, lr=1e-3, weight_decay=0.1, engine=eng)
        T = 16 if rank == 0 else 8
        g = torch.Generator().manual_seed(rank)
        for _ in range(3):
            b = torch.randint(0, 97, (2, T + 1), generator=g)
            opt.zero_grad()
            loss = m(b[:, :-1], b[:, 1:])
            loss.backward()
            opt.clip_grad_norm_(1.0)
            opt.step()
        # residency: a training forward keeps only the head gathered, an eval forward nothing
        b = torch.randint(0, 97, (2, T + 1), generator=g)
        loss = m(b[:, :-1], b[:, 1:])
        after_train = [u.state["gathered"] for u in eng.units]
        loss.backward()
        m.eval()
        with torch.no_grad():
            m(b[:, :-1], b[:, 1:])
        after_eval = [u.state["gathered"] for u in eng.units]
        depths = [None] * world
        dist.all_gather_object(depths, eng.prefetch)
        if rank == 0:
            torch.save({"depths": depths, "after_train": after_train, "after_eval": after_eval}, out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_auto_prefetch_depth_is_rank_invariant_and_residency():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_worker, args=(world, out, os.path.join(d, "store")), nprocs=world, join=True,
                           start_method="spawn")
        r = torch.load(out, weights_only=True)
    assert r["depths"] == [1, 1], r["depths"]      # sized from the MAX token count (32) on both ranks
    assert r["after_train"][-1] and not any(r["after_train"][:-1]), r["after_train"]
    assert not any(r["after_eval"]), r["after_eval"]
