"""Sharded initialisation of a meta-built model (CPU, gloo).

A model built on the ``meta`` device has no values; ``flatten`` initialises each unit right after
allocating its flat, under a per-unit seed (models/base.py:init_unit_), and FSDP shards and frees
that unit before allocating the next.  Every rank therefore computes the same initial weights
without holding the whole model and without a broadcast.  Checked here:

* the FSDP engines at world 2 and 4 issue NO broadcast and, after 3 training steps, match a
  single-process run of the same meta-built model (same per-unit seeds);
* DDP / ZeRO-1 on a meta-built model do the same;
* the values follow the reference modules' own initialisation (nn.Linear kaiming-uniform bound,
  nn.Embedding N(0, 1), RMSNorm ones, LoRA B zeros), and a unit's values do not depend on which
  engine or world size built it.
"""
import math
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from building_llm_from_scratch_amd.config import get_config
from building_llm_from_scratch_amd.models import build_model, replace_linear_with_lora
from building_llm_from_scratch_amd.parallel import setup_engine
from building_llm_from_scratch_amd.train.optim import FusedAdamW


def _cfg():
    return get_config("llama3_2", "1B").replace(context_length=16, emb_dim=64, n_heads=4, n_kv_groups=2,
                                                hidden_dim=96, n_layers=3, vocab_size=97, dtype=torch.float32)


def _meta_model(lora=False):
    m = build_model(_cfg(), device="meta")
    if lora:
        for p in m.parameters():
            p.requires_grad = False
        replace_linear_with_lora(m, rank=4, alpha=8)
    return m


def _batches():
    g = torch.Generator().manual_seed(7)
    return [torch.randint(0, 97, (4, 17), generator=g) for _ in range(3)]


def _train(m, opt, batches):
    losses = []
    for b in batches:
        opt.zero_grad()
        loss = m(b[:, :-1], b[:, 1:])
        loss.backward()
        opt.clip_grad_norm_(1.0)
        opt.step()
        losses.append(loss.item())
    return losses


def _reference():
    m = _meta_model()
    setup_engine(m, "local", device="cpu")
    init = {k: v.clone() for k, v in m.state_dict().items()}
    opt = FusedAdamW(m, lr=1e-2, weight_decay=0.1)
    losses = _train(m, opt, _batches())
    return init, {k: v.clone() for k, v in m.state_dict().items()}, losses


def _worker(rank, world, kind, out, store):
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    try:
        def no_broadcast(*a, **k):
            raise AssertionError("a meta-built model must not be broadcast")
        dist.broadcast = no_broadcast
        m = _meta_model()
        eng = setup_engine(m, kind, device="cpu", bucket_mb=0.05, prefetch=1)
        assert eng.deferred_init
        opt = FusedAdamW(m, lr=1e-2, weight_decay=0.1, engine=eng)
        per = 4 // world
        losses = _train(m, opt, [b[rank * per:(rank + 1) * per] for b in _batches()])
        t = torch.tensor(losses)
        dist.all_reduce(t)
        sd = eng.full_state_dict() if hasattr(eng, "full_state_dict") else \
            {k: v.detach().clone() for k, v in m.state_dict().items()}
        if rank == 0:
            torch.save({"sd": sd, "losses": (t / world).tolist()}, out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,world", [("fsdp", 2), ("fsdp", 4), ("ddp", 2), ("zero1", 2)])
def test_meta_built_engines_match_single_process(kind, world):
    _, ref_sd, ref_losses = _reference()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_worker, args=(world, kind, out, os.path.join(d, "store")), nprocs=world, join=True,
                           start_method="spawn")
        res = torch.load(out, weights_only=True)
    for a, b in zip(res["losses"], ref_losses):
        assert abs(a - b) < 1e-4, (res["losses"], ref_losses)
    for k in ref_sd:
        assert torch.allclose(res["sd"][k].float(), ref_sd[k].float(), atol=1e-4, rtol=1e-4), k


def test_meta_init_follows_module_defaults_and_is_deterministic():
    init, _, _ = _reference()
    init2, _, _ = _reference()
    for k in init:
        assert torch.equal(init[k], init2[k]), k
    d = 64
    w = init["trf_blocks.0.att.W_query.weight"]
    bound = 1.0 / math.sqrt(d)                      # kaiming_uniform(a=sqrt 5) on fan_in d
    assert w.abs().max() <= bound + 1e-6 and w.abs().max() > 0.9 * bound
    e = init["tok_emb.weight"]
    assert abs(e.std().item() - 1.0) < 0.1            # nn.Embedding: N(0, 1)
    assert torch.equal(init["trf_blocks.1.norm1.weight"], torch.ones(d))
    # different units get different draws
    assert not torch.equal(init["trf_blocks.0.att.W_query.weight"], init["trf_blocks.1.att.W_query.weight"])


def test_meta_built_lora_init():
    m = _meta_model(lora=True)
    setup_engine(m, "local", device="cpu")
    sd = m.state_dict()
    a = sd["trf_blocks.0.att.W_query.lora.A"]
    assert a.abs().max() > 0
    assert torch.count_nonzero(sd["trf_blocks.0.att.W_query.lora.B"]) == 0
    assert sd["trf_blocks.0.att.W_query.linear.weight"].abs().max() > 0


def test_meta_init_leaves_caller_rng_untouched():
    """Per-unit seeded initialisation runs under a forked RNG: the caller's stream continues
    exactly where it was (dropout, sampling and shuffling are not re-seeded by the build)."""
    torch.manual_seed(4242)
    expect = torch.rand(5)
    torch.manual_seed(4242)
    m = _meta_model()
    setup_engine(m, "local", device=torch.device("cpu"))
    assert torch.equal(torch.rand(5), expect)
