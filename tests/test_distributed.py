"""DDP / ZeRO-1 / FSDP on CPU with gloo at world sizes 2, 4 and 8 must match single-process
training on the concatenated batch (fp32, several optimizer steps incl. clipping).

Beyond the basic matrix: flat sizes that force shard padding at world 4/8 (odd vocab / dims),
LoRA + FSDP at world 4, ``full`` activation checkpointing under DDP and FSDP, fp16 with loss
scaling under the engines, many tiny buckets, the ``bf16_hybrid`` reduce dtype (fp32 params,
bf16 collectives) and a full-state-dict load into already-sharded FSDP / ZeRO engines."""
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

STEPS = 3


def free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _cfg(family, odd=False):
    if odd:  # every flat's numel is coprime with 4 and 8: shards need tail padding
        return get_config("llama3_2", "1B").replace(context_length=16, emb_dim=36, n_heads=3, n_kv_groups=1,
                                                    hidden_dim=50, n_layers=3, vocab_size=101, dtype=torch.float32)
    if family == "llama":
        return get_config("llama3_2", "1B").replace(context_length=16, emb_dim=64, n_heads=4, n_kv_groups=2,
                                                    hidden_dim=96, n_layers=3, vocab_size=97, dtype=torch.float32)
    return get_config("GPT2", "124M").replace(context_length=16, emb_dim=64, n_heads=4, n_kv_groups=4,
                                              hidden_dim=256, n_layers=3, vocab_size=97, dtype=torch.float32,
                                              drop_rate=0.0)


def _data(cfg, rows=4):
    g = torch.Generator().manual_seed(7)
    return [torch.randint(0, cfg.vocab_size, (rows, 17), generator=g) for _ in range(STEPS)]


def _build(family, lora, ckpt="none", odd=False, dtype=None):
    torch.manual_seed(0)
    cfg = _cfg(family, odd)
    if dtype is not None:
        cfg = cfg.replace(dtype=dtype)
    m = build_model(cfg, use_actv_ckpt=ckpt)
    if lora:
        for p in m.parameters():
            p.requires_grad = False
        replace_linear_with_lora(m, rank=4, alpha=8)
        for mod in m.modules():
            if hasattr(mod, "B") and isinstance(mod.B, torch.nn.Parameter):
                torch.nn.init.normal_(mod.B, std=0.05)
    return cfg, m


def _train(m, opt, batches, loss_scale=None):
    losses = []
    for b in batches:
        opt.zero_grad()
        loss = m(b[:, :-1], b[:, 1:])
        if loss_scale is None:
            loss.backward()
            opt.clip_grad_norm_(0.5)
        else:  # fp16 path of the Trainer: scaled backward, norm of the unscaled grads
            (loss * loss_scale).backward()
            opt.clip_grad_norm_(0.5, extra_scale=torch.tensor([1.0 / loss_scale]))
        opt.step()
        losses.append(loss.float().item())
    return losses


def _reference(family, lora, odd=False, rows=4, dtype=None, loss_scale=None, ckpt="none", lr=1e-2):
    cfg, m = _build(family, lora, ckpt=ckpt, odd=odd, dtype=dtype)
    setup_engine(m, "local", device="cpu")
    opt = FusedAdamW(m, lr=lr, weight_decay=0.1)
    losses = _train(m, opt, _data(cfg, rows), loss_scale)
    return {k: v.clone() for k, v in m.state_dict().items()}, losses


def _worker(rank, world, kind, family, lora, ckpt, out, store, opts=None):
    # file-based rendezvous: no TCP-store port to race for between consecutive tests
    opts = opts or {}
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    try:
        cfg, m = _build(family, lora, ckpt, odd=opts.get("odd", False), dtype=opts.get("dtype"))
        if opts.get("load"):  # build from another init, then load the reference init into the live engine
            torch.manual_seed(99)
            for p in m.parameters():
                p.data.normal_()
        eng = setup_engine(m, kind, device="cpu", bucket_mb=opts.get("bucket_mb", 0.05),
                           reduce_dtype=opts.get("reduce_dtype"), prefetch=opts.get("prefetch", 1))
        opt = FusedAdamW(m, lr=opts.get("lr", 1e-2), weight_decay=0.1, engine=eng)
        if opts.get("load"):
            _, init = _build(family, lora, ckpt, odd=opts.get("odd", False), dtype=opts.get("dtype"))
            eng.load_full_state_dict(init.state_dict())
            opt.reload_master()
        rows = opts.get("rows", 4)
        per = rows // world
        batches = [b[rank * per:(rank + 1) * per] for b in _data(cfg, rows)]
        losses = _train(m, opt, batches, opts.get("loss_scale"))
        t = torch.tensor(losses)
        dist.all_reduce(t)
        sd = eng.full_state_dict() if hasattr(eng, "full_state_dict") else \
            {k: v.detach().clone() for k, v in m.state_dict().items()}
        if rank == 0:
            torch.save({"sd": sd, "losses": (t / world).tolist()}, out)
        dist.barrier()  # no rank tears the group down while a peer still has traffic in flight
    finally:
        dist.destroy_process_group()


def _spawn(world, kind, family, lora, ckpt="none", opts=None):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_worker, args=(world, kind, family, lora, ckpt, out, os.path.join(d, "store"), opts),
                           nprocs=world, join=True, start_method="spawn")
        return torch.load(out, weights_only=True)


def _check(res, ref_sd, ref_losses, tol=1e-4):
    for a, b in zip(res["losses"], ref_losses):
        assert abs(a - b) < tol, (res["losses"], ref_losses)
    sd = res["sd"]
    assert set(sd) == set(ref_sd)
    for k in ref_sd:
        assert torch.allclose(sd[k].float(), ref_sd[k].float(), atol=tol, rtol=tol), \
            (k, (sd[k].float() - ref_sd[k].float()).abs().max())


@pytest.mark.parametrize("kind", ["ddp", "zero1", "fsdp"])
@pytest.mark.parametrize("family,lora", [("llama", False), ("gpt2", False), ("llama", True)])
def test_engine_matches_single_process(kind, family, lora):
    ref_sd, ref_losses = _reference(family, lora)
    _check(_spawn(2, kind, family, lora), ref_sd, ref_losses)


@pytest.mark.parametrize("kind", ["ddp", "zero1", "fsdp"])
def test_world4_padding_forcing_flats(kind):
    ref_sd, ref_losses = _reference("llama", False, odd=True, rows=8)
    _check(_spawn(4, kind, "llama", False, opts=dict(odd=True, rows=8)), ref_sd, ref_losses)


@pytest.mark.parametrize("kind", ["fsdp", "zero1"])
def test_world8_padding_forcing_flats(kind):
    ref_sd, ref_losses = _reference("llama", False, odd=True, rows=8)
    _check(_spawn(8, kind, "llama", False, opts=dict(odd=True, rows=8)), ref_sd, ref_losses)


def test_world4_lora_fsdp():
    ref_sd, ref_losses = _reference("llama", True, rows=8)
    _check(_spawn(4, "fsdp", "llama", True, opts=dict(rows=8)), ref_sd, ref_losses)


@pytest.mark.parametrize("kind,prefetch", [("ddp", 1), ("fsdp", 1), ("fsdp", 3)])
def test_world4_full_actv_ckpt(kind, prefetch):
    """(fsdp, 3): three units gathered ahead in forward and in backward."""
    ref_sd, ref_losses = _reference("gpt2", False, rows=8)
    _check(_spawn(4, kind, "gpt2", False, ckpt="full", opts=dict(rows=8, prefetch=prefetch)), ref_sd, ref_losses)


@pytest.mark.parametrize("kind", ["ddp", "zero1", "fsdp"])
def test_world2_fp16_loss_scaling(kind):
    # small lr: AdamW normalises every update to ~lr, so fp16 rounding differences in the
    # (differently ordered) gradient sums move a parameter by at most ~2*lr per step
    ref_sd, ref_losses = _reference("llama", False, dtype=torch.float16, loss_scale=1024.0, lr=1e-4)
    res = _spawn(2, kind, "llama", False, opts=dict(dtype=torch.float16, loss_scale=1024.0, lr=1e-4))
    _check(res, ref_sd, ref_losses, tol=2e-3)


def test_world4_many_buckets_ddp():
    """~1 KiB buckets: dozens of async all-reduces in flight, launched out of order."""
    ref_sd, ref_losses = _reference("gpt2", False, rows=8)
    _check(_spawn(4, "ddp", "gpt2", False, opts=dict(rows=8, bucket_mb=0.001)), ref_sd, ref_losses)


@pytest.mark.parametrize("kind", ["zero1", "fsdp"])
def test_bf16_hybrid_reduce_dtype(kind):
    """fp32 params, bf16 gradient collectives (reference bf16_hybrid_policy): close to the fp32
    result but not bit-equal -- the reduction really ran in bf16."""
    ref_sd, ref_losses = _reference("llama", False)
    res = _spawn(2, kind, "llama", False, opts=dict(reduce_dtype=torch.bfloat16))
    _check(res, ref_sd, ref_losses, tol=3e-2)
    diff = max((res["sd"][k].float() - ref_sd[k].float()).abs().max().item() for k in ref_sd)
    assert diff > 0.0


@pytest.mark.parametrize("kind", ["fsdp", "zero1", "ddp"])
def test_load_full_state_dict_into_live_engine(kind):
    ref_sd, ref_losses = _reference("llama", False)
    _check(_spawn(2, kind, "llama", False, opts=dict(load=True)), ref_sd, ref_losses)


def test_fsdp_full_ckpt_and_zero2_mode():
    """FSDP with activation checkpointing ('full' recompute under re-gather)."""
    ref_sd, _ = _reference("llama", False)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_worker, args=(2, "fsdp", "llama", False, "full", out, os.path.join(d, "store")), nprocs=2,
                           join=True, start_method="spawn")
        sd = torch.load(out, weights_only=True)["sd"]
    for k in ref_sd:
        assert torch.allclose(sd[k].float(), ref_sd[k].float(), atol=1e-4, rtol=1e-4), k


@pytest.mark.parametrize("kind", ["ddp", "zero1", "fsdp"])
def test_world1_forced_comm_path(kind, monkeypatch):
    """BLLM_FORCE_COMM=1: the world-1 engines take their N>1 collective path (shards freed and
    re-gathered, reduce-scatter into grad shards) and still match single-process training."""
    monkeypatch.setenv("BLLM_FORCE_COMM", "1")
    ref_sd, ref_losses = _reference("llama", False)
    _check(_spawn(1, kind, "llama", False, ckpt="full"), ref_sd, ref_losses)
