"""World-size-8 shape / bucket-plan checks on one CPU process with torch's fake process group
(SURVEY §4 item 4): the DDP arena buckets, ZeRO-1 shards and FSDP per-unit shards are sized for
8 ranks exactly as on an 8-GPU node, and a training step runs through every engine hook.
The fake backend's collectives are no-ops, so only shapes / plumbing are asserted here; the
numerics at world size 2 are covered by test_distributed.py (gloo)."""
import multiprocessing as mp

import pytest

WORLD, RANK = 8, 3


def _worker(kind, q):
    try:
        import torch
        import torch.distributed as dist
        from torch.testing._internal.distributed.fake_pg import FakeStore

        from building_llm_from_scratch_amd.config import get_config
        from building_llm_from_scratch_amd.models import build_model
        from building_llm_from_scratch_amd.models.flat import ALIGN
        from building_llm_from_scratch_amd.parallel import setup_engine
        from building_llm_from_scratch_amd.train.optim import FusedAdamW

        dist.init_process_group("fake", rank=RANK, world_size=WORLD, store=FakeStore())
        cfg = get_config("llama3_2", "1B").replace(context_length=32, emb_dim=128, n_heads=4, n_kv_groups=2,
                                                   hidden_dim=192, n_layers=3, vocab_size=301, dtype=torch.float32)
        torch.manual_seed(0)
        m = build_model(cfg)
        eng = setup_engine(m, kind, device="cpu", bucket_mb=0.25)
        opt = FusedAdamW(m, lr=1e-3, weight_decay=0.1, engine=eng)
        n_params = sum(p.numel() for p in m.parameters())
        if kind == "fsdp":
            total = 0
            for u in eng.units:
                for fb in u.state["bufs"]:
                    assert fb.numel % (WORLD * ALIGN) == 0
                    assert fb.shard.numel() * WORLD == fb.numel
                    if fb is u.train:
                        assert fb.grad_shard.numel() == fb.shard.numel()
                    total += fb.numel
            assert total >= n_params
            assert len(opt.slots) == len(eng.units)
        else:
            ar = eng.arena
            covered = []
            for b, (s, e) in enumerate(ar.ranges):
                assert (e - s) % (WORLD * ALIGN) == 0
                covered += ar.buckets[b]
            assert covered == sorted(covered) == [u.index for u in m.units if u.train is not None]
            assert len(opt.slots) == len(ar.buckets)
            if kind == "zero1":
                for b, s in enumerate(opt.slots):
                    assert s.param.numel() * WORLD == ar.bucket_param(b).numel()
                    assert s.grad.numel() == s.param.numel()
            else:
                for b, s in enumerate(opt.slots):
                    assert s.param.numel() == ar.bucket_param(b).numel()
        idx = torch.randint(0, cfg.vocab_size, (2, 17))
        for _ in range(2):
            loss = m(idx[:, :-1], idx[:, 1:])
            loss.backward()
            opt.clip_grad_norm_(1.0)
            opt.step()
        assert torch.isfinite(loss)
        dist.destroy_process_group()
        q.put("ok")
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put(traceback.format_exc())


@pytest.mark.parametrize("kind", ["ddp", "zero1", "fsdp"])
def test_world8_plans_with_fake_pg(kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(kind, q))
    p.start()
    p.join(300)
    assert p.exitcode == 0, p.exitcode
    res = q.get(timeout=5)
    assert res == "ok", res

