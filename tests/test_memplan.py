"""The activation-checkpoint planner (train/memplan.py, ``bench.py --actv_ckpt auto``)."""
import pytest
import torch

from building_llm_from_scratch_amd.config import get_config
from building_llm_from_scratch_amd.train import memplan as M

GIB = 2 ** 30


def _cfg():
    return get_config("llama3", "8B").replace(dtype=torch.bfloat16)


# per-rank peaks measured on one MI355X with the FSDP engine (world 1), in GiB
MEASURED = [
    ("profiles/r2_bsweep_b24.log", 24, ["full"] * 31 + ["none"], 130.6),
    ("profiles/r2_bsweep_b40.log", 40, ["full"] * 31 + ["none"], 137.8),
    ("profiles/r2s3_bsweep_b64.log", 64, ["full"] * 31 + ["none"], 149.6),
    ("profiles/r2_bench_llama_none.log", 24, ["none"] * 32, 229.3),
    ("profiles/r2_bench_llama_full_seg2_b40.log", 40, ["full"] * 16 + ["none"] * 16, 214.7),
]


@pytest.mark.parametrize("src,B,modes,gib", MEASURED)
def test_estimate_matches_measured(src, B, modes, gib):
    est = M.estimate_peak(_cfg(), B, 1024, modes) / GIB
    assert abs(est - gib) <= 3.0, (src, est, gib)
    assert est >= gib - 0.5          # conservative within rounding: the planner must not under-shoot


def test_selective_saves_less_than_none():
    cfg = _cfg()
    s, n, f = (M.saved_bytes_per_token(cfg, m) for m in ("selective", "none", "full"))
    assert f < s < n
    # selective drops h1, h2 (2 d) and the SwiGLU act (F)
    assert n - s == 2 * (2 * cfg.emb_dim + cfg.hidden_dim)


def test_plan_world1_vs_world8_on_fake_budget():
    """At a tight budget one rank must recompute blocks; at world 8 FSDP shards 112 GiB of
    optimizer state and the same budget needs none."""
    cfg = _cfg()
    p1 = M.plan_ckpt(cfg, 48, 1024, world=1, budget=200 * GIB)
    p8 = M.plan_ckpt(cfg, 48, 1024, world=8, budget=200 * GIB)
    assert p1.fits and p8.fits
    assert p1.full_blocks > 0 and p8.full_blocks == 0
    assert p1.est_peak <= 200 * GIB and p8.est_peak <= 200 * GIB
    # minimality: one fewer fully recomputed block would not fit
    k = p1.full_blocks
    fewer = ["full"] * (k - 1) + ["selective"] * (cfg.n_layers - k + 1)
    assert M.estimate_peak(cfg, 48, 1024, fewer) > 200 * GIB
    # checkpointing never switches off
    for p in (p1, p8):
        assert "none" not in p.modes


def test_plan_monotone_in_budget_and_world():
    cfg = _cfg()
    ks = [M.plan_ckpt(cfg, 40, 1024, world=1, budget=b * GIB).full_blocks for b in (160, 180, 200, 220, 250)]
    assert ks == sorted(ks, reverse=True)
    kw = [M.plan_ckpt(cfg, 64, 1024, world=w, budget=200 * GIB).full_blocks for w in (1, 2, 4, 8)]
    assert kw == sorted(kw, reverse=True)


def test_plan_does_not_fit():
    p = M.plan_ckpt(_cfg(), 40, 1024, world=1, budget=100 * GIB)
    assert not p.fits and p.full_blocks == 32


def test_device_capacity_caps_budget():
    assert M.budget_for(288e9) == M.DEFAULT_BUDGET            # 268 GiB device: the 250 GiB default holds
    assert M.budget_for(200 * GIB) == 200 * GIB - M.HEADROOM
    assert M.budget_for(None) == M.DEFAULT_BUDGET
    assert M.budget_for(64 * GIB, 250 * GIB) == 64 * GIB - M.HEADROOM


def test_replan_after_probe_adds_blocks():
    cfg = _cfg()
    p = M.plan_ckpt(cfg, 40, 1024, world=1, budget=250 * GIB)
    assert M.replan_after_probe(p, cfg, 40, 1024, 240 * GIB) is p        # measured under budget
    q = M.replan_after_probe(p, cfg, 40, 1024, 262 * GIB)
    assert q.full_blocks > p.full_blocks and q.est_peak <= 250 * GIB and q.fits


def test_block_modes_drive_the_model():
    from building_llm_from_scratch_amd.models import build_model
    cfg = get_config("llama3_2", "1B").replace(n_layers=4, emb_dim=64, n_heads=4, n_kv_groups=2, hidden_dim=96,
                                               vocab_size=128, context_length=16)
    m = build_model(cfg, use_actv_ckpt="selective")
    m.set_block_modes(["full", "selective", "selective", "none"])
    assert m.ckpt_summary() == {"full": 1, "selective": 2, "none": 1}
    assert [m.rctx.block_mode(i) for i in range(4)] == ["full", "selective", "selective", "none"]
    m.set_actv_ckpt("full")
    assert m.ckpt_summary()["full"] == 3


def test_lora_kaug_copies_counted():
    """A frozen base under LoRA keeps two augmented copies of the block weights per rank
    (models/linear.py _waug) unless FSDP shards the base: memplan counts them."""
    from building_llm_from_scratch_amd.config import get_config
    from building_llm_from_scratch_amd.train import memplan
    cfg = get_config("llama3", "8B")
    full = memplan.static_bytes(cfg, world=8, engine="ddp", elt=2, trainable_frac=1.0)
    lora = memplan.static_bytes(cfg, world=8, engine="ddp", elt=2, trainable_frac=0.0)
    blocks = cfg.n_layers * 218.11e6        # SURVEY §2.5 per-block params
    # full: params + grads + 12 B/param optimizer; lora: params + 2 block copies
    assert abs(lora - (cfg.num_params() * 2 + 2 * blocks * 2)) / lora < 0.01
    assert full > lora
    sharded = memplan.static_bytes(cfg, world=8, engine="fsdp", elt=2, trainable_frac=0.0)
    assert sharded < lora / 4    # no augmented copies under FSDP sharding
