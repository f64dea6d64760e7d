"""Activation-checkpoint granularity chosen from the HBM budget (``--actv_ckpt auto``).

The reference has one switch, ``--use_actv_ckpt``, which recomputes every block but the last
(``checkpoint_sequential(blocks, segments=n_layers)``, Llama3.py:198-199, GPT2.py:115-116) —
sized for a 16 GB T4.  On a 288 GB MI355X that recomputes far more than memory requires.
This module predicts the per-rank peak of one training step for a per-block mode assignment
and picks the cheapest assignment that fits a budget:

  * ``selective`` on every block (recompute the norm outputs and the SwiGLU / GELU activation,
    memory-bound passes that the backward folds into kernels it runs anyway), then
  * ``full`` on the first k blocks (save only the block input, re-run the block forward in
    backward) with k as small as the budget allows.

``none`` is never chosen: the planner keeps checkpointing on (BASELINE config #3 is "FSDP +
activation checkpointing").  FSDP / ZeRO-1 sharding of the flat params, gradients and fp32
optimizer state at world size N is part of the static term, so the choice is per N.

Model (bytes per rank):
    peak = static(N) + C0 + sum_i saved(mode_i) * tokens + W * tokens
  * ``saved`` — what a block's forward keeps for its backward, counted from the shapes the
    block code saves (models/llama.py / gpt2.py ``forward``);
  * ``static`` — param + grad flats in the compute dtype, fp32 master + Adam moments (sharded
    by the engine), plus FSDP's gathered working units;
  * ``C0`` (head workspace: logits chunk, transposed head weight, head gradient) and ``W``
    (the working set of the block in backward, per token) fitted to the Llama-3-8B peaks
    measured on MI355X (profiles/r2_bsweep_b*.log, r2_bench_llama_{none,selective,
    full_seg2_b40}.log): the fit is within 0.2 GiB for full checkpointing at B = 24-64 and
    for 16/32 blocks recomputed; ``none`` / ``selective`` measure 3.0 GiB above the linear
    fit (the head workspace then coincides with every block's saved set), which
    ``FWD_END_MARGIN`` covers.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

GIB = 2 ** 30
HEAD_WORKSPACE = 3.5 * GIB          # C0, fitted (see module docstring)
BLOCK_WORKING_PER_TOKEN = 44.6e3    # W, fitted: bytes per token of the block being back-propagated
FWD_END_MARGIN = 3.0 * GIB          # none/selective-heavy plans peak at the end of the forward
DEFAULT_BUDGET = 250 * GIB          # per-rank ceiling the planner fills (MI355X: 288 GB = 268 GiB)
HEADROOM = 18 * GIB                 # kept free below the device capacity when it is smaller


def saved_bytes_per_token(cfg, mode: str, elt: int = 2) -> float:
    """Bytes per token one block keeps for its backward in ``mode``."""
    d, F, H, hd = cfg.emb_dim, cfg.hidden_dim, cfg.n_heads, cfg.head_dim
    if mode == "full":
        return d * elt                                   # the block input only
    if cfg.is_llama:
        G = cfg.n_kv_groups
        # x, qkv, o, x2, gate|up (+ act, h1, h2 unless selective); r1, r2, lse in fp32
        n = d + (H + 2 * G) * hd + d + d + 2 * F
        f32 = 2 + H
        if mode == "none":
            n += F + 2 * d
        return n * elt + 4 * f32
    # GPT-2: x, qkv, o, x2, c_fc out (+ gelu out, h1, h2 unless selective); LN mean/rstd x2,
    # lse fp32; attention-dropout keep bits (1 per score) when dropout is on
    n = d + 3 * d + d + d + F
    f32 = 4 + H
    if mode == "none":
        n += F + 2 * d
    keep = H * cfg.context_length / 8 if cfg.drop_rate > 0 else 0
    return n * elt + 4 * f32 + keep


def static_bytes(cfg, world: int = 1, engine: str = "fsdp", elt: int = 2, prefetch: int = 1,
                 trainable_frac: float = 1.0) -> float:
    """Per-rank bytes that do not scale with the batch: params + grads (compute dtype), fp32
    master + Adam m, v; FSDP/ZeRO shard what they shard, FSDP adds its gathered units."""
    P = cfg.num_params()
    Pt = P * trainable_frac
    opt = 12 * Pt                                       # fp32 master, m, v
    # LoRA on a frozen, unsharded base (models/linear.py ``_waug``): every augmented block group
    # keeps [W | B^T] and its transpose [W^T ; B] across steps -- two more copies of the block
    # weights (the head and embedding are not augmented this way)
    kaug = 0.0
    if trainable_frac < 1.0 and not (engine == "fsdp" and world > 1):
        d, F = cfg.emb_dim, cfg.hidden_dim
        kv = cfg.n_kv_groups * cfg.head_dim if cfg.is_llama else d
        per_block = d * (d + 2 * kv) + d * d + (3 if cfg.is_llama else 2) * d * F
        kaug = 2 * per_block * cfg.n_layers * elt
    if engine == "fsdp" and world > 1:
        d, F, V = cfg.emb_dim, cfg.hidden_dim, cfg.vocab_size
        kv = cfg.n_kv_groups * cfg.head_dim
        unit = (d * (d + 2 * kv) + d * d + 3 * d * F) * elt          # one block, gathered
        head = V * d * elt                                           # head / embedding unit
        # prefetch+1 gathered units in forward/backward, 3 full unit gradients in flight
        # (reduce-scatter keep=2 + the one computing), the head unit kept across forward->backward
        gathered = (prefetch + 1) * max(unit, head) + 3 * unit + head
        return (P * elt + Pt * elt + opt) / world + gathered
    if engine == "zero1" and world > 1:
        return P * elt + Pt * elt + opt / world + kaug
    return P * elt + Pt * elt + opt + kaug


def estimate_peak(cfg, batch: int, seq: int, modes: List[str], world: int = 1, engine: str = "fsdp",
                  elt: int = 2, prefetch: int = 1, trainable_frac: float = 1.0) -> float:
    tokens = batch * seq
    act = sum(saved_bytes_per_token(cfg, m, elt) for m in modes) * tokens
    non_full = sum(m != "full" for m in modes)
    margin = FWD_END_MARGIN if non_full * 2 > len(modes) else 0.0
    return (static_bytes(cfg, world, engine, elt, prefetch, trainable_frac) + HEAD_WORKSPACE
            + act + BLOCK_WORKING_PER_TOKEN * tokens + margin)


@dataclass
class CkptPlan:
    modes: List[str]
    est_peak: float
    budget: float
    rule: str
    fits: bool = True
    candidates: list = field(default_factory=list)

    @property
    def full_blocks(self) -> int:
        return self.modes.count("full")

    def summary(self) -> dict:
        return {"full": self.modes.count("full"), "selective": self.modes.count("selective"),
                "none": self.modes.count("none"), "est_peak_gib": round(self.est_peak / GIB, 1),
                "budget_gib": round(self.budget / GIB, 1), "rule": self.rule}


def budget_for(device_total: Optional[float], budget: Optional[float] = None) -> float:
    """The per-rank ceiling: ``budget`` (default 250 GiB), never above device capacity minus
    ``HEADROOM``."""
    b = DEFAULT_BUDGET if budget is None else float(budget)
    if device_total:
        b = min(b, float(device_total) - HEADROOM)
    return b


def plan_ckpt(cfg, batch: int, seq: int, world: int = 1, engine: str = "fsdp", budget: Optional[float] = None,
              device_total: Optional[float] = None, elt: int = 2, prefetch: int = 1,
              trainable_frac: float = 1.0) -> CkptPlan:
    """Fewest fully recomputed blocks (all others ``selective``) whose estimated peak fits the
    budget.  Fully recomputed blocks are the first ones, as in checkpoint_sequential.  If even
    every block ``full`` does not fit, the all-full plan is returned with ``fits=False``."""
    b = budget_for(device_total, budget)
    L = cfg.n_layers
    cands = []
    for k in range(L + 1):
        modes = ["full"] * k + ["selective"] * (L - k)
        est = estimate_peak(cfg, batch, seq, modes, world, engine, elt, prefetch, trainable_frac)
        cands.append((k, est))
        if est <= b:
            rule = (f"fewest fully recomputed blocks (rest selective) with estimated peak "
                    f"<= {b / GIB:.0f} GiB per rank (train/memplan.py, world {world}, {engine})")
            return CkptPlan(modes, est, b, rule, True, cands)
    modes = ["full"] * L
    return CkptPlan(modes, cands[-1][1], b, "no plan fits the budget: every block recomputed", False, cands)


def replan_after_probe(plan: CkptPlan, cfg, batch: int, seq: int, measured_peak: float,
                       elt: int = 2) -> CkptPlan:
    """Correct the plan with a measured peak (one training step run with ``plan``): shift the
    estimate by the measured error and add fully recomputed blocks until it fits."""
    err = measured_peak - plan.est_peak
    if measured_peak <= plan.budget:
        return plan
    L = cfg.n_layers
    tokens = batch * seq
    save = (saved_bytes_per_token(cfg, "selective", elt) - saved_bytes_per_token(cfg, "full", elt)) * tokens
    k = plan.full_blocks
    est = measured_peak
    while est > plan.budget and k < L:
        k += 1
        est -= save
    modes = ["full"] * k + ["selective"] * (L - k)
    return CkptPlan(modes, est, plan.budget, plan.rule + f"; re-planned after a measured peak "
                    f"{measured_peak / GIB:.1f} GiB (estimate error {err / GIB:+.1f} GiB)",
                    est <= plan.budget, plan.candidates)
