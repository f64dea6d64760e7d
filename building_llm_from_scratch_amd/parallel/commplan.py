"""Collective plans of the engines: what one training step sends over RCCL, per op and bytes.

``step_plan(engine)`` derives, from an engine's own layout (DDP / ZeRO-1 arena buckets, FSDP
units), the ordered list of collectives one training step issues; ``Recorder`` captures the
collectives an engine really issues (it wraps the ``torch.distributed`` entry points).  The
tests (tests/test_comm_plan.py) check plan == recording on small models stepped on the fake
process group at world 8, then evaluate the plan at full size (meta-device models: Llama-3-8B
FSDP, GPT2-774M DDP / ZeRO-1) against SURVEY §2.5's message table (X6, X8-X10).

Reference call pattern (for contrast): torch DDP's 25 MiB all-reduce buckets plus
a per-forward buffer broadcast (X5); ZeRO's one broadcast per parameter per step (X7); FSDP's
per-unit all-gather / reduce-scatter with the Llama block stack in one root unit (X8-X9).

``fsdp_prefetch_depth`` sizes FSDP's all-gather prefetch from the per-unit gather time over
xGMI against the unit's compute time, instead of a fixed depth.
"""
from __future__ import annotations

import math
from contextlib import contextmanager
from typing import Dict, List

import torch
import torch.distributed as dist

# xGMI (MI355X): 7 links x ~153 GB/s per GPU, fully connected.  A ring collective is bound by
# one link per direction; RCCL's multi-channel all-gather reaches several links.  The planner
# uses the ring figure (conservative: a deeper prefetch only costs one gathered unit of memory).
XGMI_RING_BPS = 150e9
# forward MFMA throughput assumed for the unit's compute (conservative vs the measured 1.5 PF)
UNIT_FLOPS_PER_S = 1.0e15


def _elt(dtype) -> int:
    return torch.empty((), dtype=dtype).element_size()


def _op(op, phase, numel, dtype, what, world):
    return {"op": op, "phase": phase, "bytes": int(numel) * _elt(dtype), "dtype": str(dtype).replace("torch.", ""),
            "what": what, "world": world}


def step_plan(engine) -> List[Dict]:
    """Ordered collectives of one steady-state training step (forward, backward, clip, step)."""
    from .ddp import DDPEngine
    from .fsdp import FSDPEngine
    from .zero import ZeroEngine
    W = engine.world_size
    plan: List[Dict] = []
    if isinstance(engine, FSDPEngine):
        if engine.no_shard:
            return plan
        units = engine.units
        last = len(units) - 1
        # forward: one all-gather per buffer of every unit (units 0..prefetch_after_step-1 are
        # issued right after their optimizer update of the previous step: same bytes)
        for u in units:
            for fb in u.state["bufs"]:
                plan.append(_op("all_gather", "forward", fb.numel, fb.dtype, u.name, W))
        # backward (reverse): re-gather every unit resharded after forward (all but the head),
        # then reduce-scatter its gradient; the recompute of a checkpointed block reuses the
        # gather its backward already holds
        for u in reversed(units):
            if engine.reshard_after_forward and u.index != last:
                for fb in u.state["bufs"]:
                    plan.append(_op("all_gather", "backward", fb.numel, fb.dtype, u.name, W))
            if u.train is not None:
                rd = engine.reduce_dtype or u.train.grad.dtype
                plan.append(_op("reduce_scatter", "backward", u.train.numel, rd, u.name, W))
        plan.append(_op("all_reduce", "clip", 1, torch.float32, "grad_sq_norm", W))
        return plan
    if isinstance(engine, (DDPEngine, ZeroEngine)):
        if engine.no_comm:
            return plan
        ar = engine.arena
        zero = isinstance(engine, ZeroEngine)
        if zero:
            # buckets complete in reverse unit order during backward
            order = sorted(range(len(ar.buckets)), key=lambda b: -max(ar.buckets[b]))
            for b in order:
                g = ar.bucket_grad(b)
                rd = engine.reduce_dtype or g.dtype
                plan.append(_op("reduce_scatter", "backward", g.numel(), rd, f"bucket{b}", W))
        else:
            # DDP all-reduces launch groups (runs of buckets, merged by the warm-up adaptation)
            order = sorted(range(len(engine.groups)), key=lambda gi: -max(engine.groups[gi]))
            for gi in order:
                g = engine._group_grad(gi)
                rd = engine.reduce_dtype or g.dtype
                plan.append(_op("all_reduce", "backward", g.numel(), rd, f"group{gi}", W))
        if zero:
            plan.append(_op("all_reduce", "clip", 1, torch.float32, "grad_sq_norm", W))
            for b in range(len(ar.buckets)):
                p = ar.bucket_param(b)
                plan.append(_op("all_gather", "step", p.numel(), p.dtype, f"bucket{b}", W))
        return plan
    return plan


def summarize(plan: List[Dict]) -> Dict:
    out: Dict = {}
    for e in plan:
        k = (e["op"], e["phase"])
        c = out.setdefault(k, {"count": 0, "bytes": 0})
        c["count"] += 1
        c["bytes"] += e["bytes"]
    return out


class Recorder:
    """Record the collectives issued through ``torch.distributed`` (op, bytes, dtype, async).
    ``execute=False`` skips the real call and returns a completed dummy work (for meta-device
    models on the fake process group, whose collectives have no meta kernels)."""

    OPS = ("all_reduce", "all_gather_into_tensor", "reduce_scatter_tensor", "broadcast")
    NAMES = {"all_gather_into_tensor": "all_gather", "reduce_scatter_tensor": "reduce_scatter"}

    def __init__(self, execute: bool = True):
        self.execute = execute
        self.log: List[Dict] = []
        self.phase = "init"

    @contextmanager
    def active(self):
        saved = {n: getattr(dist, n) for n in self.OPS}

        class _Done:
            def wait(self):
                return True

            def is_completed(self):
                return True

        def wrap(name, fn):
            def inner(*args, **kw):
                # bytes of the full tensor: all-gather's output, reduce-scatter's input
                t = args[1] if name == "reduce_scatter_tensor" else args[0]
                self.log.append({"op": self.NAMES.get(name, name), "phase": self.phase,
                                 "bytes": t.numel() * t.element_size(), "dtype": str(t.dtype).replace("torch.", ""),
                                 "async": bool(kw.get("async_op", False))})
                if self.execute:
                    return fn(*args, **kw)
                return _Done() if kw.get("async_op", False) else None
            return inner

        for n, fn in saved.items():
            setattr(dist, n, wrap(n, fn))
        try:
            yield self
        finally:
            for n, fn in saved.items():
                setattr(dist, n, fn)


def fsdp_prefetch_depth(unit_bytes: float, unit_params: float, tokens: int, world: int,
                        link_bps: float = XGMI_RING_BPS, flops_per_s: float = UNIT_FLOPS_PER_S,
                        max_depth: int = 4) -> int:
    """Units to all-gather ahead so a unit's gather (ring over one xGMI link: (W-1)/W of the
    unit's bytes) is covered by the compute of the units before it (forward: 2 FLOP per param
    per token).  Llama-3-8B block (436 MB bf16) at 40 x 1024 tokens: gather 2.5 ms vs 18 ms of
    compute -> 1; at the reference's batch 4 (1.8 ms of compute) -> 2."""
    if world <= 1 or tokens <= 0:
        return 1
    gather_s = unit_bytes * (world - 1) / world / link_bps
    compute_s = 2.0 * unit_params * tokens / flops_per_s
    return int(max(1, min(max_depth, math.ceil(gather_s / max(compute_s, 1e-9)))))
