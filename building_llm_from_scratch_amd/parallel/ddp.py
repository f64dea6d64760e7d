"""Data parallelism with bucketed, backward-overlapped gradient all-reduce.

Reference: ``DDP(model, device_ids=[rank])`` (build_components.py:176) — 25 MiB buckets,
buffer broadcast before every training forward.

Here: parameters are broadcast once from rank 0; no buffers exist to sync (masks / RoPE
tables are recomputed deterministically, never communicated); gradients live in the
contiguous arena (parallel/arena.py) and each bucket's all-reduce is launched
asynchronously (RCCL runs it on its own HIP stream) the moment the last unit of that
bucket finishes its backward, overlapping with the remaining backward compute.  The
1/world averaging is folded into the optimizer's gradient scale (no extra pass).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..models.base import LocalEngine
from ..train.optim import OptSlot
from .arena import Arena


class DDPEngine(LocalEngine):
    def __init__(self, model, device, reduce_dtype: Optional[torch.dtype] = None, bucket_mb: float = 256.0,
                 pg=None, broadcast: bool = True):
        self.pg = pg
        self.world_size = dist.get_world_size(pg)
        self.rank = dist.get_rank(pg)
        self.model = model
        dtype = next(model.parameters()).dtype
        # meta-built model: every rank initialises the same values (seeded per unit), no broadcast
        self.deferred_init = any(p.is_meta for p in model.parameters())
        self.arena = Arena(model, device, dtype, self.world_size, bucket_mb * 2 ** 20)
        self.bucket_mb = bucket_mb
        from .commstats import CommStats
        self.comm = CommStats(device, self.world_size)
        self.adapt_log: List[dict] = []
        # launch groups: runs of consecutive arena buckets all-reduced as ONE collective over
        # their contiguous range (the arena keeps its buckets; the warm-up adaptation merges them)
        self._set_groups(bucket_mb)
        self.reduce_dtype = reduce_dtype if reduce_dtype not in (None, dtype) else None
        # a single rank has nothing to average with: no broadcast, no all-reduce (same hooks)
        from . import force_comm
        self.no_comm = self.world_size == 1 and not force_comm()
        if broadcast and not self.no_comm and not self.deferred_init:
            self._broadcast_params()
        self.grad_prescale = 1.0 / self.world_size
        self.sync_grads = True
        self._pending: List[int] = []
        self._works = []
        self._started = False
        model.set_engine(self)

    def _broadcast_params(self):
        dist.broadcast(self.arena.param, src=0, group=self.pg)
        for u in self.model.units:
            if u.frozen is not None:
                dist.broadcast(u.frozen.data, src=0, group=self.pg)

    def _set_groups(self, group_mb: float):
        """Group consecutive buckets (in backward completion order: last bucket first) until a
        group holds >= group_mb of gradient."""
        ar = self.arena
        elt = ar.grad.element_size()
        groups, cur, sz = [], [], 0
        for b in reversed(range(len(ar.buckets))):
            cur.insert(0, b)
            s, e = ar.ranges[b]
            sz += (e - s) * elt
            if sz >= group_mb * 2 ** 20:
                groups.append(cur)
                cur, sz = [], 0
        if cur:
            groups.append(cur)
        self.groups = groups[::-1]
        self.group_of = {b: gi for gi, g in enumerate(self.groups) for b in g}
        self.bucket_mb = group_mb

    # ------------------------------------------------------------------ hooks
    def pre_backward(self, unit):
        if not self._started:
            self._started = True
            self._pending = [sum(len(self.arena.buckets[b]) for b in g) for g in self.groups]
            self._works = []

    def post_backward(self, unit):
        if self.no_comm or not self.sync_grads or unit.index not in self.arena.bucket_of:
            return
        gi = self.group_of[self.arena.bucket_of[unit.index]]
        self._pending[gi] -= 1
        if self._pending[gi] == 0:
            self._launch(gi)

    def _group_grad(self, gi):
        bs = self.groups[gi]
        return self.arena.grad[self.arena.ranges[bs[0]][0]:self.arena.ranges[bs[-1]][1]]

    def _launch(self, gi):
        g = self._group_grad(gi)
        if self.reduce_dtype is not None:
            tmp = g.to(self.reduce_dtype)
            w = dist.all_reduce(tmp, group=self.pg, async_op=True)
            self.comm.issued("all_reduce", w, tmp.numel() * tmp.element_size())
            self._works.append((w, tmp, g))
        else:
            w = dist.all_reduce(g, group=self.pg, async_op=True)
            self.comm.issued("all_reduce", w, g.numel() * g.element_size())
            self._works.append((w, None, None))

    def finish_backward(self):
        if self.sync_grads and not self.no_comm:
            for gi, n in enumerate(self._pending):
                if n > 0:  # units that saw no backward this step (e.g. frozen paths)
                    self._launch(gi)
            for w, tmp, g in self._works:
                with self.comm.waiting("all_reduce"):
                    w.wait()
                self.comm.completed(w)
                if tmp is not None:
                    g.copy_(tmp)
        self._works = []
        self._started = False

    def adapt(self, step_ms: float) -> Optional[dict]:
        """Warm-up adaptation: if the exposed all-reduce wait (MAX over ranks) exceeds
        ``ADAPT_FRAC`` of the step, double the launch-group size (fewer, larger all-reduces:
        per-collective latency amortised over more bytes on the point-to-point xGMI links).
        The same MAX on every rank keeps the collective order identical."""
        if self.no_comm:
            return None
        from .commstats import ADAPT_FRAC, max_over_ranks
        s = self.comm.summary()
        ar, step = max_over_ranks([s.get("all_reduce", {}).get("ms", 0.0), step_ms], self.pg,
                                  self.arena.grad.device)
        rec = {"exposed_all_reduce_ms": round(ar, 3), "step_ms": round(step, 2), "bucket_mib": self.bucket_mb}
        total_mb = self.arena.grad.numel() * self.arena.grad.element_size() / 2 ** 20
        if ar > ADAPT_FRAC * step and len(self.groups) > 1 and self.bucket_mb < total_mb:
            self._set_groups(self.bucket_mb * 2)
            rec["bucket_mib_new"] = self.bucket_mb
        self.adapt_log.append(rec)
        return rec

    @torch.no_grad()
    def load_full_state_dict(self, sd, strict: bool = True):
        self.model.rctx.sync_all_params()
        return self.model.load_state_dict(sd, strict=strict)

    # ------------------------------------------------------------------ optimizer
    def optimizer_slots(self, model):
        return [OptSlot(self.arena.bucket_param(b), self.arena.bucket_grad(b), f"bucket{b}",
                        tuple(self.arena.buckets[b])) for b in range(len(self.arena.buckets))]
