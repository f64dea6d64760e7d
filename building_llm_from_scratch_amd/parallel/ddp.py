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
        self.comm = CommStats(device)
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

    # ------------------------------------------------------------------ hooks
    def pre_backward(self, unit):
        if not self._started:
            self._started = True
            self._pending = [len(b) for b in self.arena.buckets]
            self._works = []

    def post_backward(self, unit):
        if self.no_comm or not self.sync_grads or unit.index not in self.arena.bucket_of:
            return
        b = self.arena.bucket_of[unit.index]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._launch(b)

    def _launch(self, b):
        g = self.arena.bucket_grad(b)
        if self.reduce_dtype is not None:
            tmp = g.to(self.reduce_dtype)
            w = dist.all_reduce(tmp, group=self.pg, async_op=True)
            self._works.append((w, tmp, g))
        else:
            self._works.append((dist.all_reduce(g, group=self.pg, async_op=True), None, None))

    def finish_backward(self):
        if self.sync_grads and not self.no_comm:
            for b, n in enumerate(self._pending):
                if n > 0:  # units that saw no backward this step (e.g. frozen paths)
                    self._launch(b)
            for w, tmp, g in self._works:
                with self.comm.waiting("all_reduce"):
                    w.wait()
                if tmp is not None:
                    g.copy_(tmp)
        self._works = []
        self._started = False

    @torch.no_grad()
    def load_full_state_dict(self, sd, strict: bool = True):
        self.model.rctx.sync_all_params()
        return self.model.load_state_dict(sd, strict=strict)

    # ------------------------------------------------------------------ optimizer
    def optimizer_slots(self, model):
        return [OptSlot(self.arena.bucket_param(b), self.arena.bucket_grad(b), f"bucket{b}",
                        tuple(self.arena.buckets[b])) for b in range(len(self.arena.buckets))]
