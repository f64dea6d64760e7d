"""ZeRO-1: data parallel with the optimizer state sharded over ranks.

Reference: ``ZeroRedundancyOptimizer(params, optimizer_class=AdamW, lr, weight_decay=0.1)`` on
top of DDP (build_components.py:250-256): gradients all-reduced by DDP, each rank steps its
greedy partition, then ONE BROADCAST PER PARAMETER re-syncs weights.

Here: per arena bucket, the gradient is REDUCE-SCATTERED (half the bytes of an all-reduce)
asynchronously as soon as the bucket's units finish backward; each rank runs the fused
AdamW on its contiguous 1/world shard (fp32 master + moments only for that shard); then one
all-gather per bucket rebuilds the full bf16 parameters in place.  With a mixed-precision
policy whose ``reduce_dtype`` differs from the parameter dtype (``bf16_hybrid``), each bucket's
gradient is cast once, reduce-scattered in the reduce dtype and cast back into the shard.
"""
from __future__ import annotations

from contextlib import contextmanager
from typing import Optional

import torch
import torch.distributed as dist

from ..models.base import LocalEngine
from ..train.optim import OptSlot
from .arena import Arena


class ZeroEngine(LocalEngine):
    def __init__(self, model, device, reduce_dtype: Optional[torch.dtype] = None, bucket_mb: float = 256.0, pg=None):
        self.pg = pg
        self.world_size = dist.get_world_size(pg)
        self.rank = dist.get_rank(pg)
        self.model = model
        dtype = next(model.parameters()).dtype
        # meta-built model: every rank initialises the same values (seeded per unit), no broadcast
        self.deferred_init = any(p.is_meta for p in model.parameters())
        self.reduce_dtype = reduce_dtype if reduce_dtype not in (None, dtype) else None
        self.arena = Arena(model, device, dtype, self.world_size, bucket_mb * 2 ** 20)
        self.bucket_mb = bucket_mb
        from .commstats import CommStats
        self.comm = CommStats(device, self.world_size)
        from . import force_comm
        self.no_comm = self.world_size == 1 and not force_comm()  # one rank: its shard is the whole bucket
        if not self.no_comm and not self.deferred_init:
            dist.broadcast(self.arena.param, src=0, group=pg)
            for u in model.units:
                if u.frozen is not None:
                    dist.broadcast(u.frozen.data, src=0, group=pg)
        self.grad_shards = []
        for b in range(len(self.arena.buckets)):
            if self.no_comm:
                self.grad_shards.append(self.arena.bucket_grad(b))
                continue
            n = self.arena.bucket_grad(b).numel() // self.world_size
            self.grad_shards.append(torch.zeros(n, dtype=dtype, device=device))
        self.grad_prescale = 1.0 / self.world_size
        self._pending = []
        self._works = []
        self._started = False
        self._ag_works = {}
        model.set_engine(self)

    def _shard(self, t: torch.Tensor) -> torch.Tensor:
        n = t.numel() // self.world_size
        return t[self.rank * n:(self.rank + 1) * n]

    def pre_backward(self, unit):
        if not self._started:
            self._started = True
            self._pending = [len(b) for b in self.arena.buckets]
            self._works = []

    def post_backward(self, unit):
        if unit.index not in self.arena.bucket_of:
            return
        b = self.arena.bucket_of[unit.index]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._launch(b)

    def _launch(self, b):
        if self.no_comm:
            return
        g = self.arena.bucket_grad(b)
        if self.reduce_dtype is not None:
            full = g.to(self.reduce_dtype)
            part = torch.empty(self.grad_shards[b].numel(), dtype=self.reduce_dtype, device=g.device)
            w = dist.reduce_scatter_tensor(part, full, group=self.pg, async_op=True)
            self.comm.issued("reduce_scatter", w, full.numel() * full.element_size())
            self._works.append((w, b, full, part))
        else:
            w = dist.reduce_scatter_tensor(self.grad_shards[b], g, group=self.pg, async_op=True)
            self.comm.issued("reduce_scatter", w, g.numel() * g.element_size())
            self._works.append((w, b, None, None))

    def finish_backward(self):
        for b, n in enumerate(self._pending):
            if n > 0:
                self._launch(b)
        for w, b, full, part in self._works:
            with self.comm.waiting("reduce_scatter"):
                w.wait()
            self.comm.completed(w)
            if part is not None:
                self.grad_shards[b].copy_(part)
        self._works = []
        self._started = False

    def optimizer_slots(self, model):
        return [OptSlot(self._shard(self.arena.bucket_param(b)), self.grad_shards[b], f"bucket{b}",
                        tuple(self.arena.buckets[b])) for b in range(len(self.arena.buckets))]

    def all_reduce_grad_sq_norm(self, sq: torch.Tensor) -> torch.Tensor:
        if not self.no_comm:
            with self.comm.waiting("all_reduce"):
                dist.all_reduce(sq, group=self.pg)
        return sq

    def after_slot_update(self, slot):
        if self.no_comm:
            return
        # one all-gather per bucket, issued right behind that bucket's AdamW (on the optimizer
        # stream when overlapped); unit i's next forward waits only for its own bucket
        b = self.arena.bucket_of[slot.units[0]]
        full = self.arena.bucket_param(b)
        shard = self._shard(full)
        inp = shard if full.device.type == "cuda" else shard.clone()  # RCCL all-gathers in place
        self._ag_works[b] = dist.all_gather_into_tensor(full, inp, group=self.pg, async_op=True)
        self.comm.issued("all_gather", self._ag_works[b], full.numel() * full.element_size())

    def pre_forward(self, unit):
        b = self.arena.bucket_of.get(unit.index)
        if b is not None and b in self._ag_works:
            with self.comm.waiting("all_gather"):
                w = self._ag_works.pop(b)
                w.wait()
            self.comm.completed(w)

    def sync(self):
        for w in self._ag_works.values():
            w.wait()
        self._ag_works = {}

    @contextmanager
    def params_resident(self):
        self.model.rctx.sync_all_params()
        self.sync()
        yield

    @torch.no_grad()
    def load_full_state_dict(self, sd, strict: bool = True):
        """Parameters are replicated: load into the (arena-backed) parameter views; call
        ``optimizer.reload_master()`` afterwards."""
        self.sync()
        self.model.rctx.sync_all_params()
        return self.model.load_state_dict(sd, strict=strict)

    def full_state_dict(self):
        self.model.rctx.sync_all_params()
        self.sync()
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()} if self.rank == 0 else None
