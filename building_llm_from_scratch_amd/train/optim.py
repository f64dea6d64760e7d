"""Fused AdamW over flat unit buffers (+ on-device gradient clipping).

Reference: ``torch.optim.AdamW(model.parameters(), lr, weight_decay=0.1)`` /
``ZeroRedundancyOptimizer(AdamW)`` (build_components.py:243-258) and
``clip_grad_norm_(max_norm=1.0)`` (train.py:114-120).

Design: the optimizer steps *slots* — (param, grad) pairs of equal numel — supplied by the
distributed engine: whole flat buffers for single-process / DDP, the local shard for ZeRO-1
and FSDP.  Low-precision params get an fp32 master copy; exp_avg / exp_avg_sq are fp32.
One fused HIP launch per slot (ops.adamw_step_).  ``clip_grad_norm_`` computes the global
norm with one multi-tensor kernel (+ one all-reduce for sharded engines) and leaves the clip
coefficient ON DEVICE; ``step`` multiplies it in, so clipping never syncs with the host.
Weight decay applies to every parameter (the reference's single param group).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch

from .. import ops


@dataclass
class OptSlot:
    param: torch.Tensor      # updated in place (compute dtype)
    grad: torch.Tensor       # same numel
    name: str = ""
    units: tuple = ()        # unit indices whose parameters this slot updates


def local_slots(model) -> List[OptSlot]:
    return [OptSlot(c.unit.train.data, c.unit.train.grad, c.unit.name, (c.unit.index,))
            for c in model.computes if c.unit.train is not None]


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, model=None, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.01, slots: Optional[List[OptSlot]] = None, engine=None,
                 overlap: bool = False):
        if slots is None:
            eng = engine or (model.rctx.engine if model is not None else None)
            slots = eng.optimizer_slots(model) if eng is not None and hasattr(eng, "optimizer_slots") \
                else local_slots(model)
        self.slots = slots
        self.engine = engine or (model.rctx.engine if model is not None else None)
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__([s.param for s in slots], defaults)
        for s in slots:
            st = self.state[s.param]
            st["step"] = 0
            st["exp_avg"] = torch.zeros(s.param.numel(), dtype=torch.float32, device=s.param.device)
            st["exp_avg_sq"] = torch.zeros_like(st["exp_avg"])
            if s.param.dtype != torch.float32:
                st["master"] = s.param.detach().reshape(-1).float().clone()
        self._gscale: Optional[torch.Tensor] = None
        self.last_grad_norm: Optional[torch.Tensor] = None
        # data-parallel engines reduce with SUM; the 1/world average is folded in here
        self.grad_prescale = float(getattr(self.engine, "grad_prescale", 1.0))
        self._prescale_t: Optional[torch.Tensor] = None
        # Overlapped update (opt-in): the (HBM-bound) AdamW of unit i runs on a side HIP stream
        # and the next forward of unit i waits on its event only.  Measured on MI355X
        # (profiles/r1_llama3_8b_1gpu_v2.md): the forward GEMMs hold every CU's full register
        # file, so the update only runs in the gaps and slows the memory-bound forward kernels
        # that it does overlap (norm/rope/swiglu 15-60 us -> ~1 ms) -- no net gain, hence off by
        # default.  It pays when compute leaves CUs idle (small models, sharded updates).
        self.rctx = model.rctx if model is not None else None
        dev = slots[0].param.device if slots else torch.device("cpu")
        self.overlap = bool(overlap and dev.type == "cuda" and self.rctx is not None
                            and all(s.units for s in slots))
        self.opt_stream = torch.cuda.Stream(device=dev) if self.overlap else None

    # torch's zero_grad would try to walk p.grad of the slot tensors; the unit backward
    # OVERWRITES the flat gradients every step (accumulation is explicit), so this is a no-op
    def zero_grad(self, set_to_none: bool = True):
        self._gscale = None

    def grad_sq_norm(self) -> torch.Tensor:
        sq = ops.sq_norm_multi([s.grad.reshape(-1) for s in self.slots])
        if self.engine is not None and hasattr(self.engine, "all_reduce_grad_sq_norm"):
            sq = self.engine.all_reduce_grad_sq_norm(sq)
        return sq

    def clip_grad_norm_(self, max_norm: float = 1.0, extra_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Global L2 norm; sets the on-device multiplier min(1, max_norm/(norm+1e-6))."""
        sq = self.grad_sq_norm()
        scale = None
        if self.grad_prescale != 1.0:
            scale = torch.full((1,), self.grad_prescale, dtype=torch.float32, device=sq.device)
        if extra_scale is not None:  # gradients carry a loss scale: norm of the unscaled grads
            scale = extra_scale.float() if scale is None else scale * extra_scale.float()
        if scale is not None:
            sq = sq * scale ** 2
        norm = sq.sqrt()
        coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
        self._gscale = coef if scale is None else coef * scale
        self.last_grad_norm = norm
        return norm

    @torch.no_grad()
    def step(self, closure=None):
        g = self.param_groups[0]
        lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
        if self._gscale is None and self.grad_prescale != 1.0:
            if self._prescale_t is None:
                self._prescale_t = torch.full((1,), self.grad_prescale, dtype=torch.float32,
                                              device=self.slots[0].param.device)
            self._gscale = self._prescale_t
        if self.overlap:
            cur = torch.cuda.current_stream()
            self.opt_stream.wait_stream(cur)
            if self._gscale is not None:
                self._gscale.record_stream(self.opt_stream)
            with torch.cuda.stream(self.opt_stream):
                for s in self.slots:
                    self._update(s, lr, b1, b2, eps, wd)
                    if self.engine is not None and hasattr(self.engine, "after_slot_update"):
                        self.engine.after_slot_update(s)
                    ev = torch.cuda.Event()
                    ev.record(self.opt_stream)
                    for u in s.units:
                        self.rctx.param_ready[u] = ev
        else:
            for s in self.slots:
                self._update(s, lr, b1, b2, eps, wd)
                if self.engine is not None and hasattr(self.engine, "after_slot_update"):
                    self.engine.after_slot_update(s)
        self._gscale = None
        return None

    def _update(self, s, lr, b1, b2, eps, wd):
        st = self.state[s.param]
        st["step"] += 1
        ops.adamw_step_(s.param.reshape(-1), st.get("master"), s.grad.reshape(-1), st["exp_avg"],
                        st["exp_avg_sq"], lr, b1, b2, eps, wd, st["step"], self._gscale)

    @torch.no_grad()
    def reload_master(self):
        """Re-seed the fp32 master copies from the (just loaded) parameters.  Needed whenever
        weights are loaded after the optimizer was built: ``step`` writes master -> param, so a
        stale master would silently revert the load."""
        self.synchronize()
        for s in self.slots:
            st = self.state[s.param]
            if "master" in st:
                st["master"].copy_(s.param.detach().reshape(-1).float())

    def synchronize(self):
        """Block the current stream until every overlapped update has been applied."""
        if self.overlap:
            torch.cuda.current_stream().wait_stream(self.opt_stream)
            self.rctx.param_ready.clear()
