"""Flat parameter storage for model *units*.

A unit is a logical group of parameters that is computed, communicated and optimised as
one piece: the embedding(s), one transformer block, or the final-norm + LM head.  Each
unit stores its parameters in (at most) two contiguous buffers — trainable and frozen —
and the named ``nn.Parameter`` objects the user / state_dict sees are *views* into them.

Why this layout (MI355X-first, not a reference translation):
  * fused GEMM operands for free: a block lays out ``[W_query; W_key; W_value]`` and
    ``[fc1; fc2]`` adjacently, so the fused QKV / gate-up weights are plain views
    (one hipBLASLt GEMM each, no per-step concatenation);
  * weight gradients are written by the unit's backward straight into a flat gradient
    buffer, which IS the DDP all-reduce bucket / FSDP reduce-scatter input / optimizer
    input — no copies, no per-parameter collectives (the reference's ZeRO issues one
    broadcast per parameter);
  * FSDP shards whole units: one all_gather_into_tensor / reduce_scatter_tensor per unit.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

ALIGN = 64  # elements; every fused group starts 128-B aligned for bf16


class FlatBuffer:
    """One contiguous buffer holding an ordered list of fused groups."""

    def __init__(self, groups: List[List[nn.Parameter]], dtype: torch.dtype, device,
                 pad_to: int = 1, storage: Optional[torch.Tensor] = None,
                 grad_storage: Optional[torch.Tensor] = None):
        self.groups = [g for g in groups if g]
        self.index: Dict[int, Tuple[int, torch.Size]] = {}
        off = 0
        for g in self.groups:
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            for p in g:
                self.index[id(p)] = (off, p.shape)
                off += p.numel()
        self.numel_used = off
        total = max((off + pad_to - 1) // pad_to * pad_to, pad_to)
        self.numel = total
        self.dtype = dtype
        self.device = torch.device(device)
        if storage is not None:
            assert storage.numel() >= total and storage.dtype == dtype
            self.data = storage[:total]
        else:
            self.data = torch.zeros(total, dtype=dtype, device=device)
        self.params: List[nn.Parameter] = [p for g in self.groups for p in g]
        self.grad: Optional[torch.Tensor] = None
        self._grad_storage = grad_storage

    @staticmethod
    def size_of(groups: List[List[nn.Parameter]], pad_to: int = 1) -> int:
        off = 0
        for g in groups:
            if not g:
                continue
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            off += sum(p.numel() for p in g)
        return max((off + pad_to - 1) // pad_to * pad_to, pad_to)

    def view(self, buf: torch.Tensor, p: nn.Parameter) -> torch.Tensor:
        off, shape = self.index[id(p)]
        return buf[off:off + shape.numel()].view(shape)

    def fused_view(self, buf: torch.Tensor, ps: Sequence[nn.Parameter]) -> torch.Tensor:
        """Rows of all ``ps`` stacked: [sum(rows), cols]; asserts they are adjacent."""
        off0, shape0 = self.index[id(ps[0])]
        cols = shape0[-1] if len(shape0) > 1 else 1
        off, rows = off0, 0
        for p in ps:
            o, s = self.index[id(p)]
            assert o == off, "fused parameters are not adjacent in the flat buffer"
            assert (s[-1] if len(s) > 1 else 1) == cols
            off += s.numel()
            rows += s.numel() // cols
        v = buf[off0:off]
        return v.view(rows, cols) if len(shape0) > 1 else v

    def bind(self):
        """Re-point every parameter's ``.data`` at its view (and ``.grad`` if allocated)."""
        for p in self.params:
            if p.is_meta:   # set_data cannot change a tensor's device type: swap the impl in place
                torch.utils.swap_tensors(p, nn.Parameter(self.view(self.data, p), requires_grad=p.requires_grad))
            else:
                p.data = self.view(self.data, p)
            if self.grad is not None:
                p.grad = self.view(self.grad, p)

    def alloc_grad(self, dtype: Optional[torch.dtype] = None):
        if self._grad_storage is not None:
            self.grad = self._grad_storage[:self.numel]
        else:
            self.grad = torch.zeros(self.numel, dtype=dtype or self.dtype, device=self.device)
        for p in self.params:
            p.grad = self.view(self.grad, p)


class FlatUnit:
    """A unit = trainable FlatBuffer + frozen FlatBuffer built from a fused-group layout."""

    def __init__(self, name: str, index: int):
        self.name = name
        self.index = index
        self.train: Optional[FlatBuffer] = None
        self.frozen: Optional[FlatBuffer] = None
        self._owner: Dict[int, FlatBuffer] = {}
        # distributed-engine state (set by parallel/*)
        self.state: dict = {}

    # ------------------------------------------------------------------ build
    def flatten(self, layout: List[List[nn.Parameter]], device, dtype: torch.dtype, pad_to: int = 1,
                grad_dtype: Optional[torch.dtype] = None, train_storage=None, train_grad_storage=None):
        seen = set()
        for g in layout:
            for p in g:
                assert id(p) not in seen, "parameter listed twice in a unit layout"
                seen.add(id(p))
        tr = [[p for p in g if p.requires_grad] for g in layout]
        fz = [[p for p in g if not p.requires_grad] for g in layout]
        self.train = FlatBuffer(tr, dtype, device, pad_to, train_storage, train_grad_storage) if any(tr) else None
        self.frozen = FlatBuffer(fz, dtype, device, pad_to) if any(fz) else None
        self._owner = {}
        for fb in (self.train, self.frozen):
            if fb is None:
                continue
            with torch.no_grad():
                for p in fb.params:
                    if not p.is_meta:   # meta-built model: values come from BaseLM.init_unit_
                        fb.view(fb.data, p).copy_(p.data.to(device=device, dtype=dtype))
                    self._owner[id(p)] = fb
            fb.bind()
        if self.train is not None:
            self.train.alloc_grad(grad_dtype)

    # ------------------------------------------------------------------ access
    def data(self, p: nn.Parameter) -> torch.Tensor:
        fb = self._owner[id(p)]
        return fb.view(fb.data, p)

    def grad(self, p: nn.Parameter) -> Optional[torch.Tensor]:
        fb = self._owner[id(p)]
        if fb is not self.train or fb.grad is None:
            return None
        return fb.view(fb.grad, p)

    def fused_data(self, ps: Sequence[nn.Parameter]) -> torch.Tensor:
        fb = self._owner[id(ps[0])]
        assert all(self._owner[id(p)] is fb for p in ps)
        return fb.fused_view(fb.data, ps)

    def fused_grad(self, ps: Sequence[nn.Parameter]) -> Optional[torch.Tensor]:
        fb = self._owner[id(ps[0])]
        if fb is not self.train or fb.grad is None:
            return None
        return fb.fused_view(fb.grad, ps)

    def trainable(self, p: nn.Parameter) -> bool:
        return self._owner.get(id(p)) is self.train and self.train is not None

    def buffers(self):
        return [fb for fb in (self.train, self.frozen) if fb is not None]

    def numel(self) -> int:
        return sum(fb.numel_used for fb in self.buffers())


def split_layout(layout: List[List[nn.Parameter]]):
    """(trainable groups, frozen groups) of a unit layout."""
    return ([[p for p in g if p.requires_grad] for g in layout],
            [[p for p in g if not p.requires_grad] for g in layout])
