"""Fused (multi-)linear forward/backward on flat-unit views, with LoRA folded in.

A :class:`FusedLinear` covers one or more reference ``nn.Linear`` modules that share an
input (Q/K/V; gate/up) and whose weights are adjacent in the unit's flat buffer, so the
whole group is ONE GEMM ``y = x @ W_cat^T (+ b_cat) (+ residual)`` on hipBLASLt.  LoRA
members add ``scaling * (x @ A) @ B`` into their column slice of ``y`` in place.

Backward writes ``dW`` / ``db`` / ``dA`` / ``dB`` directly into the unit's flat gradient
buffer (``out=`` GEMMs; ``addmm_`` when accumulating micro-batches).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.nn as nn

from .. import ops

from .flat import FlatUnit
from .lora import LinearWithLoRA


@dataclass
class LinearSpec:
    module: nn.Module
    weight: nn.Parameter
    bias: Optional[nn.Parameter]
    lora_A: Optional[nn.Parameter] = None
    lora_B: Optional[nn.Parameter] = None
    scaling: float = 0.0

    @property
    def out_features(self) -> int:
        return self.weight.shape[0]


def resolve(mod: nn.Module) -> LinearSpec:
    if isinstance(mod, LinearWithLoRA):
        lin = mod.linear
        return LinearSpec(mod, lin.weight, lin.bias, mod.lora.A, mod.lora.B, mod.lora.scaling)
    assert isinstance(mod, nn.Linear), f"expected nn.Linear, got {type(mod)}"
    return LinearSpec(mod, mod.weight, mod.bias)


def layout_groups(specs: Sequence[LinearSpec]) -> List[List[nn.Parameter]]:
    """Fused layout: [all weights], [all biases], then each LoRA's A and B."""
    groups = [[s.weight for s in specs]]
    biases = [s.bias for s in specs if s.bias is not None]
    if biases:
        assert len(biases) == len(specs), "mixed bias / no-bias in a fused linear group"
        groups.append(biases)
    for s in specs:
        if s.lora_A is not None:
            groups.append([s.lora_A])
            groups.append([s.lora_B])
    return groups


def _mm_out(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, accumulate: bool):
    if accumulate:
        out.addmm_(a, b)
    else:
        torch.mm(a, b, out=out)


def _weight_grad(dy: torch.Tensor, x: torch.Tensor, gW: torch.Tensor, accumulate: bool):
    """gW[out, in] (+)= dy^T x, issued as gW^T = x^T dy into the transposed view: the same
    memory, but hipBLASLt then picks a kernel family that measured 3-6 % faster for the Llama
    projections on MI355X (tools/bench_gemm.py: dw_dyTx vs dw_xTdy_outT)."""
    if gW.is_cuda:
        _mm_out(x.t(), dy, gW.t(), accumulate)
    else:
        _mm_out(dy.t(), x, gW, accumulate)


class FusedLinear:
    def __init__(self, modules: Sequence[nn.Module]):
        self.modules = list(modules)
        self.specs: List[LinearSpec] = []

    def refresh(self):
        self.specs = [resolve(m) for m in self.modules]
        return self

    def layout(self) -> List[List[nn.Parameter]]:
        self.refresh()
        return layout_groups(self.specs)

    def bind(self, unit: FlatUnit):
        self.unit = unit
        ws = [s.weight for s in self.specs]
        self.W_params = ws
        self.b_params = [s.bias for s in self.specs] if self.specs[0].bias is not None else None
        self.cols = []
        c = 0
        for s in self.specs:
            self.cols.append((c, c + s.out_features))
            c += s.out_features
        self.out_total = c
        self.has_lora = any(s.lora_A is not None for s in self.specs)

    # views are re-fetched every call: FSDP may have re-materialised the storage
    def W(self):
        return self.unit.fused_data(self.W_params)

    def b(self):
        return self.unit.fused_data(self.b_params) if self.b_params else None

    # ------------------------------------------------------------------ fwd
    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None):
        W = self.W()
        b = self.b()
        if residual is not None:
            assert b is None
            y = torch.addmm(residual, x, W.t())
        elif b is not None:
            y = torch.addmm(b, x, W.t())
        else:
            y = torch.mm(x, W.t())
        xa = None
        if self.has_lora:
            xa = []
            for (c0, c1), s in zip(self.cols, self.specs):
                if s.lora_A is None:
                    xa.append(None)
                    continue
                A = self.unit.data(s.lora_A)
                B = self.unit.data(s.lora_B)
                t = torch.mm(x, A)
                y[:, c0:c1].addmm_(t, B, alpha=s.scaling)
                xa.append(t)
        return y, xa

    # ------------------------------------------------------------------ bwd
    def backward(self, dy: torch.Tensor, x: torch.Tensor, xa, need_dx: bool = True,
                 accumulate: bool = False, dx_acc: Optional[torch.Tensor] = None):
        """Returns dx (plus ``dx_acc`` if given) and writes parameter grads into the flat."""
        u = self.unit
        gW = u.fused_grad(self.W_params)
        if gW is not None:
            _weight_grad(dy, x, gW, accumulate)
        if self.b_params is not None:
            gb = u.fused_grad(self.b_params)
            if gb is not None:
                ops.bias_grad_(dy, gb, accumulate)
        dx = None
        if need_dx:
            W = self.W()
            if dx_acc is not None:
                dx = torch.addmm(dx_acc, dy, W)
            else:
                dx = torch.mm(dy, W)
        if self.has_lora:
            for (c0, c1), s, t in zip(self.cols, self.specs, xa):
                if s.lora_A is None:
                    continue
                A = u.data(s.lora_A)
                B = u.data(s.lora_B)
                dys = dy[:, c0:c1]
                dyB = torch.mm(dys, B.t())                                   # [N, r]
                gB = u.grad(s.lora_B)
                if gB is not None:
                    if accumulate:
                        gB.addmm_(t.t(), dys, alpha=s.scaling)
                    else:
                        torch.mm(t.t(), dys, out=gB)
                        gB.mul_(s.scaling)
                gA = u.grad(s.lora_A)
                if gA is not None:
                    if accumulate:
                        gA.addmm_(x.t(), dyB, alpha=s.scaling)
                    else:
                        torch.mm(x.t(), dyB, out=gA)
                        gA.mul_(s.scaling)
                if need_dx:
                    dx.addmm_(dyB, A.t(), alpha=s.scaling)
        return dx
