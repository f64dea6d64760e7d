"""LoRA (reference lora.py:6-65).

Module-level semantics are kept exactly: ``A`` [in, r] kaiming-uniform(a=sqrt 5), ``B`` [r, out]
zeros, ``scaling = alpha / rank``, ``y = linear(x) + scaling * (x @ A @ B)``, and
``replace_linear_with_lora`` swaps EVERY ``nn.Linear`` recursively — output head included —
so checkpoints carry ``X.linear.weight`` / ``X.lora.A`` / ``X.lora.B`` keys.

Execution is not module-by-module: the unit compute (models/linear.py) folds the rank-r
update into the base GEMM's output in place (``y.addmm_(x@A, B, alpha=scaling)``) and, in
backward, produces only dA / dB (the frozen base weight gets no gradient buffer at all).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn


class LoRALayer(nn.Module):
    def __init__(self, in_dim: int, out_dim: int, rank: int, alpha: float, dtype=torch.float32,
                 device=None):
        super().__init__()
        self.rank = rank
        self.alpha = alpha
        self.scaling = alpha / rank
        self.A = nn.Parameter(torch.empty(in_dim, rank, dtype=dtype, device=device))
        self.B = nn.Parameter(torch.zeros(rank, out_dim, dtype=dtype, device=device))
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.kaiming_uniform_(self.A, a=math.sqrt(5))
        with torch.no_grad():
            self.B.zero_()

    def forward(self, x):
        return self.scaling * (x @ self.A @ self.B)


class LinearWithLoRA(nn.Module):
    def __init__(self, linear: nn.Linear, rank: int, alpha: float, dtype=None):
        super().__init__()
        self.linear = linear
        dt = dtype if dtype is not None else linear.weight.dtype
        self.lora = LoRALayer(linear.in_features, linear.out_features, rank, alpha, dtype=dt,
                              device=linear.weight.device)

    @property
    def in_features(self):
        return self.linear.in_features

    @property
    def out_features(self):
        return self.linear.out_features

    def forward(self, x):
        return self.linear(x) + self.lora(x)


def replace_linear_with_lora(model: nn.Module, rank: int, alpha: float, dtype=None) -> nn.Module:
    for name, module in model.named_children():
        if isinstance(module, nn.Linear):
            setattr(model, name, LinearWithLoRA(module, rank, alpha, dtype))
        else:
            replace_linear_with_lora(module, rank, alpha, dtype)
    return model
