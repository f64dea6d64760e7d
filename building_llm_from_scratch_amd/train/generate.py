"""Autoregressive sampling (reference generate.py:4-75).

Same contract: sliding window of ``context_size`` tokens, optional top-k threshold, temperature
+ multinomial (else greedy argmax), stop only when EVERY row emits ``eos_id``.  Each step runs
the unit forward with ``last_only=True`` so only the last position goes through the LM head
(the reference computes the full [B, T, V] logits per generated token).
"""
from __future__ import annotations

from typing import Optional

import torch


@torch.no_grad()
def generate(model, idx: torch.Tensor, max_new_tokens: int, context_size: int, temperature: float = 0.0,
             top_k: Optional[int] = None, eos_id: Optional[int] = None,
             generator: Optional[torch.Generator] = None) -> torch.Tensor:
    was_training = model.training
    model.eval()
    device = next(model.parameters()).device
    idx = idx.to(device)
    for _ in range(max_new_tokens):
        idx_cond = idx[:, -context_size:]
        logits = model(idx_cond, last_only=True)[:, -1, :].float()
        if top_k is not None:
            top, _ = torch.topk(logits, top_k)
            logits = torch.where(logits < top[:, -1:], torch.full_like(logits, float("-inf")), logits)
        if temperature > 0.0:
            probs = torch.softmax(logits / temperature, dim=-1)
            idx_next = torch.multinomial(probs, num_samples=1, generator=generator)
        else:
            idx_next = torch.argmax(logits, dim=-1, keepdim=True)
        if eos_id is not None and bool((idx_next == eos_id).all()):
            break
        idx = torch.cat((idx, idx_next), dim=1)
    model.train(was_training)
    return idx
