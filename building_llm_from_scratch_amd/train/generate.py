"""Autoregressive sampling (reference generate.py:4-75).

Same contract: sliding window of ``context_size`` tokens, optional top-k threshold, temperature
+ multinomial (else greedy argmax), stop only when EVERY row emits ``eos_id``.

* :func:`generate` — recomputes the window per token like the reference, but only the last
  position goes through the LM head (``last_only=True``).
* :func:`generate_cached` — KV-cache decode: one prefill of the window, then one token per
  forward through the HIP decode-attention kernel over the cache (the window slides by
  re-prefilling, exactly reproducing the reference's conditioning).  Under FSDP the parameters
  are gathered once for the whole sample instead of once per token.
"""
from __future__ import annotations

from typing import Optional

import torch


def _sample(logits, temperature, top_k, generator):
    logits = logits.float()
    if top_k is not None:
        top, _ = torch.topk(logits, top_k)
        logits = torch.where(logits < top[:, -1:], torch.full_like(logits, float("-inf")), logits)
    if temperature > 0.0:
        probs = torch.softmax(logits / temperature, dim=-1)
        return torch.multinomial(probs, num_samples=1, generator=generator)
    return torch.argmax(logits, dim=-1, keepdim=True)


@torch.no_grad()
def generate_cached(model, idx: torch.Tensor, max_new_tokens: int, context_size: int, temperature: float = 0.0,
                    top_k: Optional[int] = None, eos_id: Optional[int] = None,
                    generator: Optional[torch.Generator] = None) -> torch.Tensor:
    was_training = model.training
    model.eval()
    device = next(model.parameters()).device
    idx = idx.to(device)
    B = idx.shape[0]
    eng = model.rctx.engine
    resident = eng.params_resident() if hasattr(eng, "params_resident") else _null()
    with resident:
        cache = model.new_kv_cache(B, context_size)
        cond = idx[:, -context_size:]
        logits = model.forward_cached(cond, cache, 0)
        pos = cond.shape[1]
        for i in range(max_new_tokens):
            idx_next = _sample(logits, temperature, top_k, generator)
            if eos_id is not None and bool((idx_next == eos_id).all()):
                break
            idx = torch.cat((idx, idx_next), dim=1)
            if i == max_new_tokens - 1:
                break
            if pos >= context_size:          # window full: slide by re-prefilling
                cond = idx[:, -context_size:]
                logits = model.forward_cached(cond, cache, 0)
                pos = context_size
            else:
                logits = model.forward_cached(idx_next, cache, pos)
                pos += 1
    model.train(was_training)
    return idx


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


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
