"""Autoregressive sampling (reference generate.py:4-75).

Same contract: sliding window of ``context_size`` tokens, optional top-k threshold, temperature
+ multinomial (else greedy argmax), stop only when EVERY row emits ``eos_id``.

* :func:`generate` — recomputes the window per token like the reference, but only the last
  position goes through the LM head (``last_only=True``).
* :func:`generate_cached` — KV-cache decode: one prefill of the window, then one token per
  forward through the HIP decode-attention kernel over the cache (the window slides by
  re-prefilling, exactly reproducing the reference's conditioning).  Under FSDP the parameters
  are gathered once for the whole sample instead of once per token.  Tokens go into a
  preallocated buffer and the all-rows-eos stop test runs every ``EOS_CHECK_EVERY`` tokens (the
  output is cut at the first all-eos step, so the result is identical): the host never waits
  on the GPU per token, so each token's ~12 launches per layer queue up behind the previous
  token's kernels instead of running while the GPU idles.
* On the GPU the single-token step (every layer: norm, QKV GEMM, RoPE, K/V append + decode
  attention, projections, MLP, head) is captured ONCE per sample into a HIP graph
  (``torch.cuda.CUDAGraph``) with the position kept in device memory, and replayed per token:
  one graph launch instead of ~12 kernel launches per layer (the decode loop is launch-bound
  below Llama-3-8B size).  ``BLLM_DECODE_GRAPH=0`` runs it eagerly.
"""
from __future__ import annotations

import os

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


EOS_CHECK_EVERY = int(os.environ.get("BLLM_EOS_CHECK_EVERY", "16"))


def _graph_enabled() -> bool:
    return os.environ.get("BLLM_DECODE_GRAPH", "1") != "0"


class DecodeGraph:
    """A model's single-token decode step (``forward_cached_dev``) captured into a HIP graph.
    Capture runs with the position set to the cache's LAST slot, so the warm-up / capture
    passes only write that slot, which every later decode step overwrites before reading it."""

    def __init__(self, model, cache, B: int, device):
        Tmax = cache[0][0].shape[2]
        self.idx = torch.zeros(B, 1, dtype=torch.long, device=device)
        self.pos = torch.full((1,), Tmax - 1, dtype=torch.int32, device=device)
        cur = torch.cuda.current_stream(device)
        side = torch.cuda.Stream(device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):          # warm-up: hipBLASLt heuristics, allocator pool
            for _ in range(2):
                model.forward_cached_dev(self.idx, cache, self.pos)
        cur.wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: the sample print runs mid-epoch while DataLoader worker / pin-memory
        # threads may make allocator or event calls; in "global" mode those would invalidate
        # (or be rejected during) this capture
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.logits = model.forward_cached_dev(self.idx, cache, self.pos)

    def step(self, idx_next: torch.Tensor, pos: int) -> torch.Tensor:
        self.idx.copy_(idx_next)
        self.pos.fill_(pos)
        self.graph.replay()
        return self.logits


@torch.no_grad()
def generate_cached(model, idx: torch.Tensor, max_new_tokens: int, context_size: int, temperature: float = 0.0,
                    top_k: Optional[int] = None, eos_id: Optional[int] = None,
                    generator: Optional[torch.Generator] = None) -> torch.Tensor:
    was_training = model.training
    model.eval()
    device = next(model.parameters()).device
    idx = idx.to(device)
    B, T0 = idx.shape
    out = torch.empty(B, T0 + max(max_new_tokens, 0), dtype=idx.dtype, device=device)
    out[:, :T0] = idx
    n = checked = T0
    eng = model.rctx.engine
    resident = eng.params_resident() if hasattr(eng, "params_resident") else _null()
    with resident:
        cache = model.new_kv_cache(B, context_size)
        cond = idx[:, -context_size:]
        logits = model.forward_cached(cond, cache, 0) if max_new_tokens > 0 else None
        pos = cond.shape[1]
        dec = None
        if max_new_tokens > 8 and _graph_enabled() and hasattr(model, "decode_graph_ok") \
                and model.decode_graph_ok(cache):
            logits = logits.clone()            # the prefill output must survive the capture
            dec = DecodeGraph(model, cache, B, device)
        for i in range(max_new_tokens):
            idx_next = _sample(logits, temperature, top_k, generator)
            out[:, n] = idx_next[:, 0]
            n += 1
            last = i == max_new_tokens - 1
            if eos_id is not None and (n - checked >= EOS_CHECK_EVERY or last):
                # reference semantics (generate.py:68-70): stop before the first step at which
                # EVERY row sampled eos; later tokens were speculative and are dropped
                alleos = (out[:, checked:n] == eos_id).all(dim=0)
                if bool(alleos.any()):
                    n = checked + int(alleos.nonzero()[0, 0])
                    break
                checked = n
            if last:
                break
            if pos >= context_size:          # window full: slide by re-prefilling
                cond = out[:, n - context_size:n]
                logits = model.forward_cached(cond, cache, 0)
                pos = context_size
            elif dec is not None:
                logits = dec.step(idx_next, pos)
                pos += 1
            else:
                logits = model.forward_cached(idx_next, cache, pos)
                pos += 1
    model.train(was_training)
    return out[:, :n]


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
