"""Independent eager-autograd models that follow the reference repository's math
(Models/GPT2/GPT2.py, Models/Llama/Llama3.py, common_components.py) — written here as a
test oracle for the hand-written unit forward/backward.  They read parameters from a
framework model's state_dict so both see identical weights."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _rope(x, cos, sin):
    # x [B, h, T, hd]; cos/sin [T, hd/2]
    half = x.shape[-1] // 2
    c = torch.cat([cos, cos], -1)[: x.shape[2]]
    s = torch.cat([sin, sin], -1)[: x.shape[2]]
    rot = torch.cat([-x[..., half:], x[..., :half]], -1)
    return x * c + rot * s


def _attn(q, k, v, causal=True):
    T = q.shape[2]
    s = q @ k.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if causal:
        s = s.masked_fill(torch.ones(T, T, dtype=torch.bool).triu(1), float("-inf"))
    return torch.softmax(s, -1) @ v


def llama_loss(sd, cfg, idx, targets, cos, sin, lora=None):
    """Eager Llama forward + CE (fp32)."""
    p = {k: v.float().detach().clone().requires_grad_(True) for k, v in sd.items()
         if not (k.endswith(".mask") or k.endswith(".cos") or k.endswith(".sin"))}
    B, T = idx.shape
    H, G, hd, d = cfg.n_heads, cfg.n_kv_groups, cfg.head_dim, cfg.emb_dim

    def lin(x, name):
        if lora and (name + ".linear.weight") in p:
            y = x @ p[name + ".linear.weight"].t()
            return y + lora * (x @ p[name + ".lora.A"] @ p[name + ".lora.B"])
        return x @ p[name + ".weight"].t()

    def rms(x, name):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * p[name + ".weight"]

    x = p["tok_emb.weight"][idx]
    for i in range(cfg.n_layers):
        pre = f"trf_blocks.{i}."
        h = rms(x, pre + "norm1")
        q = lin(h, pre + "att.W_query").view(B, T, H, hd).transpose(1, 2)
        k = lin(h, pre + "att.W_key").view(B, T, G, hd).transpose(1, 2)
        v = lin(h, pre + "att.W_value").view(B, T, G, hd).transpose(1, 2)
        q, k = _rope(q, cos, sin), _rope(k, cos, sin)
        k = k.repeat_interleave(H // G, 1)
        v = v.repeat_interleave(H // G, 1)
        o = _attn(q, k, v).transpose(1, 2).reshape(B, T, d)
        x = x + lin(o, pre + "att.out_proj")
        h = rms(x, pre + "norm2")
        x = x + lin(F.silu(lin(h, pre + "ff.fc1")) * lin(h, pre + "ff.fc2"), pre + "ff.fc3")
    x = rms(x, "final_norm")
    logits = lin(x, "out_head")
    loss = F.cross_entropy(logits.flatten(0, 1), targets.flatten())
    return loss, p


def gpt2_loss(sd, cfg, idx, targets, lora=None):
    p = {k: v.float().detach().clone().requires_grad_(True) for k, v in sd.items() if not k.endswith(".mask")}
    B, T = idx.shape
    H, hd, d = cfg.n_heads, cfg.head_dim, cfg.emb_dim

    def lin(x, name, bias=True):
        if lora and (name + ".linear.weight") in p:
            y = x @ p[name + ".linear.weight"].t()
            if (name + ".linear.bias") in p:
                y = y + p[name + ".linear.bias"]
            return y + lora * (x @ p[name + ".lora.A"] @ p[name + ".lora.B"])
        y = x @ p[name + ".weight"].t()
        if (name + ".bias") in p:
            y = y + p[name + ".bias"]
        return y

    def ln(x, name):
        return F.layer_norm(x, (d,), p[name + ".weight"], p[name + ".bias"], 1e-5)

    x = p["tok_emb.weight"][idx] + p["pos_emb.weight"][torch.arange(T)]
    for i in range(cfg.n_layers):
        pre = f"blocks.{i}."
        h = ln(x, pre + "norm1")
        q = lin(h, pre + "att.W_query").view(B, T, H, hd).transpose(1, 2)
        k = lin(h, pre + "att.W_key").view(B, T, H, hd).transpose(1, 2)
        v = lin(h, pre + "att.W_value").view(B, T, H, hd).transpose(1, 2)
        o = _attn(q, k, v).transpose(1, 2).reshape(B, T, d)
        x = x + lin(o, pre + "att.out_proj")
        h = ln(x, pre + "norm2")
        x = x + lin(F.gelu(lin(h, pre + "ff.layers.0")), pre + "ff.layers.2")
    x = ln(x, "norm")
    logits = lin(x, "output_head")
    loss = F.cross_entropy(logits.flatten(0, 1), targets.flatten())
    return loss, p
