"""Offline pretrained-weight loaders (local files only — the GPU boxes have no network).

Key maps follow the reference loaders:
  * GPT-2 (Models/GPT2/load_weights.py:23-108): HF ``GPT2Model`` names ``wte``, ``wpe``,
    ``h.{b}.attn.c_attn`` (Conv1D [in, 3*out] -> split into Q/K/V and transposed),
    ``h.{b}.attn.c_proj``, ``h.{b}.mlp.c_fc|c_proj``, ``h.{b}.ln_1|ln_2``, ``ln_f``; the LM head
    is tied to ``wte``.  The reference writes into ``trf_blocks`` / ``final_norm`` / ``out_head``
    which GPTModel does not have (SURVEY §2.8 defect 4); here the real names are used.
  * Llama-3.x (load_weights_llama3.py:19-85): safetensors ``model.embed_tokens``,
    ``model.layers.{l}.self_attn.{q,k,v,o}_proj``, ``mlp.{gate,up,down}_proj -> fc1, fc2, fc3``,
    ``input_layernorm``, ``post_attention_layernorm``, ``model.norm``, ``lm_head`` (tied fallback).
  * Llama-2 (load_weights_llama2.py:18-71): Meta ``consolidated.00.pth`` names
    ``tok_embeddings``, ``layers.{l}.attention.w{q,k,v,o}``, ``feed_forward.w1 -> fc1, w3 -> fc2,
    w2 -> fc3``, ``attention_norm``, ``ffn_norm``, ``norm``, ``output``.

Files are read with safe loaders only (safetensors, ``torch.load(weights_only=True)``).
Call BEFORE LoRA replacement and before the model is flattened (or re-flatten afterwards).
"""
from __future__ import annotations

import glob
import os
from typing import Dict, Optional

import torch

GPT2_HF_DIRS = {"124M": "gpt2", "355M": "gpt2-medium", "774M": "gpt2-large", "1.5B": "gpt2-xl"}
LLAMA_DIRS = {"llama2": "Llama-2-7b", "llama3": "Llama-3-8B", "llama3_1": "Llama-3.1-8B", "llama3_2": "Llama-3.2-1B"}


def _read_tensors(path: str) -> Dict[str, torch.Tensor]:
    files = []
    if os.path.isdir(path):
        files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        if not files:
            files = sorted(glob.glob(os.path.join(path, "*.bin")) + glob.glob(os.path.join(path, "*.pth")))
    elif os.path.isfile(path):
        files = [path]
    if not files:
        raise FileNotFoundError(f"no weight files (*.safetensors, *.bin, *.pth) under '{path}'")
    out: Dict[str, torch.Tensor] = {}
    for f in files:
        if f.endswith(".safetensors"):
            from safetensors.torch import load_file
            out.update(load_file(f))
        else:
            out.update(torch.load(f, map_location="cpu", weights_only=True))
    return out


def _assign(param: torch.nn.Parameter, value: torch.Tensor, name: str):
    if tuple(param.shape) != tuple(value.shape):
        raise ValueError(f"Shape mismatch for '{name}': model {tuple(param.shape)} vs file {tuple(value.shape)}")
    with torch.no_grad():
        param.copy_(value.to(device=param.device, dtype=param.dtype))


def load_gpt2_weights(model, sd: Dict[str, torch.Tensor]):
    sd = {k[len("transformer."):] if k.startswith("transformer.") else k: v for k, v in sd.items()}
    _assign(model.pos_emb.weight, sd["wpe.weight"], "wpe")
    _assign(model.tok_emb.weight, sd["wte.weight"], "wte")
    d = model.cfg.emb_dim
    for b, blk in enumerate(model.blocks):
        p = f"h.{b}."
        qkv_w = sd[p + "attn.c_attn.weight"]          # Conv1D [in, 3*out]
        q, k, v = torch.split(qkv_w, d, dim=-1)
        _assign(blk.att.W_query.weight, q.t(), p + "q")
        _assign(blk.att.W_key.weight, k.t(), p + "k")
        _assign(blk.att.W_value.weight, v.t(), p + "v")
        if blk.att.W_query.bias is not None:
            qb, kb, vb = torch.split(sd[p + "attn.c_attn.bias"], d, dim=-1)
            _assign(blk.att.W_query.bias, qb, p + "qb")
            _assign(blk.att.W_key.bias, kb, p + "kb")
            _assign(blk.att.W_value.bias, vb, p + "vb")
        _assign(blk.att.out_proj.weight, sd[p + "attn.c_proj.weight"].t(), p + "c_proj")
        _assign(blk.att.out_proj.bias, sd[p + "attn.c_proj.bias"], p + "c_proj.b")
        _assign(blk.ff.layers[0].weight, sd[p + "mlp.c_fc.weight"].t(), p + "c_fc")
        _assign(blk.ff.layers[0].bias, sd[p + "mlp.c_fc.bias"], p + "c_fc.b")
        _assign(blk.ff.layers[2].weight, sd[p + "mlp.c_proj.weight"].t(), p + "mlp.c_proj")
        _assign(blk.ff.layers[2].bias, sd[p + "mlp.c_proj.bias"], p + "mlp.c_proj.b")
        _assign(blk.norm1.weight, sd[p + "ln_1.weight"], p + "ln_1")
        _assign(blk.norm1.bias, sd[p + "ln_1.bias"], p + "ln_1.b")
        _assign(blk.norm2.weight, sd[p + "ln_2.weight"], p + "ln_2")
        _assign(blk.norm2.bias, sd[p + "ln_2.bias"], p + "ln_2.b")
    _assign(model.norm.weight, sd["ln_f.weight"], "ln_f")
    _assign(model.norm.bias, sd["ln_f.bias"], "ln_f.b")
    _assign(model.output_head.weight, sd["wte.weight"], "wte (tied head)")


def load_llama3_weights(model, sd: Dict[str, torch.Tensor]):
    _assign(model.tok_emb.weight, sd["model.embed_tokens.weight"], "embed_tokens")
    for l, blk in enumerate(model.trf_blocks):
        p = f"model.layers.{l}."
        _assign(blk.att.W_query.weight, sd[p + "self_attn.q_proj.weight"], p + "q_proj")
        _assign(blk.att.W_key.weight, sd[p + "self_attn.k_proj.weight"], p + "k_proj")
        _assign(blk.att.W_value.weight, sd[p + "self_attn.v_proj.weight"], p + "v_proj")
        _assign(blk.att.out_proj.weight, sd[p + "self_attn.o_proj.weight"], p + "o_proj")
        _assign(blk.norm1.weight, sd[p + "input_layernorm.weight"], p + "input_layernorm")
        _assign(blk.ff.fc1.weight, sd[p + "mlp.gate_proj.weight"], p + "gate_proj")
        _assign(blk.ff.fc2.weight, sd[p + "mlp.up_proj.weight"], p + "up_proj")
        _assign(blk.ff.fc3.weight, sd[p + "mlp.down_proj.weight"], p + "down_proj")
        _assign(blk.norm2.weight, sd[p + "post_attention_layernorm.weight"], p + "post_attention_layernorm")
    _assign(model.final_norm.weight, sd["model.norm.weight"], "model.norm")
    head = sd.get("lm_head.weight", sd["model.embed_tokens.weight"])
    _assign(model.out_head.weight, head, "lm_head")


def load_llama2_weights(model, sd: Dict[str, torch.Tensor]):
    _assign(model.tok_emb.weight, sd["tok_embeddings.weight"], "tok_embeddings")
    for l, blk in enumerate(model.trf_blocks):
        p = f"layers.{l}."
        _assign(blk.att.W_query.weight, sd[p + "attention.wq.weight"], p + "wq")
        _assign(blk.att.W_key.weight, sd[p + "attention.wk.weight"], p + "wk")
        _assign(blk.att.W_value.weight, sd[p + "attention.wv.weight"], p + "wv")
        _assign(blk.att.out_proj.weight, sd[p + "attention.wo.weight"], p + "wo")
        _assign(blk.norm1.weight, sd[p + "attention_norm.weight"], p + "attention_norm")
        _assign(blk.ff.fc1.weight, sd[p + "feed_forward.w1.weight"], p + "w1")
        _assign(blk.ff.fc2.weight, sd[p + "feed_forward.w3.weight"], p + "w3")
        _assign(blk.ff.fc3.weight, sd[p + "feed_forward.w2.weight"], p + "w2")
        _assign(blk.norm2.weight, sd[p + "ffn_norm.weight"], p + "ffn_norm")
    _assign(model.final_norm.weight, sd["norm.weight"], "norm")
    _assign(model.out_head.weight, sd["output.weight"], "output")


def find_weights(model_name: str, num_params: str, weights_path: Optional[str] = None) -> str:
    cands = [weights_path] if weights_path else []
    if model_name == "GPT2":
        sub = GPT2_HF_DIRS[num_params]
        cands += [sub, os.path.join("hf_checkpoints", sub)]
        cands += glob.glob(os.path.join("hf_checkpoints", f"models--openai-community--{sub}", "snapshots", "*"))
    else:
        cands += [LLAMA_DIRS[model_name]]
    for c in cands:
        if c and os.path.exists(c):
            return c
    raise FileNotFoundError(
        f"--load_weights: no local weights for {model_name} {num_params} (looked in {cands}). This build is "
        f"offline: place the HF files there or pass --weights_path.")


def load_pretrained(model, model_name: str, num_params: str, weights_path: Optional[str] = None):
    path = find_weights(model_name, num_params, weights_path)
    sd = _read_tensors(path)
    if model_name == "GPT2":
        load_gpt2_weights(model, sd)
    elif model_name == "llama2":
        load_llama2_weights(model, sd)
    else:
        load_llama3_weights(model, sd)
    return path
