"""Model configuration registry.

Parity targets (reference, read-only):
  * GPT-2 sizes / constants  — Models/GPT2/config.py:5-50
  * Llama-2/3/3.1/3.2 dicts  — Models/Llama/config.py:8-71
  * ctx clamp to 1024 + RoPE theta rescale — Models/Llama/config.py:97-126,
    common_components.py:38-51
  * ``--debug`` tiny-model override — build_components.py:72-80
  * dtype override / qkv_bias-on-load — build_components.py:67-70

Differences from the reference (documented defects):
  * configs are immutable; ``get_config`` returns a fresh ``ModelConfig`` every call
    (reference mutates module-level dicts, defect 11);
  * Llama-2 gets ``rope_base`` 10000, ``eos_id`` 2 / ``eos_text`` ``</s>`` and
    ``n_kv_groups == n_heads`` (defect 1);
  * the context clamp is a parameter (``context_length``), default 1024 = parity.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Optional

import torch

# ---------------------------------------------------------------------------
# dtype / size mappings (reference utils.py:30-50)
# ---------------------------------------------------------------------------
datasize_mapping = {"fp32": 4, "fp16": 2, "bf16": 2}
datatype_mapping = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
model_params_mapping = {
    "GPT2": ["124M", "355M", "774M", "1.5B"],
    "llama2": ["7B"],
    "llama3": ["8B"],
    "llama3_1": ["8B"],
    "llama3_2": ["1B"],
}

DEFAULT_CONTEXT_LENGTH = 1024


@dataclass(frozen=True)
class RopeFreqConfig:
    """Llama-3.1 "by-parts" RoPE frequency smoothing (reference Llama3.py:79-96)."""

    factor: float
    low_freq_factor: float
    high_freq_factor: float
    original_context_length: int

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


@dataclass(frozen=True)
class ModelConfig:
    family: str                      # "gpt2" | "llama"
    name: str                        # CLI model name: GPT2 / llama2 / llama3 / llama3_1 / llama3_2
    size: str                        # "124M", "8B", ...
    vocab_size: int
    context_length: int
    emb_dim: int
    n_heads: int
    n_layers: int
    hidden_dim: int                  # FFN hidden (GPT-2: 4*emb_dim)
    n_kv_groups: int                 # == n_heads for MHA
    drop_rate: float = 0.0
    qkv_bias: bool = False
    rope_base: float = 10_000.0
    rope_freq: Optional[RopeFreqConfig] = None
    eos_id: int = 50256
    eos_text: str = "<|endoftext|>"
    dtype: torch.dtype = torch.float32
    norm_eps: float = 1e-5

    # ------------------------------------------------------------------
    @property
    def head_dim(self) -> int:
        return self.emb_dim // self.n_heads

    @property
    def is_llama(self) -> bool:
        return self.family == "llama"

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)

    def to_dict(self) -> dict:
        """Dict view with the reference's key names (config dicts in Models/*/config.py)."""
        d = {
            "vocab_size": self.vocab_size,
            "context_length": self.context_length,
            "emb_dim": self.emb_dim,
            "n_heads": self.n_heads,
            "n_layers": self.n_layers,
            "hidden_dim": self.hidden_dim,
            "n_kv_groups": self.n_kv_groups,
            "drop_rate": self.drop_rate,
            "qkv_bias": self.qkv_bias,
            "rope_base": self.rope_base,
            "rope_freq": self.rope_freq.to_dict() if self.rope_freq else None,
            "eos_id": self.eos_id,
            "eos_text": self.eos_text,
            "dtype": self.dtype,
        }
        return d

    # dict-style access so code written against the reference's config dicts works
    def __getitem__(self, key):
        return self.to_dict()[key]

    def get(self, key, default=None):
        return self.to_dict().get(key, default)

    def __contains__(self, key):
        return key in self.to_dict()

    # ------------------------------------------------------------------
    def num_params(self, tied_head: bool = False) -> int:
        """Analytic parameter count (matches instantiating the reference)."""
        d, F, V, L = self.emb_dim, self.hidden_dim, self.vocab_size, self.n_layers
        kv = self.n_kv_groups * self.head_dim
        if self.family == "gpt2":
            blk = d * d + 2 * d * kv + d * d + d          # q,k,v,out (+out bias)
            if self.qkv_bias:
                blk += d + 2 * kv
            blk += d * F + F + F * d + d                  # mlp with biases
            blk += 4 * d                                  # 2 layernorms
            total = V * d + self.context_length * d + L * blk + 2 * d
        else:
            blk = d * d + 2 * d * kv + d * d + 3 * d * F + 2 * d
            total = V * d + L * blk + d
        if not tied_head:
            total += V * d
        return total

    def train_flops_per_token(self, seq_len: Optional[int] = None) -> float:
        """6*N_nonemb + 12*L*d*T; N_nonemb includes the LM head."""
        T = seq_len or self.context_length
        n_emb = self.vocab_size * self.emb_dim
        if self.family == "gpt2":
            n_emb += self.context_length * self.emb_dim
        n = self.num_params() - n_emb
        return 6.0 * n + 12.0 * self.n_layers * self.emb_dim * T

    def recompute_flops_per_token(self, seq_len: Optional[int] = None) -> float:
        """Extra FLOPs of full activation checkpointing: every block's forward re-run in
        backward, minus its last projection (down / c_proj), whose output backward never reads
        (models/llama.py, gpt2.py ``recompute``)."""
        T = seq_len or self.context_length
        d, F = self.emb_dim, self.hidden_dim
        kv = self.n_kv_groups * self.head_dim
        proj = d * (d + 2 * kv) + d * d + (2 * d * F if self.is_llama else d * F)
        return self.n_layers * (2.0 * proj + 4.0 * d * T)


# ---------------------------------------------------------------------------
# GPT-2 registry (reference Models/GPT2/config.py)
# ---------------------------------------------------------------------------
_GPT2_SIZES = {
    "124M": (768, 12, 12),
    "355M": (1024, 16, 24),
    "774M": (1280, 20, 36),
    "1.5B": (1600, 25, 48),
}


def _gpt2(size: str) -> ModelConfig:
    d, h, L = _GPT2_SIZES[size]
    return ModelConfig(
        family="gpt2", name="GPT2", size=size, vocab_size=50257, context_length=1024,
        emb_dim=d, n_heads=h, n_layers=L, hidden_dim=4 * d, n_kv_groups=h,
        drop_rate=0.1, qkv_bias=False, eos_id=50256, eos_text="<|endoftext|>",
    )


# ---------------------------------------------------------------------------
# Llama registry (reference Models/Llama/config.py:8-71)
# ---------------------------------------------------------------------------
def _llama(name: str, size: str) -> ModelConfig:
    if name == "llama2" and size == "7B":
        return ModelConfig(
            family="llama", name=name, size=size, vocab_size=32_000, context_length=4096,
            emb_dim=4096, n_heads=32, n_layers=32, hidden_dim=11_008, n_kv_groups=32,
            rope_base=10_000.0, rope_freq=None, eos_id=2, eos_text="</s>", dtype=torch.bfloat16,
        )
    if name == "llama3" and size == "8B":
        return ModelConfig(
            family="llama", name=name, size=size, vocab_size=128_256, context_length=8192,
            emb_dim=4096, n_heads=32, n_layers=32, hidden_dim=14_336, n_kv_groups=8,
            rope_base=500_000.0, rope_freq=None, eos_id=128_001, eos_text="<|end_of_text|>",
            dtype=torch.bfloat16,
        )
    if name == "llama3_1" and size == "8B":
        return ModelConfig(
            family="llama", name=name, size=size, vocab_size=128_256, context_length=131_072,
            emb_dim=4096, n_heads=32, n_layers=32, hidden_dim=14_336, n_kv_groups=8,
            rope_base=500_000.0,
            rope_freq=RopeFreqConfig(8.0, 1.0, 4.0, 8192),
            eos_id=128_001, eos_text="<|end_of_text|>", dtype=torch.bfloat16,
        )
    if name == "llama3_2" and size == "1B":
        return ModelConfig(
            family="llama", name=name, size=size, vocab_size=128_256, context_length=131_072,
            emb_dim=2048, n_heads=32, n_layers=16, hidden_dim=8192, n_kv_groups=8,
            rope_base=500_000.0,
            rope_freq=RopeFreqConfig(32.0, 1.0, 4.0, 8192),
            eos_id=128_001, eos_text="<|end_of_text|>", dtype=torch.bfloat16,
        )
    raise ValueError(f"A {name} model with {size} parameters does not exist. "
                     f"Supported sizes: {model_params_mapping.get(name, [])}")


def rescale_theta(theta_old: float, context_length_old: int, context_length_new: int) -> float:
    """Linear RoPE theta rescale (reference common_components.py:38-51)."""
    return theta_old * (context_length_new / context_length_old)


def get_config(model: str, num_params: str,
               context_length: Optional[int] = DEFAULT_CONTEXT_LENGTH) -> ModelConfig:
    """Return a fresh config. Llama configs are clamped to ``context_length`` with the
    reference's linear theta rescale (Llama/config.py:115-124); GPT-2 keeps 1024."""
    if model == "GPT2":
        if num_params not in _GPT2_SIZES:
            raise ValueError(f"GPT-2 config for model '{num_params}' not found. "
                             f"Available options: {list(_GPT2_SIZES)}")
        cfg = _gpt2(num_params)
        if context_length is not None and context_length != cfg.context_length:
            cfg = cfg.replace(context_length=context_length)
        return cfg
    if model.startswith("llama"):
        cfg = _llama(model, num_params)
        if context_length is not None and cfg.context_length != context_length:
            # Llama-2's attention always builds its tables with theta 10000 at the clamped
            # ctx and never reads rope_base (reference Llama2.py:34,86): no rescale there
            base = cfg.rope_base if model == "llama2" else \
                rescale_theta(cfg.rope_base, cfg.context_length, context_length)
            cfg = cfg.replace(rope_base=base, context_length=context_length)
        return cfg
    raise ValueError(f"Unsupported model '{model}'")


def get_config_gpt2(num_params: str) -> ModelConfig:
    return get_config("GPT2", num_params)


def get_config_llama(num_params: str, model_name: str) -> ModelConfig:
    return get_config(model_name, num_params)


def debug_config(cfg: ModelConfig) -> ModelConfig:
    """``--debug`` tiny model (reference build_components.py:72-80): ctx 10, d 32, F 10,
    16 heads (head_dim 2), 2 layers, no qkv bias. For Llama we keep GQA valid by using
    n_kv_groups = gcd(original groups, 16)."""
    import math
    kv = 16 if cfg.family == "gpt2" else math.gcd(cfg.n_kv_groups, 16)
    return cfg.replace(context_length=10, emb_dim=32, hidden_dim=10 if cfg.is_llama else 4 * 32,
                       n_heads=16, n_layers=2, qkv_bias=False, n_kv_groups=kv)
