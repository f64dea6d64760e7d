"""Config registry and RoPE tables pinned against an independent transcription of the
reference (Models/Llama/config.py:8-71,97-126; common_components.py:38-51;
Llama3.py:74-104; Llama2.py:34-55,86).  The transcription below is written from the
reference's formulas in plain float64 numpy, NOT by calling the framework's helpers, so a
registry / table bug (e.g. rescaling Llama-2's theta) cannot hide behind a shared helper."""
import math

import numpy as np
import pytest
import torch

from building_llm_from_scratch_amd import ops
from building_llm_from_scratch_amd.config import get_config
from building_llm_from_scratch_amd.models import build_model

# reference dicts, transcribed (Models/Llama/config.py:8-71)
REF = {
    "llama2": dict(ctx=4096, theta=None, freq=None),           # no rope_base key; attention uses 10000
    "llama3": dict(ctx=8192, theta=500_000.0, freq=None),
    "llama3_1": dict(ctx=131_072, theta=500_000.0,
                     freq=dict(factor=8.0, low_freq_factor=1.0, high_freq_factor=4.0, original_context_length=8192)),
    "llama3_2": dict(ctx=131_072, theta=500_000.0,
                     freq=dict(factor=32.0, low_freq_factor=1.0, high_freq_factor=4.0, original_context_length=8192)),
}
SIZES = {"llama2": "7B", "llama3": "8B", "llama3_1": "8B", "llama3_2": "1B"}


def ref_theta(name, ctx=1024):
    r = REF[name]
    if r["theta"] is None:
        return 10_000.0
    return r["theta"] * ctx / r["ctx"]            # rescale_theta (common_components.py:50-51)


def ref_tables(head_dim, theta, ctx, freq):
    inv = 1.0 / theta ** (np.arange(0, head_dim, 2, dtype=np.float64) / head_dim)
    if freq is not None:
        low_wl = freq["original_context_length"] / freq["low_freq_factor"]
        high_wl = freq["original_context_length"] / freq["high_freq_factor"]
        out = []
        for f in inv:
            wl = 2 * math.pi / f
            if wl < high_wl:
                out.append(f)
            elif wl > low_wl:
                out.append(f / freq["factor"])
            else:
                s = (freq["original_context_length"] / wl - freq["low_freq_factor"]) / (
                    freq["high_freq_factor"] - freq["low_freq_factor"])
                out.append((1 - s) * f / freq["factor"] + s * f)
        inv = np.array(out)
    ang = np.arange(ctx, dtype=np.float64)[:, None] * inv[None, :]
    return np.cos(ang), np.sin(ang)


def test_registry_theta_values():
    assert get_config("llama3", "8B").rope_base == 62_500.0
    assert get_config("llama3_1", "8B").rope_base == 3_906.25
    assert get_config("llama3_2", "1B").rope_base == 3_906.25
    assert get_config("llama2", "7B").rope_base == 10_000.0
    for name, size in SIZES.items():
        cfg = get_config(name, size)
        assert cfg.context_length == 1024
        assert cfg.rope_base == ref_theta(name), name


@pytest.mark.parametrize("name", list(SIZES))
@pytest.mark.parametrize("ctx", [1024, 2048])
def test_rope_tables_match_reference(name, ctx):
    cfg = get_config(name, SIZES[name], context_length=ctx)
    c, s = ops.rope_tables(cfg.head_dim, cfg.context_length, cfg.rope_base, cfg.rope_freq)
    rc, rs = ref_tables(cfg.head_dim, ref_theta(name, ctx), ctx, REF[name]["freq"])
    assert c.shape == (ctx, cfg.head_dim // 2)
    np.testing.assert_allclose(c.numpy(), rc, atol=2e-6)
    np.testing.assert_allclose(s.numpy(), rs, atol=2e-6)


def test_llama2_parity_buffers_use_theta_10000_fp32():
    cfg = get_config("llama2", "7B").replace(n_layers=1, emb_dim=256, n_heads=2, n_kv_groups=2, hidden_dim=64,
                                            vocab_size=64)
    m = build_model(cfg)
    sd = m.state_dict()
    cos, sin = sd["trf_blocks.0.att.cos"], sd["trf_blocks.0.att.sin"]
    assert cos.dtype == torch.float32 and cos.shape == (1024, 128)
    rc, rs = ref_tables(128, 10_000.0, 1024, None)
    np.testing.assert_allclose(cos.numpy(), np.concatenate([rc, rc], 1), atol=2e-6)
    np.testing.assert_allclose(sin.numpy(), np.concatenate([rs, rs], 1), atol=2e-6)


def test_llama3_parity_buffers_bf16():
    cfg = get_config("llama3_2", "1B").replace(n_layers=1, emb_dim=128, n_heads=2, n_kv_groups=1, hidden_dim=64,
                                              vocab_size=64)
    sd = build_model(cfg).state_dict()
    cos = sd["trf_blocks.0.att.cos"]
    assert cos.dtype == torch.bfloat16 and cos.shape == (1024, 64)
    rc, _ = ref_tables(64, 3_906.25, 1024, REF["llama3_2"]["freq"])
    np.testing.assert_allclose(cos.float().numpy(), np.concatenate([rc, rc], 1), atol=8e-3)
