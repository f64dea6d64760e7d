"""CPU fallbacks of the fused ops equal the compositions they replace (the GPU kernels are
pinned against the same compositions in test_kernels_gpu.py)."""
import torch

from building_llm_from_scratch_amd import ops
from building_llm_from_scratch_amd.ops import reference as ref


def test_swiglu_bwd_act_cpu():
    gu = torch.randn(7, 2 * 24)
    da = torch.randn(7, 24)
    d2 = da.clone()
    dgu = ops.swiglu_bwd_act(gu, d2)
    assert torch.allclose(dgu, ref.swiglu_bwd(gu, da))
    assert torch.allclose(d2, ref.swiglu_fwd(gu))


def test_bias_fused_backward_cpu():
    dy = torch.randn(33, 16)
    f = torch.randn(33, 16)
    for acc in (False, True):
        db0 = torch.randn(16)
        db = db0.clone()
        d = ops.dropout_bwd_bias(dy, 0.1, 5, 9, db, acc)
        want = ops.dropout_bwd(dy, 0.1, 5, 9)
        assert torch.equal(d, want)
        assert torch.allclose(db, want.sum(0) + (db0 if acc else 0), atol=1e-5)
        db = db0.clone()
        d = ops.gelu_bwd_bias(f, dy, db, acc)
        want = ops.gelu_bwd(f, dy)
        assert torch.equal(d, want)
        assert torch.allclose(db, want.sum(0) + (db0 if acc else 0), atol=1e-5)


def test_flash_attn_bwd_rope_cpu():
    B, T, H, G, hd = 2, 12, 4, 2, 16
    cos, sin = ops.rope_tables(hd, 32, 10000.0)
    qkv = torch.randn(B * T, (H + 2 * G) * hd)
    do = torch.randn(B * T, H * hd)
    o, lse = ops.flash_attn_fwd(qkv, B, T, H, G, hd, True)
    fused = ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, True, rope=(cos, sin))
    sep = ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, True)
    ops.rope_(sep, cos, sin, T, H, G, hd, inverse=True)
    assert torch.allclose(fused, sep, atol=1e-6)
