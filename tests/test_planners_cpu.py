"""CPU checks of the host-side planners that route GPU work (pure Python, no GPU needed)."""
from building_llm_from_scratch_amd import ops


def test_wgrad_plan_gpt2_shapes_match_measured_best():
    """The dW split-K planner's picks at the GPT2-774M shapes (65,536 tokens) are the splits the
    sweep measured fastest or within 3.5 % of it (profiles/r5/wgrad_splits/gpt2_774m_sweep.jsonl:
    qkv S=3 544 us, o S=8 202 us (S=10: 195), fc1 / fc2 S=5)."""
    assert ops.wgrad_plan(3840, 1280, 65536) == ("split", 3)
    assert ops.wgrad_plan(1280, 1280, 65536) == ("split", 8)
    assert ops.wgrad_plan(5120, 1280, 65536) == ("split", 5)
    assert ops.wgrad_plan(1280, 5120, 65536) == ("split", 5)


def test_wgrad_plan_headline_tails():
    """Llama-3-8B at B=40: a ragged last wave runs as whole-K waves + a 2-way split tail."""
    assert ops.wgrad_plan(4096, 14336, 40960) == ("tail", 768, 2)
    assert ops.wgrad_plan(6144, 4096, 40960) == ("tail", 256, 2)
    assert ops.wgrad_plan(28672, 4096, 40960) == ("split", 1)


def test_lora_head_fused_conditions(monkeypatch):
    """The one-pass LoRA head backward applies to rank 16 and a vocabulary that is a multiple of
    64 (Llama-3's 128,256, Llama-2's 32,000, GPT-2's padded 50,432), and is switched off by
    BLLM_LORA_HEAD_FUSED=0."""
    for V in (128256, 32000, 50432, 1088):
        assert ops.lora_head_bwd_ok(V, 16)
    assert not ops.lora_head_bwd_ok(50257, 16)
    assert not ops.lora_head_bwd_ok(128256, 32)
    monkeypatch.setattr(ops, "LORA_HEAD_FUSED", False)
    assert not ops.lora_head_bwd_ok(128256, 16)
