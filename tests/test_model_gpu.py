"""Whole-model parity on the GPU: the HIP kernel path (bf16) vs the CPU reference path (fp32)
with identical weights — loss and every parameter gradient."""
import pytest
import torch

from building_llm_from_scratch_amd import ops
from building_llm_from_scratch_amd.config import get_config
from building_llm_from_scratch_amd.models import build_model, replace_linear_with_lora
from building_llm_from_scratch_amd.train.optim import FusedAdamW

pytestmark = pytest.mark.gpu


def _cfgs():
    llama = get_config("llama3_1", "8B").replace(context_length=256, emb_dim=512, n_heads=8, n_kv_groups=2,
                                                 hidden_dim=768, n_layers=2, vocab_size=1000)
    llama128 = get_config("llama3", "8B").replace(context_length=256, emb_dim=512, n_heads=4, n_kv_groups=1,
                                                  hidden_dim=512, n_layers=2, vocab_size=1000)
    gpt = get_config("GPT2", "124M").replace(context_length=256, emb_dim=256, n_heads=4, n_kv_groups=4,
                                             hidden_dim=1024, n_layers=2, vocab_size=1000, drop_rate=0.0)
    return {"llama_hd64": llama, "llama_hd128": llama128, "gpt2": gpt}


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("name", ["llama_hd64", "llama_hd128", "gpt2"])
@pytest.mark.parametrize("ckpt", ["none", "selective", "full"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_gpu_model_matches_cpu_reference(name, ckpt, dt):
    """bf16 kernels within bf16 tolerance; fp32 (the reference's default precision: fp32 flash
    attention on the f32 MFMA, fp32 GEMMs) within 1e-3."""
    ops.load_ext(required=True)
    cfg = _cfgs()[name]
    torch.manual_seed(0)
    ref = build_model(cfg.replace(dtype=torch.float32), use_actv_ckpt=ckpt)
    gpu = build_model(cfg.replace(dtype=dt), use_actv_ckpt=ckpt, device="cuda")
    gpu.load_state_dict(ref.state_dict())
    idx = torch.randint(0, cfg.vocab_size, (2, 257))
    lr = ref(idx[:, :-1], idx[:, 1:])
    lr.backward()
    lg = gpu(idx[:, :-1].cuda(), idx[:, 1:].cuda())
    lg.backward()
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    gtol = 5e-2 if dt == torch.bfloat16 else 1e-3
    assert abs(lg.item() - lr.item()) < tol * abs(lr.item()), (lg.item(), lr.item())
    named = dict(ref.named_parameters())
    for k, p in gpu.named_parameters():
        e = _rel(p.grad, named[k].grad)
        assert e < gtol, (k, e)


def test_gpu_lora_and_training_decreases_loss():
    ops.load_ext(required=True)
    cfg = _cfgs()["llama_hd64"]
    torch.manual_seed(0)
    m = build_model(cfg, device="cuda")
    for p in m.parameters():
        p.requires_grad = False
    replace_linear_with_lora(m, rank=16, alpha=32)
    m.flatten()
    opt = FusedAdamW(m, lr=2e-3, weight_decay=0.1)
    idx = torch.randint(0, cfg.vocab_size, (4, 129), device="cuda")
    losses = []
    for _ in range(30):
        loss = m(idx[:, :-1], idx[:, 1:])
        loss.backward()
        opt.clip_grad_norm_(1.0)
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] - 0.5, losses


def test_overlapped_optimizer_matches_serial():
    """The side-stream (overlapped) AdamW must produce exactly the serial result."""
    ops.load_ext(required=True)
    cfg = _cfgs()["llama_hd64"]
    idx = torch.randint(0, cfg.vocab_size, (3, 4, 129), device="cuda")
    finals = []
    for overlap in (False, True):
        torch.manual_seed(0)
        m = build_model(cfg, device="cuda")
        m.flatten()
        opt = FusedAdamW(m, lr=1e-3, weight_decay=0.1, overlap=overlap)
        assert opt.overlap == overlap
        for i in range(3):
            loss = m(idx[i, :, :-1], idx[i, :, 1:])
            loss.backward()
            opt.clip_grad_norm_(1.0)
            opt.step()
        finals.append({k: v.float().cpu() for k, v in m.state_dict().items()})
    for k in finals[0]:
        assert torch.equal(finals[0][k], finals[1][k]), k


@pytest.mark.parametrize("name", ["llama_hd64", "llama_hd128", "gpt2"])
def test_kv_cache_decode_matches_full_forward(name):
    """Prefill (flash kernel) + token-by-token decode (HIP decode kernel over the KV cache)
    must reproduce the full-sequence forward's logits at every decoded position."""
    ops.load_ext(required=True)
    cfg = _cfgs()[name]
    torch.manual_seed(0)
    m = build_model(cfg, device="cuda")
    m.flatten()
    m.eval()
    idx = torch.randint(0, cfg.vocab_size, (2, 40), device="cuda")
    with torch.no_grad():
        full = m(idx).float()
        cache = m.new_kv_cache(2, cfg.context_length)
        lg = m.forward_cached(idx[:, :24], cache, 0)
        assert _rel(lg, full[:, 23]) < 2e-2
        for p in range(24, 40):
            lg = m.forward_cached(idx[:, p:p + 1], cache, p)
            assert _rel(lg, full[:, p]) < 2e-2, p


@pytest.mark.parametrize("name", ["llama_hd64", "llama_hd128", "gpt2"])
def test_device_position_decode_matches_full_forward(name):
    """forward_cached_dev (position in device memory, fused K/V append + decode attention,
    device-side RoPE) reproduces the full forward's logits, eagerly and replayed from a HIP graph."""
    from building_llm_from_scratch_amd.train.generate import DecodeGraph
    ops.load_ext(required=True)
    cfg = _cfgs()[name].replace(dtype=torch.bfloat16)
    torch.manual_seed(0)
    m = build_model(cfg, device="cuda")
    m.flatten()
    m.eval()
    idx = torch.randint(0, cfg.vocab_size, (2, 40), device="cuda")
    with torch.no_grad():
        full = m(idx).float()
        for graph in (False, True):
            cache = m.new_kv_cache(2, cfg.context_length)
            m.forward_cached(idx[:, :24], cache, 0)
            dec = DecodeGraph(m, cache, 2, idx.device) if graph else None
            pos_t = torch.zeros(1, dtype=torch.int32, device="cuda")
            for p in range(24, 40):
                if graph:
                    lg = dec.step(idx[:, p:p + 1], p)
                else:
                    pos_t.fill_(p)
                    lg = m.forward_cached_dev(idx[:, p:p + 1], cache, pos_t)
                assert _rel(lg, full[:, p]) < 2e-2, (graph, p)


@pytest.mark.parametrize("name", ["llama_hd128", "gpt2"])
def test_generate_graph_matches_eager(name, monkeypatch):
    """The whole sample (top-k 5, temperature 1, seeded) is token-identical with and without the
    HIP-graph decode step."""
    from building_llm_from_scratch_amd.train import generate as G
    ops.load_ext(required=True)
    cfg = _cfgs()[name].replace(dtype=torch.bfloat16)
    torch.manual_seed(0)
    m = build_model(cfg, device="cuda")
    m.flatten()
    idx = torch.randint(0, cfg.vocab_size, (1, 6), device="cuda")
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("BLLM_DECODE_GRAPH", flag)
        g = torch.Generator(device="cuda").manual_seed(5)
        outs.append(G.generate_cached(m, idx, 60, cfg.context_length, temperature=1.0, top_k=5, generator=g))
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("name", ["llama_hd128", "gpt2"])
def test_training_is_bitwise_deterministic(name):
    """Two identical runs (same seed, same data) must give bit-identical parameters: every
    HIP kernel reduces in a fixed order (no float atomics), dropout masks are counter-based."""
    ops.load_ext(required=True)
    cfg = _cfgs()[name]
    if name == "gpt2":
        cfg = cfg.replace(drop_rate=0.1)
    idx = torch.randint(0, cfg.vocab_size, (3, 4, 129), device="cuda")
    finals = []
    for _ in range(2):
        torch.manual_seed(0)
        m = build_model(cfg, device="cuda")
        m.flatten()
        opt = FusedAdamW(m, lr=1e-3, weight_decay=0.1)
        for i in range(3):
            loss = m(idx[i, :, :-1], idx[i, :, 1:])
            loss.backward()
            opt.clip_grad_norm_(1.0)
            opt.step()
        finals.append({k: v.float().cpu() for k, v in m.state_dict().items()})
    for k in finals[0]:
        assert torch.equal(finals[0][k], finals[1][k]), k


@pytest.mark.parametrize("name", ["gpt2", "llama_hd64"])
def test_fp16_fused_head_under_loss_scaling(name, monkeypatch):
    """fp16 + dynamic loss scaling (the Trainer's fp16 path, loss scale 2^16): the fused chunked
    head + CE takes the logit gradient inside its forward at the announced loss scale, so softmax
    tails p / nvalid below fp16's subnormal range are not flushed before scaling.  Its gradients
    must match the unfused head (full fp16 logits, CE backward at dloss = scale) and the fp32
    CPU oracle."""
    from building_llm_from_scratch_amd.models import llama as L
    ops.load_ext(required=True)
    cfg = _cfgs()[name].replace(vocab_size=32000)
    S = 65536.0
    torch.manual_seed(0)
    ref = build_model(cfg.replace(dtype=torch.float32))
    idx = torch.randint(0, cfg.vocab_size, (2, 257))
    lr = ref(idx[:, :-1], idx[:, 1:])
    lr.backward()
    named = dict(ref.named_parameters())
    head = "output_head.weight" if name == "gpt2" else "out_head.weight"
    grads = {}
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(L.HeadComputeMixin, "_fused_ok", lambda self, h: False)
        m = build_model(cfg.replace(dtype=torch.float16), device="cuda")
        m.load_state_dict(ref.state_dict())
        m.rctx.loss_scale = S
        loss = m(idx[:, :-1].cuda(), idx[:, 1:].cuda())
        (loss * S).backward()
        grads[fused] = {k: p.grad.float() / S for k, p in m.named_parameters()}
        assert abs(loss.item() - lr.item()) < 1e-2 * lr.item()
    for k in (head, "tok_emb.weight"):
        e_fused = _rel(grads[True][k], named[k].grad)
        e_unfused = _rel(grads[False][k], named[k].grad)
        assert e_fused < 1e-2, (k, e_fused)
        assert e_fused <= 1.5 * e_unfused + 1e-3, (k, e_fused, e_unfused)


@pytest.mark.parametrize("ckpt", ["none", "selective", "full"])
def test_fused_swiglu_gemm_in_model(ckpt, monkeypatch):
    """BLLM_FUSED_SWIGLU: the gate/up GEMM with the SwiGLU epilogue gives the same loss and
    gradients as the separate GEMM + swiglu_fwd kernel (bitwise-equal act; the GEMM itself is a
    different kernel from hipBLASLt, so gradients agree to rounding)."""
    from building_llm_from_scratch_amd.models import linear
    ops.load_ext(required=True)
    cfg = _cfgs()["llama_hd64"].replace(dtype=torch.bfloat16)
    idx = torch.randint(0, cfg.vocab_size, (2, 257), device="cuda")
    res = {}
    calls = []
    orig = ops.gemm_nt_swiglu
    monkeypatch.setattr(ops, "gemm_nt_swiglu", lambda *a: (calls.append(1), orig(*a))[1])
    for fused in (False, True):
        monkeypatch.setattr(linear, "FUSED_SWIGLU", fused)
        torch.manual_seed(0)
        m = build_model(cfg, use_actv_ckpt=ckpt, device="cuda")
        m.flatten()
        loss = m(idx[:, :-1], idx[:, 1:])
        loss.backward()
        res[fused] = (loss.item(), {k: p.grad.float().clone() for k, p in m.named_parameters()})
    assert calls, "fused gate/up + SwiGLU kernel not used"
    (l0, g0), (l1, g1) = res[False], res[True]
    assert abs(l0 - l1) < 1e-2 * abs(l0)
    for k in g0:
        assert _rel(g1[k], g0[k]) < 2e-2, (k, _rel(g1[k], g0[k]))


@pytest.mark.parametrize("ckpt", ["none", "selective", "full"])
def test_fused_rope_and_swiglu_epilogues_in_model(ckpt, monkeypatch):
    """BLLM_FUSED_ROPE + BLLM_FUSED_SWIGLU (head dim 128): the QKV GEMM with RoPE in its epilogue
    and the gate/up GEMM with SwiGLU in its epilogue (persistent 4-wave kernel) give the loss and
    gradients of the separate GEMM + rope_ / swiglu_fwd passes to rounding, in every checkpoint
    mode (the recompute re-runs the fused forward)."""
    from building_llm_from_scratch_amd.models import linear
    ops.load_ext(required=True)
    cfg = _cfgs()["llama_hd128"].replace(dtype=torch.bfloat16)
    idx = torch.randint(0, cfg.vocab_size, (2, 257), device="cuda")
    res, calls = {}, []
    orig = ops.gemm_nt_rope
    monkeypatch.setattr(ops, "gemm_nt_rope", lambda *a: (calls.append(1), orig(*a))[1])
    for fused in (False, True):
        monkeypatch.setattr(linear, "FUSED_ROPE", fused)
        monkeypatch.setattr(linear, "FUSED_SWIGLU", fused)
        torch.manual_seed(0)
        m = build_model(cfg, use_actv_ckpt=ckpt, device="cuda")
        m.flatten()
        loss = m(idx[:, :-1], idx[:, 1:])
        loss.backward()
        res[fused] = (loss.item(), {k: p.grad.float().clone() for k, p in m.named_parameters()})
    assert calls, "fused QKV + RoPE kernel not used"
    (l0, g0), (l1, g1) = res[False], res[True]
    assert abs(l0 - l1) < 1e-2 * abs(l0)
    for k in g0:
        assert _rel(g1[k], g0[k]) < 2e-2, (k, _rel(g1[k], g0[k]))


@pytest.mark.parametrize("ckpt", ["none", "selective", "full"])
def test_fused_bias_gelu_epilogue_in_model(ckpt, monkeypatch):
    """BLLM_FUSED_GELU: GPT-2's c_fc with bias + GELU in the GEMM epilogue gives the loss and
    gradients of hipBLASLt's bias GEMM + the separate gelu_fwd pass to rounding (no dropout)."""
    from building_llm_from_scratch_amd.models import linear
    ops.load_ext(required=True)
    cfg = _cfgs()["gpt2"].replace(dtype=torch.bfloat16)
    idx = torch.randint(0, cfg.vocab_size, (2, 257), device="cuda")
    res, calls = {}, []
    orig = ops.gemm_nt_bias_gelu
    monkeypatch.setattr(ops, "gemm_nt_bias_gelu", lambda *a: (calls.append(1), orig(*a))[1])
    for fused in (False, True):
        monkeypatch.setattr(linear, "FUSED_GELU", fused)
        torch.manual_seed(0)
        m = build_model(cfg, use_actv_ckpt=ckpt, device="cuda")
        m.flatten()
        loss = m(idx[:, :-1], idx[:, 1:])
        loss.backward()
        res[fused] = (loss.item(), {k: p.grad.float().clone() for k, p in m.named_parameters()})
    assert calls, "fused c_fc + bias + GELU kernel not used"
    (l0, g0), (l1, g1) = res[False], res[True]
    assert abs(l0 - l1) < 1e-2 * abs(l0)
    for k in g0:
        assert _rel(g1[k], g0[k]) < 2e-2, (k, _rel(g1[k], g0[k]))


def test_gemm_nt_kernel_in_model(monkeypatch):
    """BLLM_GEMM_NT=1: the forward-layout GEMMs (projections, the dX GEMMs on the transposed
    weight copy, the fused head's logits and dh) on csrc/gemm_nt.hip give hipBLASLt's loss and
    gradients to rounding (B*T = 512 tokens: every GEMM takes the kernel)."""
    from building_llm_from_scratch_amd.models import linear
    ops.load_ext(required=True)
    cfg = _cfgs()["llama_hd64"].replace(dtype=torch.bfloat16, vocab_size=1024)
    idx = torch.randint(0, cfg.vocab_size, (2, 257), device="cuda")
    monkeypatch.setattr(linear, "DGRAD_WT_MIN_TOKENS", 256)
    calls = []
    orig = ops.gemm_nt_
    monkeypatch.setattr(ops, "gemm_nt_", lambda *a: (calls.append(1), orig(*a))[1])
    res = {}
    for on in (False, True):
        monkeypatch.setattr(linear, "GEMM_NT", on)
        torch.manual_seed(0)
        m = build_model(cfg, use_actv_ckpt="selective", device="cuda")
        m.flatten()
        loss = m(idx[:, :-1], idx[:, 1:])
        loss.backward()
        res[on] = (loss.item(), {k: p.grad.float().clone() for k, p in m.named_parameters()})
    assert len(calls) >= 10, len(calls)
    (l0, g0), (l1, g1) = res[False], res[True]
    assert abs(l0 - l1) < 1e-2 * abs(l0)
    for k in g0:
        assert _rel(g1[k], g0[k]) < 2e-2, (k, _rel(g1[k], g0[k]))


@pytest.mark.parametrize("ckpt", ["none", "selective", "full"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_fused_layernorm_dropout_in_model(ckpt, dt, monkeypatch):
    """GPT-2 with dropout: the attention residual's dropout-add + norm2 as one row pass gives the
    separate kernels' loss and gradients bitwise."""
    from building_llm_from_scratch_amd.models import gpt2
    ops.load_ext(required=True)
    cfg = _cfgs()["gpt2"].replace(dtype=dt, drop_rate=0.1)
    idx = torch.randint(0, cfg.vocab_size, (2, 257), device="cuda")
    res, calls = {}, []
    orig = ops.dropout_add_layernorm
    monkeypatch.setattr(ops, "dropout_add_layernorm", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    for fused in (False, True):
        monkeypatch.setattr(gpt2, "FUSED_LN_DROPOUT", fused)
        torch.manual_seed(0)
        m = build_model(cfg, use_actv_ckpt=ckpt, device="cuda")
        m.flatten()
        loss = m(idx[:, :-1], idx[:, 1:])
        loss.backward()
        res[fused] = (loss.item(), {k: p.grad.float().clone() for k, p in m.named_parameters()})
    assert calls, "fused dropout-add + LayerNorm not used"
    (l0, g0), (l1, g1) = res[False], res[True]
    assert l0 == l1
    for k in g0:
        assert torch.equal(g1[k], g0[k]), (k, _rel(g1[k], g0[k]))


def test_lora_swiglu_wgrad_fusion_in_model(monkeypatch):
    """A LoRA Llama step with the MLP's gate/up dB and down dA summed inside the SwiGLU backward
    (ops.swiglu_bwd_lowrank_wgrad) gives the separate lora_wgrad passes' loss and gradients."""
    from building_llm_from_scratch_amd.models import llama
    ops.load_ext(required=True)
    cfg = get_config("llama3_2", "1B").replace(context_length=128, emb_dim=256, n_heads=4, n_kv_groups=2,
                                               hidden_dim=512, n_layers=2, vocab_size=512, dtype=torch.bfloat16)
    res, calls = {}, []
    orig = ops.swiglu_bwd_lowrank_wgrad
    monkeypatch.setattr(ops, "swiglu_bwd_lowrank_wgrad", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    for fused in (False, True):
        monkeypatch.setattr(llama, "LORA_SWIGLU_WGRAD", fused)
        torch.manual_seed(0)
        m = build_model(cfg, device="cuda")
        for p in m.parameters():
            p.requires_grad = False
        replace_linear_with_lora(m, rank=16, alpha=32)
        for mod in m.modules():
            if hasattr(mod, "B") and isinstance(mod.B, torch.nn.Parameter):
                torch.nn.init.normal_(mod.B, std=0.05)
        m.flatten(device="cuda")
        idx = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=torch.Generator("cuda").manual_seed(1))
        for step in range(2):   # the second backward accumulates into the first's gradients
            loss = m(idx, idx)
            loss.backward()
        res[fused] = (loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters() if p.requires_grad})
    assert len(calls) == 4, calls     # 2 blocks x 2 steps
    (l0, g0), (l1, g1) = res[False], res[True]
    assert l0 == l1
    for k in g0:
        assert _rel(g1[k], g0[k]) < 1e-2, (k, _rel(g1[k], g0[k]))


def test_lora_head_fusion_in_model(monkeypatch):
    """A LoRA Llama step with the head's u = dl B^T and dB = (s t)^T dl from one pass over each
    logits-gradient chunk (ops.lora_head_bwd_) gives the hipBLASLt + lora_wgrad path's loss and
    gradients, and two runs of the fused path are bitwise equal (fixed-order partial sums)."""
    ops.load_ext(required=True)
    cfg = get_config("llama3_2", "1B").replace(context_length=128, emb_dim=256, n_heads=4, n_kv_groups=2,
                                               hidden_dim=512, n_layers=2, vocab_size=1088, dtype=torch.bfloat16)
    res, calls = {}, []
    orig = ops.lora_head_bwd_
    monkeypatch.setattr(ops, "lora_head_bwd_", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    for run, fused in ((0, False), (1, True), (2, True)):
        monkeypatch.setattr(ops, "LORA_HEAD_FUSED", fused)
        torch.manual_seed(0)
        m = build_model(cfg, device="cuda")
        for p in m.parameters():
            p.requires_grad = False
        replace_linear_with_lora(m, rank=16, alpha=32)
        for mod in m.modules():
            if hasattr(mod, "B") and isinstance(mod.B, torch.nn.Parameter):
                torch.nn.init.normal_(mod.B, std=0.05)
        m.flatten(device="cuda")
        idx = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=torch.Generator("cuda").manual_seed(1))
        for step in range(2):   # the second backward accumulates into the first's gradients
            loss = m(idx, idx)
            loss.backward()
        res[run] = (loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters() if p.requires_grad})
    assert len(calls) >= 4, calls     # fused runs: >= 1 chunk x 2 steps each
    (l0, g0), (l1, g1), (l2, g2) = res[0], res[1], res[2]
    assert l0 == l1 == l2
    for k in g0:
        assert _rel(g1[k], g0[k]) < 1e-2, (k, _rel(g1[k], g0[k]))
        assert torch.equal(g1[k], g2[k]), k
