"""Hand-written unit forward/backward vs an eager-autograd oracle (CPU, fp32)."""
import pytest
import torch

from building_llm_from_scratch_amd import ops
from building_llm_from_scratch_amd.config import get_config
from building_llm_from_scratch_amd.models import build_model, replace_linear_with_lora
from eager_reference import gpt2_loss, llama_loss


def _small_llama(name="llama3_2", **kw):
    cfg = get_config(name, {"llama2": "7B", "llama3": "8B", "llama3_1": "8B", "llama3_2": "1B"}[name])
    return cfg.replace(context_length=16, emb_dim=64, n_heads=4, n_kv_groups=2 if name != "llama2" else 4,
                       hidden_dim=96, n_layers=2, vocab_size=97, dtype=torch.float32, **kw)


def _small_gpt2(**kw):
    cfg = get_config("GPT2", "124M")
    return cfg.replace(context_length=16, emb_dim=64, n_heads=4, n_kv_groups=4, hidden_dim=256,
                       n_layers=2, vocab_size=97, dtype=torch.float32, drop_rate=0.0, **kw)


def _compare(model, loss_fn, idx, tgt, atol=2e-5):
    loss = model(idx, tgt)
    loss.backward()
    ref_loss, p = loss_fn(model.state_dict())
    ref_loss.backward()
    assert torch.allclose(loss, ref_loss, atol=atol, rtol=1e-5), (loss, ref_loss)
    named = dict(model.named_parameters())
    checked = 0
    for k, rp in p.items():
        mp = named[k]
        if not mp.requires_grad:
            continue
        assert mp.grad is not None, k
        assert torch.allclose(mp.grad.float(), rp.grad, atol=atol, rtol=1e-4), \
            (k, (mp.grad.float() - rp.grad).abs().max())
        checked += 1
    assert checked > 0


@pytest.mark.parametrize("name", ["llama3_2", "llama3_1", "llama2"])
@pytest.mark.parametrize("ckpt", ["none", "selective", "full"])
def test_llama_grads(name, ckpt):
    torch.manual_seed(0)
    cfg = _small_llama(name)
    m = build_model(cfg, use_actv_ckpt=ckpt)
    idx = torch.randint(0, cfg.vocab_size, (2, 16))
    tgt = torch.randint(0, cfg.vocab_size, (2, 16))
    tgt[0, :3] = -100
    cos, sin = ops.rope_tables(cfg.head_dim, cfg.context_length, cfg.rope_base, cfg.rope_freq)
    _compare(m, lambda sd: llama_loss(sd, cfg, idx, tgt, cos, sin), idx, tgt)


@pytest.mark.parametrize("qkv_bias", [False, True])
@pytest.mark.parametrize("ckpt", ["none", "full"])
def test_gpt2_grads(qkv_bias, ckpt):
    torch.manual_seed(0)
    cfg = _small_gpt2(qkv_bias=qkv_bias)
    m = build_model(cfg, use_actv_ckpt=ckpt)
    idx = torch.randint(0, cfg.vocab_size, (2, 16))
    tgt = torch.randint(0, cfg.vocab_size, (2, 16))
    _compare(m, lambda sd: gpt2_loss(sd, cfg, idx, tgt), idx, tgt)


@pytest.mark.parametrize("ckpt", ["none", "full"])
@pytest.mark.parametrize("family", ["llama", "gpt2"])
def test_lora_grads(family, ckpt):
    """``full`` also covers the recompute's skipped last projection: its LoRA intermediate is
    rebuilt without the base GEMM (FusedLinear.lora_state)."""
    torch.manual_seed(0)
    cfg = _small_llama() if family == "llama" else _small_gpt2()
    m = build_model(cfg, use_actv_ckpt=ckpt)
    for p in m.parameters():
        p.requires_grad = False
    replace_linear_with_lora(m, rank=4, alpha=8)
    # make B non-zero so dA is non-trivial
    for mod in m.modules():
        if hasattr(mod, "B") and isinstance(mod.B, torch.nn.Parameter):
            torch.nn.init.normal_(mod.B, std=0.05)
    m.flatten()
    idx = torch.randint(0, cfg.vocab_size, (2, 16))
    tgt = torch.randint(0, cfg.vocab_size, (2, 16))
    if family == "llama":
        cos, sin = ops.rope_tables(cfg.head_dim, cfg.context_length, cfg.rope_base, cfg.rope_freq)
        fn = lambda sd: llama_loss(sd, cfg, idx, tgt, cos, sin, lora=2.0)  # noqa: E731
    else:
        fn = lambda sd: gpt2_loss(sd, cfg, idx, tgt, lora=2.0)  # noqa: E731
    _compare(m, fn, idx, tgt)
    trainable = [n for n, p in m.named_parameters() if p.requires_grad]
    assert trainable and all(".lora." in n for n in trainable)
    assert any(n.startswith("out_head.lora") or n.startswith("output_head.lora") for n in trainable)


def test_logits_path_matches_loss_path():
    torch.manual_seed(0)
    cfg = _small_llama()
    m = build_model(cfg)
    idx = torch.randint(0, cfg.vocab_size, (2, 16))
    logits = m(idx)
    loss_a = torch.nn.functional.cross_entropy(logits.flatten(0, 1), idx.flatten())
    loss_b = m(idx, idx)
    assert torch.allclose(loss_a, loss_b, atol=1e-5)
    with torch.no_grad():
        last = m(idx, last_only=True)
    assert torch.allclose(last[:, 0], logits[:, -1].detach(), atol=1e-5)


@pytest.mark.parametrize("ckpt", ["none", "full"])
@pytest.mark.parametrize("family", ["llama", "gpt2"])
def test_grouped_lora_path_grads(family, monkeypatch, ckpt):
    """The grouped LoRA plumbing (pack / down / up / wgrad, as the HIP kernels run it) driven
    through the CPU oracles gives the eager-autograd gradients."""
    from building_llm_from_scratch_amd.models import linear
    monkeypatch.setattr(linear, "FORCE_GROUPED_LORA", True)
    test_lora_grads(family, ckpt)


@pytest.mark.parametrize("ckpt", ["none", "full"])
def test_kaug_grouped_lora_grads(ckpt, monkeypatch):
    """K-augmented grouped LoRA: y = [x | s t] . [W | Bd^T]^T with x written straight into the
    augmented buffer by its producer (RMSNorm for QKV and gate/up, SwiGLU for down) and the dX
    GEMM's extra columns as dy B^T, vs the eager oracle.  The out-projection (input from
    attention) stays on the grouped path; a checkpoint recompute of the down projection too."""
    from building_llm_from_scratch_amd.models import linear
    monkeypatch.setattr(linear, "FORCE_GROUPED_LORA", True)
    calls = []
    orig = linear.FusedLinear._kaug_lora_backward
    monkeypatch.setattr(linear.FusedLinear, "_kaug_lora_backward",
                        lambda self, *a, **k: (calls.append(1), orig(self, *a, **k))[1])
    torch.manual_seed(0)
    cfg = _small_llama().replace(hidden_dim=128)                 # gate/up out 256 = 4 x 64
    m = build_model(cfg, use_actv_ckpt=ckpt)
    for p in m.parameters():
        p.requires_grad = False
    replace_linear_with_lora(m, rank=16, alpha=8)
    for mod in m.modules():
        if hasattr(mod, "B") and isinstance(mod.B, torch.nn.Parameter):
            torch.nn.init.normal_(mod.B, std=0.05)
    m.flatten()
    idx = torch.randint(0, cfg.vocab_size, (2, 16))
    tgt = torch.randint(0, cfg.vocab_size, (2, 16))
    cos, sin = ops.rope_tables(cfg.head_dim, cfg.context_length, cfg.rope_base, cfg.rope_freq)
    _compare(m, lambda sd: llama_loss(sd, cfg, idx, tgt, cos, sin, lora=0.5), idx, tgt)
    n_full = sum(m.rctx.block_mode(i) == "full" for i in range(cfg.n_layers))
    assert len(calls) == 3 * cfg.n_layers - n_full, len(calls)      # recomputed blocks: down grouped


@pytest.mark.parametrize("family", ["llama", "gpt2"])
def test_fused_chunked_lora_head(family, monkeypatch):
    """LoRA head (frozen base) on the chunked head + CE with the rank-r path folded into the
    head GEMMs ([h | s t] . [W | B^T]^T): several chunks, ignore_index targets, non-unit dloss,
    vs the eager oracle."""
    from building_llm_from_scratch_amd.models import llama
    monkeypatch.setattr(llama, "MIN_CHUNK_ROWS", 8)
    monkeypatch.setattr(llama, "LOGIT_CHUNK_BYTES", 8 * 97 * 4)
    torch.manual_seed(0)
    cfg = _small_llama() if family == "llama" else _small_gpt2()
    m = build_model(cfg)
    for p in m.parameters():
        p.requires_grad = False
    replace_linear_with_lora(m, rank=4, alpha=8)
    for mod in m.modules():
        if hasattr(mod, "B") and isinstance(mod.B, torch.nn.Parameter):
            torch.nn.init.normal_(mod.B, std=0.05)
    m.flatten()
    head = m.computes[-1]
    assert head._fused_lora_ok(torch.empty(1, cfg.emb_dim))
    idx = torch.randint(0, cfg.vocab_size, (3, 13))
    tgt = torch.randint(0, cfg.vocab_size, (3, 13))
    tgt[1, :5] = -100
    if family == "llama":
        cos, sin = ops.rope_tables(cfg.head_dim, cfg.context_length, cfg.rope_base, cfg.rope_freq)
        fn = lambda sd: llama_loss(sd, cfg, idx, tgt, cos, sin, lora=2.0)  # noqa: E731
    else:
        fn = lambda sd: gpt2_loss(sd, cfg, idx, tgt, lora=2.0)  # noqa: E731
    _compare(m, fn, idx, tgt)
    (m(idx, tgt) * 4.0).backward()
    g4 = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    m(idx, tgt).backward()
    g1 = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    for n in g1:
        assert torch.allclose(g4[n], 4.0 * g1[n], rtol=1e-5, atol=1e-6), n


@pytest.mark.parametrize("family", ["llama", "gpt2"])
def test_fused_chunked_head_ce(family, monkeypatch):
    """Head + CE fused chunk by chunk (logits never materialised whole): several chunks, a
    chunk boundary inside the sequence, ignore_index targets, and a non-unit dloss (fp16 loss
    scaling path) all give the eager-autograd gradients."""
    from building_llm_from_scratch_amd.models import llama
    monkeypatch.setattr(llama, "MIN_CHUNK_ROWS", 8)
    monkeypatch.setattr(llama, "LOGIT_CHUNK_BYTES", 8 * 97 * 4)   # 8 rows of fp32 logits per chunk
    torch.manual_seed(0)
    cfg = _small_llama() if family == "llama" else _small_gpt2()
    m = build_model(cfg)
    idx = torch.randint(0, cfg.vocab_size, (3, 13))
    tgt = torch.randint(0, cfg.vocab_size, (3, 13))
    tgt[1, :5] = -100
    if family == "llama":
        cos, sin = ops.rope_tables(cfg.head_dim, cfg.context_length, cfg.rope_base, cfg.rope_freq)
        fn = lambda sd: llama_loss(sd, cfg, idx, tgt, cos, sin)  # noqa: E731
    else:
        fn = lambda sd: gpt2_loss(sd, cfg, idx, tgt)  # noqa: E731
    _compare(m, fn, idx, tgt)
    # dloss != 1: gradients scale exactly (unit backwards overwrite the flat gradients)
    (m(idx, tgt) * 4.0).backward()
    g4 = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    m(idx, tgt).backward()
    g1 = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    for n in g1:
        assert torch.allclose(g4[n], 4.0 * g1[n], rtol=1e-5, atol=1e-6), n
    # announced loss scale (the Trainer's fp16 path): the logit gradient is taken at dloss = S in
    # the forward and divided by S in backward; S = the arriving dloss gives the same gradients
    m.rctx.loss_scale = 1024.0
    (m(idx, tgt) * 1024.0).backward()
    gs = {n: p.grad.clone() / 1024.0 for n, p in m.named_parameters() if p.grad is not None}
    m.rctx.loss_scale = 1.0
    for n in g1:
        assert torch.allclose(gs[n], g1[n], rtol=1e-5, atol=1e-7), n


def test_selective_rebuilds_activation_and_norms():
    """``selective`` keeps neither the norm outputs nor the SwiGLU / GELU activation (the
    backward rebuilds them); ``none`` keeps both.  Gradients are covered by test_llama_grads."""
    from building_llm_from_scratch_amd.models.base import _BlockFn
    seen = {}
    orig = _BlockFn.forward

    def spy(ctx, x, comp):
        y = orig(ctx, x, comp)
        seen[comp.rctx.block_mode(comp.index)] = set(ctx.saved)
        return y
    for family, cfg in (("llama", _small_llama()), ("gpt2", _small_gpt2())):
        for mode in ("none", "selective"):
            m = build_model(cfg, use_actv_ckpt=mode)
            idx = torch.randint(0, cfg.vocab_size, (2, 16))
            _BlockFn.forward = staticmethod(spy)
            try:
                m(idx, idx)
            finally:
                _BlockFn.forward = staticmethod(orig)
            act = "act" if family == "llama" else "g"
            keys = seen[mode]
            assert ({"h1", "h2", act} <= keys) == (mode == "none"), (family, mode, keys)


def _torch_ckpt_blocks(n, segments):
    """Blocks torch.utils.checkpoint.checkpoint_sequential(fns, segments, x) re-runs in
    backward: it checkpoints ``segments - 1`` chunks of ``n // segments`` and runs the rest
    plainly (the reference's --use_actv_ckpt call passes segments = n_layers)."""
    size = n // segments
    return [i for i in range(n) if i < size * (segments - 1)]


@pytest.mark.parametrize("n,segments", [(5, None), (5, 2), (5, 3), (4, 4), (6, 1), (32, None), (32, 2)])
def test_ckpt_segments_match_checkpoint_sequential(n, segments):
    cfg = _small_llama().replace(n_layers=n)
    m = build_model(cfg, use_actv_ckpt="full")
    m.set_actv_ckpt("full", segments)
    got = [i for i in range(n) if m.rctx.block_mode(i) == "full"]
    assert got == _torch_ckpt_blocks(n, segments or n)


@pytest.mark.parametrize("segments", [None, 2, 3])
@pytest.mark.parametrize("family", ["llama", "gpt2"])
def test_ckpt_segments_grads(family, segments):
    """Gradients are exact for every segmentation, and exactly the checkpointed blocks re-run
    their forward in backward."""
    torch.manual_seed(0)
    cfg = (_small_llama() if family == "llama" else _small_gpt2()).replace(n_layers=5)
    m = build_model(cfg, use_actv_ckpt="full")
    m.set_actv_ckpt("full", segments)
    recomputed = []
    for comp in m.computes:
        if comp.index >= 0:
            fwd = comp.forward

            def spy(x, save, replay=None, recompute=False, _f=fwd, _i=comp.index):
                if recompute:
                    recomputed.append(_i)
                return _f(x, save, replay=replay, recompute=recompute)
            comp.forward = spy
    idx = torch.randint(0, cfg.vocab_size, (2, 16))
    tgt = torch.randint(0, cfg.vocab_size, (2, 16))
    if family == "llama":
        cos, sin = ops.rope_tables(cfg.head_dim, cfg.context_length, cfg.rope_base, cfg.rope_freq)
        _compare(m, lambda sd: llama_loss(sd, cfg, idx, tgt, cos, sin), idx, tgt)
    else:
        _compare(m, lambda sd: gpt2_loss(sd, cfg, idx, tgt), idx, tgt)
    assert sorted(recomputed) == _torch_ckpt_blocks(5, segments or 5)


def test_reference_gpt_model_smoke_shape():
    """Counterpart of the reference's only assert-based test (Models/GPT2/GPT2.py:127-149,
    test_gpt_model): a random-init small GPT (ctx 128, d 256, 4 heads, 4 layers) maps random ids
    [2, 128] to logits [2, 128, 50257]."""
    from building_llm_from_scratch_amd.config import get_config
    torch.manual_seed(123)
    cfg = get_config("GPT2", "124M").replace(context_length=128, emb_dim=256, n_heads=4, n_kv_groups=4,
                                             hidden_dim=1024, n_layers=4, dtype=torch.float32)
    m = build_model(cfg)
    idx = torch.randint(0, cfg.vocab_size, (2, 128))
    with torch.no_grad():
        logits = m(idx)
    assert logits.shape == (2, 128, 50257)
    assert torch.isfinite(logits).all()


def test_swiglu_bwd_lowrank_wgrad_reference_semantics():
    """The CPU path of ops.swiglu_bwd_lowrank_wgrad (the contract its HIP kernel is tested
    against on the GPU): dgu = swiglu_bwd(gu, base + s u P), gB_gate/up (+)= st^T dg / du,
    gA_down^T (+)= s u^T swiglu_fwd(gu)."""
    import torch
    from building_llm_from_scratch_amd import ops
    from building_llm_from_scratch_amd.ops import reference as ref
    torch.manual_seed(0)
    N, F, r, s = 37, 64, 16, 0.5
    gu, base = torch.randn(N, 2 * F), torch.randn(N, F)
    u, P, st = torch.randn(N, r), 0.1 * torch.randn(r, F), torch.randn(N, 32)
    for acc in (False, True):
        g0 = [torch.randn(r, F), torch.randn(r, F), torch.randn(F, r).t()]
        g = [x.clone() for x in g0]
        dgu = ops.swiglu_bwd_lowrank_wgrad(gu, base, u, P, s, st, g[0], g[1], g[2], acc)
        want = ref.swiglu_bwd(gu, base + s * u @ P)
        assert torch.allclose(dgu, want, atol=1e-5)
        act = ref.swiglu_fwd(gu)
        exp = [st[:, :16].t() @ want[:, :F], st[:, 16:].t() @ want[:, F:], s * u.t() @ act]
        for a, e, b in zip(g, exp, g0):
            assert torch.allclose(a, e + (b if acc else 0), atol=1e-4)


def test_lora_head_bwd_cpu_contract():
    """ops.lora_head_bwd_ (CPU path): u = dl B^T and gB (+)= st^T dl into a transposed view."""
    torch.manual_seed(0)
    R, V = 70, 192
    dl, st, B = torch.randn(R, V), torch.randn(R, 16), torch.randn(16, V)
    u = torch.empty(R, 16)
    g0 = torch.randn(V, 16)
    for acc in (False, True):
        gB = g0.clone().t()
        ops.lora_head_bwd_(dl, st, B, u, gB, acc)
        torch.testing.assert_close(u, dl @ B.t())
        torch.testing.assert_close(gB, st.t() @ dl + (g0.t() if acc else 0))
