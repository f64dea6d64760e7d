"""HIP kernels vs the plain-PyTorch fp32 reference (ops/reference.py).  GPU only.

Closeness (tests/numerics.py): the error is measured in units of what rounding the exact fp32
oracle to the kernel's output dtype costs, globally and per |ref|-magnitude decile, so an error
confined to small elements (a GQA partial, a masked-tile edge) is not hidden by the large ones;
``k`` is the allowance per kernel class (<= 5 for bf16 / fp16: test_numerics_check.py shows a 1 %
perturbation of the smallest 10 % of elements exceeds it).  Per-row statistics (log-sum-exp,
CE rows, rstd) and the optimizer state are checked elementwise (``check_elem``)."""
import math

import pytest
import torch
from numerics import check_close, check_elem

from building_llm_from_scratch_amd import ops
from building_llm_from_scratch_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
DTYPES = [torch.bfloat16, torch.float16, torch.float32]
# allowance per kernel class, in rounding units: the former max-normalised scale factor -> k
K_OF = {0.5: 1.5, 1: 2.0, 2: 3.0, 4: 5.0}
K_MAX = 5.0


def _close(a, b, dt, scale=1.0, name=""):
    k = K_OF[scale]
    assert k <= K_MAX
    check_close(a, b, dt, k=k, name=name)


def _ulps(a, b, dt, n=1.0, name=""):
    """Two GPU results that should agree to n ulps of dt (same arithmetic, different order)."""
    u = {torch.bfloat16: 2.0 ** -7, torch.float16: 2.0 ** -10, torch.float32: 2.0 ** -22}[dt]
    b = b.float()
    # atol: n ulps of the vector's RMS (a column sum that cancels to ~0 differs by the fp32
    # summation order, not by a fraction of its own tiny magnitude)
    check_elem(a.float(), b, rtol=n * u, atol=n * u * b.pow(2).mean().sqrt().item(), name=name)


LSE_TOL = dict(rtol=1e-5, atol=2e-5)      # fp32 log-sum-exp of bf16 / fp16 / fp32 scores


@pytest.fixture(autouse=True)
def _ext():
    assert ops.load_ext(required=True)
    torch.manual_seed(0)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("d", [32, 768, 1600, 4096])
def test_rmsnorm(dt, d):
    N = 67
    x = torch.randn(N, d, device=DEV).to(dt)
    w = (1 + 0.1 * torch.randn(d, device=DEV)).to(dt)
    dy = torch.randn(N, d, device=DEV).to(dt)
    acc = torch.randn(N, d, device=DEV).to(dt)
    y, r = ops.rmsnorm_fwd(x, w, 1e-5)
    y0, r0 = ref.rmsnorm_fwd(x.cpu().float(), w.cpu().float(), 1e-5)
    _close(y, y0, dt, name="y")
    check_elem(r, r0, rtol=2e-5, atol=0, name="rstd")
    dx, dw = ops.rmsnorm_bwd(dy, x, w, r, acc)
    dx0, dw0 = ref.rmsnorm_bwd(dy.cpu().float(), x.cpu().float(), w.cpu().float(), r0, acc.cpu().float())
    _close(dx, dx0, dt, 2, name="dx")
    _close(dw, dw0, dt, 2, name="dw")
    # weight gradient written / accumulated straight into a parameter-dtype buffer
    for accumulate in (False, True):
        out = torch.randn(d, device=DEV).to(dt)
        expect = dw0 + (out.cpu().float() if accumulate else 0)
        ops.rmsnorm_bwd(dy, x, w, r, acc, out, accumulate)
        _close(out, expect, dt, 4, name=f"dw_out acc={accumulate}")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("d", [32, 768, 1280])
def test_layernorm(dt, d):
    N = 53
    x = (torch.randn(N, d, device=DEV) + 0.5).to(dt)
    w = (1 + 0.1 * torch.randn(d, device=DEV)).to(dt)
    b = (0.1 * torch.randn(d, device=DEV)).to(dt)
    dy = torch.randn(N, d, device=DEV).to(dt)
    y, m, r = ops.layernorm_fwd(x, w, b, 1e-5)
    y0, m0, r0 = ref.layernorm_fwd(x.cpu().float(), w.cpu().float(), b.cpu().float(), 1e-5)
    _close(y, y0, dt, name="y")
    dx, dw, db = ops.layernorm_bwd(dy, x, w, m, r, None)
    dx0, dw0, db0 = ref.layernorm_bwd(dy.cpu().float(), x.cpu().float(), w.cpu().float(), m0, r0, None)
    _close(dx, dx0, dt, 2, name="dx")
    _close(dw, dw0, dt, 2, name="dw")
    _close(db, db0, dt, 2, name="db")
    for accumulate in (False, True):
        ow, ob = torch.randn(d, device=DEV).to(dt), torch.randn(d, device=DEV).to(dt)
        ew = dw0 + (ow.cpu().float() if accumulate else 0)
        eb = db0 + (ob.cpu().float() if accumulate else 0)
        ops.layernorm_bwd(dy, x, w, m, r, None, ow, ob, accumulate)
        _close(ow, ew, dt, 4, name="dw_out")
        _close(ob, eb, dt, 4, name="db_out")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("F", [10, 64, 1000, 4104, 14336])
def test_swiglu_gelu(dt, F):
    gu = torch.randn(33, 2 * F, device=DEV).to(dt)
    da = torch.randn(33, F, device=DEV).to(dt)
    _close(ops.swiglu_fwd(gu), ref.swiglu_fwd(gu.cpu().float()), dt, name="swiglu")
    _close(ops.swiglu_bwd(gu, da), ref.swiglu_bwd(gu.cpu().float(), da.cpu().float()), dt, 2, name="swiglu_bwd")
    # fused variant: same dgu, and act written in place of dact
    da2 = da.clone()
    dgu2 = ops.swiglu_bwd_act(gu, da2)
    assert torch.equal(dgu2, ops.swiglu_bwd(gu, da))
    assert torch.equal(da2, ops.swiglu_fwd(gu))
    f = torch.randn(33, F, device=DEV).to(dt)
    _close(ops.gelu_fwd(f), ref.gelu_fwd(f.cpu().float()), dt, name="gelu")
    _close(ops.gelu_bwd(f, da), ref.gelu_bwd(f.cpu().float(), da.cpu().float()), dt, name="gelu_bwd")


@pytest.mark.parametrize("dt", DTYPES)
def test_dropout_bitexact_mask(dt):
    x = torch.randn(37, 96, device=DEV).to(dt)
    a = torch.randn(37, 96, device=DEV).to(dt)
    out = ops.dropout_add(x, a, 0.1, 1234, 777)
    out0 = ref.dropout_add(x.cpu().float(), a.cpu().float(), 0.1, 1234, 777)
    _close(out, out0, dt, name="dropout_add")
    keep_gpu = (ops.dropout_bwd(torch.ones(37, 96, device=DEV, dtype=dt), 0.1, 1234, 777) != 0).cpu()
    keep_ref = ref.drop_keep_mask(1234, 777, 37 * 96, 0.1).view(37, 96)
    assert torch.equal(keep_gpu, keep_ref)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("hd,H,G", [(64, 4, 4), (128, 8, 2), (2, 16, 8)])
def test_rope(dt, hd, H, G):
    B, T = 2, 17
    cos, sin = ops.rope_tables(hd, 32, 500000.0, {"factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                                  "original_context_length": 8192}, device=DEV)
    qkv = torch.randn(B * T, (H + 2 * G) * hd, device=DEV).to(dt)
    q0 = ref.rope_(qkv.cpu().float().clone(), cos.cpu(), sin.cpu(), T, H, G, hd)
    q1 = ops.rope_(qkv.clone(), cos, sin, T, H, G, hd)
    _close(q1, q0, dt, name="rope")
    back = ops.rope_(q1.clone(), cos, sin, T, H, G, hd, inverse=True)
    _close(back, qkv.float(), dt, 2, name="rope inverse")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("V", [97, 50257, 128256])
def test_cross_entropy(dt, V):
    N = 24
    logits = (3 * torch.randn(N, V, device=DEV)).to(dt)
    tgt = torch.randint(0, V, (N,), device=DEV)
    tgt[3] = -100
    l, lse = ops.ce_fwd(logits, tgt)
    l0, lse0 = ref.ce_fwd(logits.cpu().float(), tgt.cpu())
    check_elem(l, l0, **LSE_TOL, name="loss")
    check_elem(lse, lse0, **LSE_TOL, name="lse")
    scale = torch.tensor([0.5], device=DEV)
    g = ops.ce_bwd_(logits.clone(), tgt, lse, scale)
    g0 = ref.ce_bwd_(logits.cpu().float().clone(), tgt.cpu(), lse0, scale.cpu())
    _close(g, g0, dt, 2, name="dlogits")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("pos", [False, True])
def test_embedding(dt, pos):
    V, d, B, T = 300, 64, 3, 16
    wte = torch.randn(V, d, device=DEV).to(dt)
    wpe = torch.randn(T, d, device=DEV).to(dt) if pos else None
    idx = torch.randint(0, 40, (B * T,), device=DEV)  # many duplicates
    x = ops.embedding_fwd(idx, wte, wpe, T)
    x0 = ref.embedding_fwd(idx.cpu(), wte.cpu().float(), None if wpe is None else wpe.cpu().float(), T)
    _close(x, x0, dt, name="emb fwd")
    dx = torch.randn(B * T, d, device=DEV).to(dt)
    g = torch.full((V, d), 7.0, device=DEV, dtype=dt)
    gp = torch.zeros(T, d, device=DEV, dtype=dt) if pos else None
    ops.embedding_bwd(idx, dx, g, gp, T, accumulate=False)
    g0 = torch.zeros(V, d)
    gp0 = torch.zeros(T, d) if pos else None
    ref.embedding_bwd(idx.cpu(), dx.cpu().float(), g0, gp0, T)
    _close(g, g0, dt, 4, name="emb dW")
    if pos:
        _close(gp, gp0, dt, 4, name="pos dW")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("d", [1280, 4096])
def test_embedding_bwd_long_runs(dt, d):
    """Byte-level vocabularies give runs of hundreds of equal ids: runs longer than one 64-id
    ballot probe and not a multiple of the 16-row index batch, a 1-row run, a partial last
    column slice (1280 = 2.5 x 512), and accumulate=True onto an existing gradient."""
    V = 50
    g_ = torch.Generator().manual_seed(5)
    # sorted runs that start / end exactly on the 128-position block boundaries of the kernel,
    # span several blocks, or are one row long; then shuffled into token order
    counts = torch.tensor([128, 256, 1, 127, 129, 300, 1, 1, 383, 64, 640])
    idx = torch.repeat_interleave(torch.arange(3, 3 + len(counts)), counts)
    idx = idx[torch.randperm(idx.numel(), generator=g_)].to(DEV)
    N = idx.numel()
    dx = torch.randn(N, d, device=DEV).to(dt)
    base = torch.randn(V, d, device=DEV).to(dt)
    g = base.clone()
    ops.embedding_bwd(idx, dx, g, None, N, accumulate=True)
    g0 = torch.zeros(V, d)
    ref.embedding_bwd(idx.cpu(), dx.cpu().float(), g0, None, N)
    _close(g, g0 + base.cpu().float(), dt, 4, name="emb dW (long runs, accumulate)")


@pytest.mark.parametrize("pdt", [torch.bfloat16, torch.float32])
def test_adamw_and_norm(pdt):
    n = 4099
    p32 = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV).to(pdt)
    m = torch.randn(n, device=DEV).abs() * 0.1
    v = torch.randn(n, device=DEV).abs() * 0.1
    scale = torch.tensor([0.7], device=DEV)
    master = p32.clone() if pdt != torch.float32 else None
    param = p32.to(pdt)
    args = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.1, step=3)
    refs = [t.cpu().clone() if t is not None else None for t in (param, master, g, m, v)]
    ops.adamw_step_(param, master, g, m, v, grad_scale=scale, **args)
    ref.adamw_step_(refs[0], refs[1], refs[2], refs[3], refs[4], grad_scale=scale.cpu(), **args)
    check_elem(m, refs[3], rtol=1e-6, atol=1e-7, name="m")
    check_elem(v, refs[4], rtol=5e-5, atol=1e-9, name="v")  # v + (1-b2)(g^2 - v) form: ~1e-5 rel
    if master is not None:
        check_elem(master, refs[1], rtol=1e-6, atol=1e-7, name="master")
    _close(param, refs[0], pdt, name="param")
    ts = [torch.randn(1000, device=DEV).to(pdt), torch.randn(37, device=DEV), torch.randn(100003, device=DEV).to(pdt)]
    sq = ops.sq_norm_multi(ts)
    sq0 = sum(t.float().pow(2).sum() for t in ts)
    assert math.isclose(sq.item(), sq0.item(), rel_tol=1e-4)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("B,T,H,G,hd", [(2, 64, 4, 4, 64), (1, 200, 8, 2, 128), (2, 33, 4, 2, 64),
                                         (1, 10, 16, 8, 2), (2, 256, 4, 1, 128), (1, 512, 8, 2, 128),
                                         (1, 300, 2, 2, 128), (1, 96, 3, 3, 64)])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention(dt, B, T, H, G, hd, p, causal):
    qkv = torch.randn(B * T, (H + 2 * G) * hd, device=DEV).to(dt)
    do = torch.randn(B * T, H * hd, device=DEV).to(dt)
    o, lse = ops.flash_attn_fwd(qkv, B, T, H, G, hd, causal, p, 99, 12345)
    o0, lse0 = ref.flash_attn_fwd(qkv.cpu().float(), B, T, H, G, hd, causal, p, 99, 12345)
    _close(o, o0, dt, 2, name="o")
    check_elem(lse, lse0, **LSE_TOL, name="lse")
    dqkv = ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, causal, p, 99, 12345)
    dqkv0 = ref.flash_attn_bwd(qkv.cpu().float(), o0, lse0, do.cpu().float(), B, T, H, G, hd, causal, p, 99,
                               12345)
    _close(dqkv, dqkv0, dt, 4, name="dqkv")


@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("B,T,H,G", [(2, 256, 4, 4), (1, 200, 4, 2), (2, 33, 2, 2), (1, 1024, 4, 1)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_keep_mask(hd, B, T, H, G, causal):
    """The forward's dropout keep bits (word (kw, q), bit j = key 32kw + j) equal the counter
    hash of the oracle for every (query, key) the softmax covers, and a backward reading them is
    bit-identical to one that re-hashes."""
    p, seed, offset = 0.1, 99, 12345
    qkv = torch.randn(B * T, (H + 2 * G) * hd, device=DEV).to(torch.bfloat16)
    do = torch.randn(B * T, H * hd, device=DEV).to(torch.bfloat16)
    km = ops.attn_keep_mask(qkv, B, T, H, hd, p)
    assert km is not None
    o, lse = ops.flash_attn_fwd(qkv, B, T, H, G, hd, causal, p, seed, offset, keep_mask=km)
    o2, lse2 = ops.flash_attn_fwd(qkv, B, T, H, G, hd, causal, p, seed, offset)
    assert torch.equal(o, o2) and torch.equal(lse, lse2)
    KW = (T + 31) // 32
    bits = (km.view(B * H, KW, T).permute(0, 2, 1).unsqueeze(-1).to(torch.int64)
            >> torch.arange(32, device=DEV)) & 1                        # [BH, T(q), KW, 32]
    got = bits.reshape(B * H, T, KW * 32)[:, :, :T].bool()
    want = ref.drop_keep_mask(seed, offset, B * H * T * T, p, device=DEV).view(B * H, T, T)
    cover = torch.ones(T, T, dtype=torch.bool, device=DEV)
    if causal:
        cover = cover.tril()
    assert torch.equal(got[:, cover], want[:, cover])
    d1 = ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, causal, p, seed, offset, keep_mask=km)
    d2 = ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, causal, p, seed, offset)
    assert torch.equal(d1, d2)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("hd,step", [(128, 0.35), (128, 0.6), (64, 0.5)])
def test_flash_attention_deferred_rescale(dt, hd, step):
    """Scores that grow tile by tile (key j scaled by step * (j // 64) along the query
    direction): each query's running max rises by 4-10 log2 units per 64-key tile, so the
    forward both defers (rise < kRescaleThr) and takes the rescale branch mid-sequence --
    random data almost never exercises the deferred path."""
    B, T, H, G = 1, 512, 4, 2
    g = torch.Generator(device=DEV).manual_seed(hd)
    u = torch.randn(hd, device=DEV, generator=g)
    q = u + 0.3 * torch.randn(B * T, H, hd, device=DEV, generator=g)
    a = step * (torch.arange(T, device=DEV) // 64).float() / (hd ** 0.5) * 8.0
    k = a[:, None, None] * u + 0.3 * torch.randn(B * T, G, hd, device=DEV, generator=g)
    v = torch.randn(B * T, G, hd, device=DEV, generator=g)
    qkv = torch.cat([q, k, v], 1).reshape(B * T, (H + 2 * G) * hd).to(dt)
    do = torch.randn(B * T, H * hd, device=DEV, generator=g).to(dt)
    o, lse = ops.flash_attn_fwd(qkv, B, T, H, G, hd, True, 0.0, 1, 0)
    o0, lse0 = ref.flash_attn_fwd(qkv.float(), B, T, H, G, hd, True, 0.0, 1, 0)
    _close(o, o0, dt, 2, name="o")
    check_elem(lse, lse0, **LSE_TOL, name="lse")
    dqkv = ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, True, 0.0, 1, 0)
    dqkv0 = ref.flash_attn_bwd(qkv.float(), o0, lse0, do.float(), B, T, H, G, hd, True, 0.0, 1, 0)
    _close(dqkv, dqkv0, dt, 4, name="dqkv")


@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_fwd_small_tiles(causal):
    """hd 64 with dropout on a grid of >= 2048 workgroups (16 x 16 heads x 8 query blocks) takes
    the 32-key-tile forward at 3 workgroups per CU (csrc/attn_mfma.hip:fwd_small_tiles): against
    the oracle, and its keep-mask words equal the oracle's hash."""
    test_flash_attention(torch.bfloat16, 16, 1024, 16, 16, 64, 0.1, causal)
    test_flash_attention_keep_mask(64, 16, 1024, 16, 16, causal)


def test_flash_attention_fp32_is_flash_not_materialised():
    """GPT-2 in the reference's default fp32 (args.py:77) at T = 4096, 12 heads: the fp32 kernels'
    footprint is O(T) -- the materialised oracle would need 12 x 4096^2 x 4 B = 805 MB per sequence."""
    B, T, H, hd = 2, 4096, 12, 64
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    o, lse = ops.flash_attn_fwd(qkv, B, T, H, H, hd, True, 0.1, 3, 0)
    dq = ops.flash_attn_bwd(qkv, o, lse, torch.randn_like(o), B, T, H, H, hd, True, 0.1, 3, 0)
    torch.cuda.synchronize()
    extra = torch.cuda.max_memory_allocated() - base
    assert extra < 3 * qkv.numel() * 4, extra
    assert torch.isfinite(dq).all()


@pytest.mark.parametrize("T", [1024, 2048, 4096, 8192])
@pytest.mark.parametrize("H,G,hd,p", [(32, 8, 128, 0.0), (12, 12, 64, 0.1)])
def test_flash_attention_long_context(T, H, G, hd, p):
    """The bench shape (Llama-3-8B: 32 q / 8 kv heads x 128) and GPT-2 (hd 64, dropout) at
    T = 1k..8k (``--context_length``); fp32 reference evaluated on the GPU (the [H,T,T] scores
    of the oracle fit in HBM; the kernels never form them)."""
    B = 1
    g = torch.Generator(device=DEV).manual_seed(T + hd)
    qkv = torch.randn(B * T, (H + 2 * G) * hd, device=DEV, generator=g).to(torch.bfloat16)
    do = torch.randn(B * T, H * hd, device=DEV, generator=g).to(torch.bfloat16)
    o, lse = ops.flash_attn_fwd(qkv, B, T, H, G, hd, True, p, 7, 4242)
    o0, lse0 = ref.flash_attn_fwd(qkv.float(), B, T, H, G, hd, True, p, 7, 4242)
    _close(o, o0, torch.bfloat16, 2, name="o")
    check_elem(lse, lse0, **LSE_TOL, name="lse")
    dqkv = ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, True, p, 7, 4242)
    del o0
    dqkv0 = ref.flash_attn_bwd(qkv.float(), o.float(), lse0, do.float(), B, T, H, G, hd, True, p, 7, 4242)
    _close(dqkv, dqkv0, torch.bfloat16, 4, name="dqkv")


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("hd", [64, 128])
def test_flash_attention_gqa_fused_heads(p, hd):
    """Grid large enough (B*G*ceil(T/128) >= 1024) that dK/dV takes the fused-GQA-heads variant."""
    test_flash_attention(torch.bfloat16, 128, 128, 16, 8, hd, p, True)


@pytest.mark.parametrize("hd", [64, 128])
def test_flash_attention_keep_mask_fused_gqa(hd):
    """The keep-mask path of the fused-GQA-heads dK/dV kernel (the workgroup sweeps its kv
    head's query heads, each with its own mask rows)."""
    test_flash_attention_keep_mask(hd, 128, 128, 16, 8, True)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("B,T,H,G,hd", [(2, 200, 4, 4, 128),     # MHA: dK written by the dK/dV kernel
                                         (1, 300, 8, 2, 128),     # GQA: fp32 partials + reduce kernel
                                         (128, 128, 16, 8, 128),  # GQA heads fused in one workgroup
                                         (2, 130, 4, 2, 64), (128, 128, 16, 8, 64)])
def test_flash_attention_bwd_fused_rope(dt, B, T, H, G, hd):
    """``flash_attn_bwd(..., rope=(cos, sin))`` un-rotates dQ / dK in the kernels' epilogues:
    equal (to rounding) to the backward followed by the separate inverse ``rope_`` pass, and to
    the fp32 oracle of that composition."""
    cos, sin = ops.rope_tables(hd, 512, 500000.0, device=DEV)
    qkv = torch.randn(B * T, (H + 2 * G) * hd, device=DEV).to(dt)
    do = torch.randn(B * T, H * hd, device=DEV).to(dt)
    o, lse = ops.flash_attn_fwd(qkv, B, T, H, G, hd, True)
    fused = ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, True, rope=(cos, sin))
    sep = ops.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, True)
    ops.rope_(sep, cos, sin, T, H, G, hd, inverse=True)
    want = ref.flash_attn_bwd(qkv.float(), o.float(), lse, do.float(), B, T, H, G, hd, True)
    ref.rope_(want, cos, sin, T, H, G, hd, inverse=True)
    _close(fused, want.cpu(), dt, 4, name="fused vs oracle")
    _close(sep, want.cpu(), dt, 4, name="separate vs oracle")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,H,G,hd,L,Tmax",[(2, 8, 2, 128, 37, 64), (1, 4, 4, 64, 1, 16), (3, 32, 8, 128, 1000, 1024)])
def test_attn_decode(dt, B, H, G, hd, L, Tmax):
    q = torch.randn(B, H, hd, device=DEV).to(dt)
    kc = torch.randn(B, G, Tmax, hd, device=DEV).to(dt)
    vc = torch.randn(B, G, Tmax, hd, device=DEV).to(dt)
    o = ops.attn_decode(q, kc, vc, L)
    o0 = ref.attn_decode(q.cpu().float(), kc.cpu().float(), vc.cpu().float(), L)
    _close(o, o0, dt, 2, name="decode")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("N,F", [(4096, 3840), (7, 64), (300, 5120), (16390, 1280)])
@pytest.mark.parametrize("acc", [False, True])
def test_bias_grad(dt, N, F, acc):
    dy = torch.randn(N, F, device=DEV).to(dt)
    db = torch.randn(F, device=DEV).to(dt)
    ref0 = dy.float().sum(0) + (db.float() if acc else 0)
    ops.bias_grad_(dy, db, acc)
    _close(db, ref0.cpu(), dt, 4, name="bias_grad")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("N,F", [(24576, 1280), (24576, 5120), (1000, 768), (37, 64)])
@pytest.mark.parametrize("acc", [False, True])
def test_bwd_bias_grad_fused(dt, N, F, acc):
    """dropout / GELU backward with the bias column sums in the same pass: outputs bitwise equal
    to the separate kernels; db (same bands, same per-lane row order, fp32 sums) within one ulp
    of db's dtype of the separate column sum."""
    dy = torch.randn(N, F, device=DEV).to(dt)
    f = torch.randn(N, F, device=DEV).to(dt)
    db0 = torch.randn(F, device=DEV).to(dt)
    for name, fused, sep in (
            ("dropout", lambda db: ops.dropout_bwd_bias(dy, 0.1, 1234, 77, db, acc),
             lambda: ops.dropout_bwd(dy, 0.1, 1234, 77)),
            ("gelu", lambda db: ops.gelu_bwd_bias(f, dy, db, acc), lambda: ops.gelu_bwd(f, dy))):
        db1, db2 = db0.clone(), db0.clone()
        out1 = fused(db1)
        out2 = sep()
        ops.bias_grad_(out2, db2, acc)
        assert torch.equal(out1, out2), name
        _ulps(db1, db2, dt, 1, name=name + " db")  # one ulp of db's dtype
    # GELU backward that also rebuilds g = gelu(f) in place of dg (GPT-2 checkpoint recompute),
    # with and without the bias sums
    for with_db in (True, False):
        d = dy.clone()
        db3 = db0.clone() if with_db else None
        out3 = ops.gelu_bwd_act(f, d, db3, acc)
        assert torch.equal(out3, ops.gelu_bwd(f, dy))
        assert torch.equal(d, ops.gelu_fwd(f))
        if with_db:
            db4 = db0.clone()
            ops.bias_grad_(out3, db4, acc)
            _ulps(db3, db4, dt, 1, name="gelu act db")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("N,d", [(4096, 1280), (53, 768), (37, 64)])
def test_dropout_add_layernorm_fused(dt, N, d):
    """GPT-2's attention residual: dropout-add + LayerNorm forward in one pass, bitwise the two
    kernels, and against the fp32 oracle."""
    p, seed, off = 0.1, 4321, 1001
    x = (torch.randn(N, d, device=DEV) + 0.5).to(dt)
    a = torch.randn(N, d, device=DEV).to(dt)
    w = (1 + 0.1 * torch.randn(d, device=DEV)).to(dt)
    b = (0.1 * torch.randn(d, device=DEV)).to(dt)
    x2, y, m, r = ops.dropout_add_layernorm(x, a, w, b, 1e-5, p, seed, off)
    x2s = ops.dropout_add(x, a, p, seed, off)
    ys, ms, rs = ops.layernorm_fwd(x2s, w, b, 1e-5)
    assert torch.equal(x2, x2s) and torch.equal(y, ys) and torch.equal(m, ms) and torch.equal(r, rs)
    x20 = ref.dropout_add(x.cpu().float(), a.cpu().float(), p, seed, off)
    y0, _, _ = ref.layernorm_fwd(x20, w.cpu().float(), b.cpu().float(), 1e-5)
    _close(x2, x20, dt, name="x2")
    _close(y, y0, dt, 2, name="y")


# ------------------------------------------------------------------ LoRA (csrc/lora.hip)
def _up_only(t, Bs, c0, offs, s, N, M):
    out = torch.zeros(N, M, device=DEV)
    for B, c, o in zip(Bs, c0, offs):
        out[:, c:c + B.shape[1]] = s * t[:, o:o + B.shape[0]].float() @ B.float()
    return out

@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("r", [16, 64])
@pytest.mark.parametrize("N", [1024, 1000, 37, 9288])
def test_lora_kernels(dt, r, N):
    """pack / down / up / wgrad against fp32 matmuls, Q/K/V-style group (3 members, unequal
    widths), including split-N partial reduction, accumulation and transposed grad views; token
    counts that are not multiples of 16 / 64 (variable-length Alpaca batches: 24 x 387 = 9288)."""
    K = 512
    outs = [512, 128, 128]
    c0 = [0, 512, 640]
    M = sum(outs)
    x = torch.randn(N, K, device=DEV).to(dt)
    As = [(0.1 * torch.randn(K, r, device=DEV)).to(dt) for _ in outs]
    Bs = [(0.1 * torch.randn(r, o, device=DEV)).to(dt) for o in outs]
    offs = [i * r for i in range(3)]
    R = 3 * r
    s = 0.5
    P = ops.lora_pack_t(As)
    assert torch.equal(P.cpu(), torch.cat([a.t() for a in As], 0).cpu())
    t = ops.lora_down(x, [P], [0], [K], [0], R)
    t0 = x.float() @ P.float().t()
    _close(t, t0, dt, 2, name="down fwd")
    y = torch.randn(N, M, device=DEV).to(dt)
    y0 = y.float().clone()
    ops.lora_up_(y, t, Bs, c0, offs, s, base=y)          # in place (base aliases y)
    for B, c, o in zip(Bs, c0, offs):
        y0[:, c:c + B.shape[1]] += s * t[:, o:o + r].float() @ B.float()
    _close(y, y0, dt, 2, name="up fwd")
    bias = torch.randn(M, device=DEV).to(dt)
    y2 = torch.empty(N, M, device=DEV, dtype=dt)
    ops.lora_up_(y2, t, Bs, c0, offs, s, bias=bias)       # write-only + bias
    _close(y2, _up_only(t, Bs, c0, offs, s, N, M) + bias.float(), dt, 2, name="up bias")
    dy = torch.randn(N, M, device=DEV).to(dt)
    u = ops.lora_down(dy, Bs, c0, outs, offs, R)
    u0 = torch.cat([dy[:, c:c + o].float() @ B.float().t() for B, c, o in zip(Bs, c0, outs)], 1)
    _close(u, u0, dt, 2, name="down bwd")
    for accumulate in (False, True):
        for gdt in (torch.float32, dt):
            gB = [torch.randn(r, o, device=DEV).to(gdt) for o in outs]
            gB0 = [s * t[:, o:o + r].float().t() @ dy[:, c:c + n].float() + (g.float() if accumulate else 0)
                   for g, o, c, n in zip(gB, offs, c0, outs)]
            ops.lora_wgrad(t, dy, gB, offs, c0, s, accumulate)
            for g, g0 in zip(gB, gB0):
                _close(g, g0, dt, 4, name=f"dB acc={accumulate} {gdt}")
            gA = [torch.randn(K, r, device=DEV).to(gdt) for _ in outs]
            gA0 = [s * x.float().t() @ u[:, o:o + r].float() + (g.float() if accumulate else 0)
                   for g, o in zip(gA, offs)]
            ops.lora_wgrad(u, x, [g.t() for g in gA], offs, [0, 0, 0], s, accumulate)
            for g, g0 in zip(gA, gA0):
                _close(g, g0, dt, 4, name=f"dA acc={accumulate} {gdt}")
    dx_acc = torch.randn(N, K, device=DEV).to(dt)
    dx0 = dx_acc.float() + s * u.float() @ P.float()
    dx = torch.empty(N, K, device=DEV, dtype=dt)
    ops.lora_up_(dx, u, [P], [0], [0], s, base=dx_acc)
    _close(dx, dx0, dt, 2, name="up bwd (rank > 64 in LDS passes)" if R > 64 else "up bwd")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N", [1000, 4096])
def test_kaug_producers_and_blocks(dt, N):
    """Zero-copy K-augmentation pieces: RMSNorm / SwiGLU written into the x part of an
    [N, K + R] buffer (bitwise their contiguous outputs), lora_down into its last R columns,
    and the [out, R] B block of [W | Bd^T] and of the transposed [W^T ; Bd]."""
    K, F, r = 512, 1024, 16
    outs, c0 = [512, 128, 128], [0, 512, 640]
    R = 3 * r
    x = torch.randn(N, K, device=DEV).to(dt)
    w = (1 + 0.1 * torch.randn(K, device=DEV)).to(dt)
    xa = torch.full((N, K + R), float("nan"), device=DEV, dtype=dt)
    y, rstd = ops.rmsnorm_fwd_into(x, w, 1e-5, xa[:, :K])
    y0, rstd0 = ops.rmsnorm_fwd(x, w, 1e-5)
    assert torch.equal(xa[:, :K], y0) and torch.equal(rstd, rstd0) and y.data_ptr() == xa.data_ptr()
    assert torch.isnan(xa[:, K:].float()).all()                        # nothing past the view written
    As = [(0.1 * torch.randn(K, r, device=DEV)).to(dt) for _ in outs]
    P = ops.lora_pack_t(As)
    ops.lora_down_into(xa[:, :K], [P], [0], [K], [0], R, 0.5, xa[:, K:])
    assert torch.equal(xa[:, K:], ops.lora_down(y0, [P], [0], [K], [0], R, 0.5))
    xp = torch.full((N, K + 64), float("nan"), device=DEV, dtype=dt)      # row padded to 128 B lines
    ops.lora_down_into(y0, [P], [0], [K], [0], R, 0.5, xp[:, K:])
    assert torch.equal(xp[:, K:K + R], xa[:, K:]) and (xp[:, K + R:] == 0).all()
    gu = torch.randn(N, 2 * F, device=DEV).to(dt)
    xd = torch.full((N, F + R), float("nan"), device=DEV, dtype=dt)
    ops.swiglu_fwd_into(gu, xd[:, :F])
    assert torch.equal(xd[:, :F], ops.swiglu_fwd(gu)) and torch.isnan(xd[:, F:].float()).all()
    Bs = [torch.randn(r, o, device=DEV).to(dt) for o in outs]
    offs = [0, r, 2 * r]
    M = sum(outs)
    ref_blk = torch.zeros(M, R, device=DEV, dtype=dt)
    for b, c, o in zip(Bs, c0, offs):
        ref_blk[c:c + b.shape[1], o:o + r] = b.t()
    Wa = torch.full((M, K + R), float("nan"), device=DEV, dtype=dt)
    ops.lora_block_(Wa[:, K:], Bs, c0, offs)
    WaT = torch.full((K + R, M), float("nan"), device=DEV, dtype=dt)
    ops.lora_block_(WaT[K:].t(), Bs, c0, offs)
    assert torch.equal(Wa[:, K:], ref_blk) and torch.equal(WaT[K:], ref_blk.t())
    assert torch.isnan(Wa[:, :K].float()).all() and torch.isnan(WaT[:K].float()).all()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N", [1000, 4096])
def test_swiglu_bwd_lowrank(dt, N):
    """SwiGLU backward with dact = base + s u P formed in the kernel (base / u: column slices of
    one K-augmented [dx_W | u | 0] buffer) vs the separate lora_up + swiglu_bwd passes."""
    F, r, Rp = 1024, 16, 64
    gu = torch.randn(N, 2 * F, device=DEV).to(dt)
    dxa = torch.randn(N, F + Rp, device=DEV).to(dt)
    P = (0.1 * torch.randn(r, F, device=DEV)).to(dt)
    base, u = dxa[:, :F], dxa[:, F:F + r]
    got = ops.swiglu_bwd_lowrank(gu, base, u, P, 0.5)
    dact = torch.empty(N, F, device=DEV, dtype=dt)
    ops.lora_up_(dact, u, [P], [0], [0], 0.5, base=base)
    want = ops.swiglu_bwd(gu, dact)
    _close(got, want, dt, 2, name="swiglu_bwd_lowrank")
    ref_dact = (base.float() + 0.5 * u.float() @ P.float()).to(dt)
    _close(got, ops.swiglu_bwd(gu, ref_dact), dt, 2, name="swiglu_bwd_lowrank vs fp32 dact")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,F", [(1000, 1024), (4096, 512), (77, 192)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_swiglu_bwd_lowrank_wgrad(dt, N, F, accumulate):
    """SwiGLU backward of a LoRA MLP with the gate/up dB and the down dA summed in the same pass
    (column-slab MFMA reductions) vs swiglu_bwd_lowrank + the separate lora_wgrad passes: dgu and
    the gradients within one ulp of their dtype; and vs an fp32 matmul oracle."""
    r, Rp = 16, 64
    gu = torch.randn(N, 2 * F, device=DEV).to(dt)
    dxa = torch.randn(N, F + Rp, device=DEV).to(dt)
    P = (0.1 * torch.randn(r, F, device=DEV)).to(dt)
    base, u = dxa[:, :F], dxa[:, F:F + r]
    sta = torch.randn(N, 64 + 32, device=DEV).to(dt)      # [x part | s t (gate 16, up 16)] rows
    st = sta[:, 64:96]
    gdA = torch.randn(F, r, device=DEV).to(dt)
    g0 = [torch.randn(r, F, device=DEV).to(dt), torch.randn(r, F, device=DEV).to(dt), gdA.t()]
    g1 = [g.clone() for g in g0[:2]] + [gdA.clone().t()]
    got = ops.swiglu_bwd_lowrank_wgrad(gu, base, u, P, 0.5, st, g1[0], g1[1], g1[2], accumulate)
    want = ops.swiglu_bwd_lowrank(gu, base, u, P, 0.5)
    _ulps(got, want, dt, 1, name="dgu")   # same math; hipcc may contract differently per kernel
    g2 = [g.clone() for g in g0[:2]] + [gdA.clone().t()]
    ops.lora_wgrad(st, want, [g2[0], g2[1]], [0, 16], [0, F], 1.0, accumulate)
    act = ops.swiglu_fwd(gu)
    ops.lora_wgrad(u, act, [g2[2]], [0], [0], 0.5, accumulate)
    for a, b, name in zip(g1, g2, ("dB gate", "dB up", "dA down")):
        _ulps(a, b, dt, 1, name=name)
    # fp32 oracle of the three reductions over the kernel's own (rounded) dg / du and act
    F_ = F
    for a, L, R, sc, g in ((g1[0], st[:, :16], want[:, :F_], 1.0, g0[0]), (g1[1], st[:, 16:], want[:, F_:], 1.0, g0[1]),
                           (g1[2], u, act, 0.5, g0[2])):
        ref32 = sc * (L.float().t() @ R.float()) + (g.float() if accumulate else 0)
        _close(a, ref32.cpu(), dt, 4, name="vs fp32")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("R,V", [(4096, 128256), (1000, 640), (77, 1088), (300, 2048)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_lora_head_bwd(dt, R, V, accumulate):
    """The LoRA head's u = dl B^T and dB (+)= st^T dl from one pass over dl (column-slab MFMA
    tiles, fixed-order partial sums) vs an fp32 matmul oracle; ragged rows and a partial last
    column slab (V not a multiple of 1,024) included; gB as a transposed view; deterministic."""
    r = 16
    dl = (0.01 * torch.randn(R, V, device=DEV)).to(dt)
    sta = torch.randn(R, 4160, device=DEV).to(dt)           # s t as a column view of a wider row
    st = sta[:, 4096:4096 + r]
    B = (0.1 * torch.randn(r, V, device=DEV)).to(dt)
    g0 = torch.randn(V, r, device=DEV)                       # fp32 [V, 16], passed as its [16, V] view
    gB = g0.clone().t()
    u = torch.empty(R, r, dtype=dt, device=DEV)
    ops.lora_head_bwd_(dl, st, B, u, gB, accumulate)
    _close(u, (dl.float() @ B.float().t()).cpu(), dt, 4, name="u")
    ref = st.float().t() @ dl.float() + (g0.t() if accumulate else 0)
    check_elem(gB, ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item(), name="gB")
    u2, gB2 = torch.empty_like(u), g0.clone().t()
    ops.lora_head_bwd_(dl, st, B, u2, gB2, accumulate)
    assert torch.equal(u, u2) and torch.equal(gB, gB2)


def test_lora_model_uses_kernels_and_matches_gemm_path(monkeypatch):
    """A LoRA Llama step on the fused kernels (K-augmented QKV / gate-up / down, grouped o, the
    fused LoRA head: V = 512) gives the same loss / LoRA grads as the per-member hipBLASLt path."""
    from building_llm_from_scratch_amd.config import get_config
    from building_llm_from_scratch_amd.models import build_model, replace_linear_with_lora
    from building_llm_from_scratch_amd.models import linear
    cfg = get_config("llama3_2", "1B").replace(context_length=128, emb_dim=256, n_heads=4, n_kv_groups=2,
                                               hidden_dim=512, n_layers=2, vocab_size=512, dtype=torch.bfloat16)
    grads = []
    calls = []
    orig = ops.lora_down
    monkeypatch.setattr(ops, "lora_down", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    for use_kernels in (True, False):
        torch.manual_seed(0)
        m = build_model(cfg, device=DEV)
        for p in m.parameters():
            p.requires_grad = False
        replace_linear_with_lora(m, rank=16, alpha=32)
        for mod in m.modules():
            if hasattr(mod, "B") and isinstance(mod.B, torch.nn.Parameter):
                torch.nn.init.normal_(mod.B, std=0.05)
        m.flatten(device=DEV)
        monkeypatch.setattr(ops, "lora_kernel_ok", (lambda *a: True) if use_kernels else (lambda *a: False))
        if not use_kernels:   # also the zero-copy K-augmented groups and the fused LoRA head
            monkeypatch.setattr(ops, "lora_kernel_ok_dims", lambda *a: False)
        idx = torch.randint(0, cfg.vocab_size, (2, 128), device=DEV, generator=torch.Generator(DEV).manual_seed(1))
        loss = m(idx, idx)
        loss.backward()
        grads.append((loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters() if p.requires_grad}))
    assert calls, "fused LoRA kernels were not used"
    (la, ga), (lb, gb) = grads
    assert abs(la - lb) < 2e-2
    for k in ga:
        err = (ga[k] - gb[k]).abs().max().item()
        assert err <= 3e-2 * max(gb[k].abs().max().item(), 1e-3), (k, err)


@pytest.mark.parametrize("gdt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("accumulate", [False, True])
def test_split_k_weight_grad(gdt, accumulate):
    """Split-K dW (batched GEMM partials + sum_partials_ kernel) vs an fp32 matmul."""
    from building_llm_from_scratch_amd.models.linear import _weight_grad, weight_grad_splits
    N, out_f, in_f = 8192, 1280, 768
    assert weight_grad_splits(N, out_f, in_f) > 1
    dy = torch.randn(N, out_f, device=DEV).to(torch.bfloat16)
    x = torch.randn(N, in_f, device=DEV).to(torch.bfloat16)
    gW = torch.randn(out_f, in_f, device=DEV).to(gdt)
    expect = dy.float().t() @ x.float() + (gW.float() if accumulate else 0)
    _weight_grad(dy, x, gW, accumulate)
    _close(gW, expect, torch.bfloat16, 2, name="split-K dW")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("K,M,N,S", [(128, 256, 256, 1), (384, 512, 768, 1), (2048, 768, 512, 3), (1024, 256, 1024, 2),
                                     (1024, 256, 512, 8)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_wgrad_gemm(dt, odt, K, M, N, S, accumulate):
    """Token-major MFMA dW kernel c (+)= a^T b (strided a, split-K) vs an fp32 matmul: the 4-wave
    schedule (S < 8) and the 8-wave one (deep split-K, S = 8)."""
    a_full = torch.randn(K, M + 64, device=DEV).to(dt)
    a = a_full[:, 32:32 + M]                      # lda = M + 64, 64-B offset
    b = torch.randn(K, N, device=DEV).to(dt)
    c = torch.randn(M, N, device=DEV).to(odt)
    assert ops.wgrad_gemm_ok(a, b, c)
    expect = a.float().t() @ b.float() + (c.float() if accumulate else 0)
    ops.wgrad_gemm_(a, b, c, accumulate, S)
    check_close(c, expect, odt, k=3.0, name="wgrad")


@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K,full,St", [(768, 512, 1024, 4, 2), (768, 512, 1536, 2, 3), (512, 1280, 2048, 8, 2),
                                           (1536, 256, 1024, 3, 4)])
@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("wmap", ["0", "2"])
def test_wgrad_gemm_split_tail(odt, M, N, K, full, St, accumulate, wmap, request):
    """dW with the grouped tile order in two launches -- tiles [0, full) whole-K into c, the rest
    split St ways into compact fp32 partials and summed -- vs an fp32 matmul (both tile maps: the
    sum kernel must place every tail tile where the GEMM's map put it)."""
    torch.ops.bllm.set_gemm_tile_maps(int(wmap), 0, 0, 0)
    request.addfinalizer(lambda: torch.ops.bllm.set_gemm_tile_maps(0, 0, 0, 0))
    a_full = torch.randn(K, M + 64, device=DEV).to(torch.bfloat16)
    a = a_full[:, 32:32 + M]
    b = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    c = torch.randn(M, N, device=DEV).to(odt)
    expect = a.float().t() @ b.float() + (c.float() if accumulate else 0)
    torch.ops.bllm.wgrad_gemm_tail_(a, b, c, accumulate, full, St)
    check_close(c, expect, odt, k=3.0, name="wgrad split tail")


def test_wgrad_plan_routes_headline_tails():
    """The planner keeps whole-K waves and splits only the ragged tail of the Llama-3-8B QKV / down
    weight gradients; the library shapes that fill whole waves stay unsplit."""
    assert ops.wgrad_plan(4096, 14336, 40960) == ("tail", 768, 2)
    assert ops.wgrad_plan(6144, 4096, 40960) == ("tail", 256, 2)
    assert ops.wgrad_plan(28672, 4096, 40960) == ("split", 1)
    assert ops.wgrad_plan(4096, 4096, 40960) == ("split", 1)
    assert ops.wgrad_plan(1280, 1280, 65536)[0] == "split"     # GPT-2: no whole wave to keep


def test_wgrad_gemm_in_weight_grad_path():
    """_weight_grad routes eligible dW through the MFMA kernel; result == hipBLASLt path."""
    from building_llm_from_scratch_amd.models.linear import _weight_grad
    N, out_f, in_f = 4096, 1536, 1024
    dy = torch.randn(N, out_f, device=DEV).to(torch.bfloat16)
    x = torch.randn(N, in_f, device=DEV).to(torch.bfloat16)
    g1 = torch.empty(out_f, in_f, device=DEV, dtype=torch.bfloat16)
    _weight_grad(dy, x, g1, False)
    g0 = (x.float().t() @ dy.float()).t()
    _close(g1, g0, torch.bfloat16, 1, name="dW")


@pytest.mark.parametrize("accumulate", [False, True])
def test_wgrad_gemm_unaligned_output(accumulate):
    """An output view that is not 16-B aligned takes the element-store epilogue."""
    K, M, N = 256, 256, 512
    a = torch.randn(K, M, device=DEV).to(torch.bfloat16)
    b = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    c_full = torch.randn(M, N + 8, device=DEV).to(torch.bfloat16)
    c = c_full[:, 1:1 + N]                         # 2-B offset, row stride N + 8
    assert c.data_ptr() % 16 != 0 and ops.wgrad_gemm_ok(a, b, c)
    before = c_full.clone()
    expect = a.float().t() @ b.float() + (c.float() if accumulate else 0)
    ops.wgrad_gemm_(a, b, c, accumulate, 1)
    check_close(c, expect, torch.bfloat16, k=3.0, name="wgrad unaligned")
    assert torch.equal(c_full[:, 0], before[:, 0]) and torch.equal(c_full[:, 1 + N:], before[:, 1 + N:])


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("odt", [None, torch.float32])
@pytest.mark.parametrize("M,K,N", [(256, 128, 256), (512, 384, 768), (768, 1024, 512), (1024, 4096, 1536)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_nt(dt, odt, M, K, N, accumulate):
    """Both-operands-K-contiguous GEMM (c = a . b^T, the forward layout) on the persistent kernel
    of csrc/gemm_nt.hip vs an fp32 matmul, strided rows."""
    a_full = torch.randn(M, K + 64, device=DEV).to(dt)
    a = a_full[:, 32:32 + K]
    b_full = torch.randn(N, K + 32, device=DEV).to(dt)
    b = b_full[:, :K]
    c = torch.randn(M, N, device=DEV).to(odt or dt)
    expect = a.float() @ b.float().t() + (c.float() if accumulate else 0)
    ops.gemm_nt_(a, b, c, accumulate)
    check_close(c, expect, odt or dt, k=3.0, name="gemm_nt")


@pytest.mark.parametrize("odt", [None, torch.float32])
@pytest.mark.parametrize("M,K,N", [(8192, 256, 4096), (4352, 128, 4096), (2048, 512, 33 * 256)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_nt_persistent_multi_tile(odt, M, K, N, accumulate):
    """Persistent kernel with more output tiles than workgroups (each workgroup walks several
    tiles, the K-tile stream running across tile boundaries; uneven tile counts per workgroup) vs
    an fp32 matmul, strided A rows."""
    dt = torch.bfloat16
    a_full = torch.randn(M, K + 64, device=DEV).to(dt)
    a = a_full[:, 32:32 + K]
    b = torch.randn(N, K, device=DEV).to(dt)
    c = torch.randn(M, N, device=DEV).to(odt or dt)
    expect = a.float() @ b.float().t() + (c.float() if accumulate else 0)
    ops.gemm_nt_(a, b, c, accumulate)
    check_close(c, expect, odt or dt, k=3.0, name="gemm_nt persistent")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("odt", [None, torch.float32])
@pytest.mark.parametrize("M,K,N", [(256, 128, 256), (512, 384, 768), (768, 1024, 512)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_nn(dt, odt, M, K, N, accumulate):
    """K-contiguous-A variant of the MFMA GEMM (dX = dY W) vs an fp32 matmul, strided A rows."""
    a_full = torch.randn(M, K + 64, device=DEV).to(dt)
    a = a_full[:, 32:32 + K]                      # lda = K + 64, 64-B offset
    b = torch.randn(K, N, device=DEV).to(dt)
    c = torch.randn(M, N, device=DEV).to(odt or dt)
    assert ops.gemm_nn_ok(a, b, c)
    expect = a.float() @ b.float() + (c.float() if accumulate else 0)
    ops.gemm_nn_(a, b, c, accumulate)
    check_close(c, expect, c.dtype, k=3.0, name="gemm_nn")


def test_dgrad_in_linear_backward(monkeypatch):
    """With ops.DGRAD_GEMM on, FusedLinear.backward routes dX through the MFMA kernel."""
    from building_llm_from_scratch_amd.models.linear import _input_grad
    monkeypatch.setattr(ops, "DGRAD_GEMM", True)
    dy = torch.randn(512, 768, device=DEV).to(torch.bfloat16)
    W = torch.randn(768, 1280, device=DEV).to(torch.bfloat16)
    assert ops.gemm_nn_ok(dy, W)
    dx = _input_grad(dy, W)
    _close(dx, dy.float() @ W.float(), torch.bfloat16, 1, name="dX")
    acc = torch.randn(512, 1280, device=DEV).to(torch.bfloat16)
    dx2 = _input_grad(dy, W, acc)
    _close(dx2, acc.float() + dy.float() @ W.float(), torch.bfloat16, 1, name="dX+acc")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("R,C", [(64, 64), (8, 16), (200, 136), (4096, 1032), (6144, 4096)])
def test_transpose2d(dt, R, C):
    a = torch.randn(R, C, device=DEV).to(dt)
    t = ops.transpose2d(a)
    assert t.shape == (C, R) and t.is_contiguous()
    assert torch.equal(t, a.t().contiguous())


def test_dgrad_transposed_weight_path(monkeypatch):
    """Above DGRAD_WT_MIN_TOKENS the input gradient runs on a transposed weight copy."""
    from building_llm_from_scratch_amd.models import linear
    monkeypatch.setattr(ops, "DGRAD_GEMM", False)
    monkeypatch.setattr(linear, "DGRAD_WT_MIN_TOKENS", 256)
    calls = []
    orig = ops.transpose2d
    monkeypatch.setattr(ops, "transpose2d", lambda w: calls.append(w.shape) or orig(w))
    dy = torch.randn(512, 768, device=DEV).to(torch.bfloat16)
    W = torch.randn(768, 1280, device=DEV).to(torch.bfloat16)
    assert linear._dgrad_wt_ok(dy, W)
    dx = linear._input_grad(dy, W)
    _close(dx, dy.float() @ W.float(), torch.bfloat16, 1, name="dX")
    acc = torch.randn(512, 1280, device=DEV).to(torch.bfloat16)
    _close(linear._input_grad(dy, W, acc), acc.float() + dy.float() @ W.float(), torch.bfloat16, 1, name="dX+acc")
    out = acc.clone()
    linear._input_grad(dy, W, out=out)
    _close(out, acc.float() + dy.float() @ W.float(), torch.bfloat16, 1, name="out+=dX")
    assert len(calls) == 3


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,K,O", [(33, 64, 40), (256, 512, 768), (1024, 4096, 4096)])
def test_linear_residual_hipblaslt(dt, N, K, O):
    """C + x W^T on hipBLASLt with C != D (csrc/binding.cpp linear_residual) vs fp32 torch."""
    x = torch.randn(N, K, device=DEV).to(dt)
    W = (torch.randn(O, K, device=DEV) / K ** 0.5).to(dt)
    C = torch.randn(N, O, device=DEV).to(dt)
    C0 = C.clone()
    y = torch.ops.bllm.linear_residual(x, W, C)
    assert y.data_ptr() != C.data_ptr()
    assert torch.equal(C, C0), "residual input must not be modified"
    want = C.float().cpu() + x.float().cpu() @ W.float().cpu().t()
    _close(y, want, dt, 2, name="linear_residual")
    assert torch.equal(ops.linear_residual(x, W, C), y)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,K,N", [(512, 256, 1024), (8192, 1280, 5120), (4096, 384, 768)])
def test_gemm_nt_bias_gelu(dt, M, K, N):
    """GPT-2 c_fc with bias + exact GELU in the persistent GEMM's epilogue (K9): f against the fp32
    oracle, g bitwise equal to the separate gelu_fwd kernel applied to that f."""
    a = torch.randn(M, K, device=DEV).to(dt)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(dt)
    bias = torch.randn(N, device=DEV).to(dt)
    assert ops.gemm_nt_bias_gelu_ok(a, w, bias)
    f, g = ops.gemm_nt_bias_gelu(a, w, bias)
    check_close(f, a.float() @ w.float().t() + bias.float(), dt, k=3.0, name="gemm_nt_bias_gelu f")
    assert torch.equal(g, ops.gelu_fwd(f))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,K,T,H,G", [(512, 256, 256, 4, 2), (2048, 512, 1024, 32, 8), (8192, 128, 1024, 16, 8)])
def test_gemm_nt_rope(dt, M, K, T, H, G):
    """QKV projection with RoPE in the persistent GEMM's epilogue (K4) against the same GEMM
    followed by the separate rope_ pass — equal to 1 ulp (same rounding
    points; the fp32 rotation may contract differently) — and against the fp32 oracle."""
    hd = 128
    N = (H + 2 * G) * hd
    a = torch.randn(M, K, device=DEV).to(dt)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(dt)
    cos, sin = ops.rope_tables(hd, T, 500000.0, None, device=DEV)
    assert ops.gemm_nt_rope_ok(a, w, hd)
    got = ops.gemm_nt_rope(a, w, cos, sin, T, H, G, hd)
    sep = torch.empty(M, N, device=DEV, dtype=dt)
    ops.gemm_nt_(a, w, sep, False)
    ops.rope_(sep, cos, sin, T, H, G, hd)
    ulp = (got.float() - sep.float()).abs() / sep.float().abs().clamp_min(1e-3)
    assert (ulp <= (2 ** -7 if dt == torch.bfloat16 else 2 ** -10)).all(), ulp.max().item()
    assert torch.equal(got[:, (H + G) * hd:], sep[:, (H + G) * hd:])      # v heads untouched
    oracle = ref.rope_((a.float() @ w.float().t()).to(dt), cos, sin, T, H, G, hd)
    check_close(got, oracle.float(), dt, k=4.0, name="gemm_nt_rope")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,K,F", [(256, 128, 128), (512, 512, 768), (1024, 4096, 1792), (4096, 256, 4096)])
def test_gemm_nt_swiglu(dt, M, K, F):
    """Gate/up GEMM with the SwiGLU forward in the epilogue (K10): gu against the fp32 oracle, act
    bitwise equal to the separate swiglu_fwd kernel applied to that gu."""
    a = torch.randn(M, K, device=DEV).to(dt)
    w = (torch.randn(2 * F, K, device=DEV) / K ** 0.5).to(dt)
    assert ops.gemm_nt_swiglu_ok(a, w)
    gu, act = ops.gemm_nt_swiglu(a, w)
    check_close(gu, a.float() @ w.float().t(), dt, k=3.0, name="gemm_nt_swiglu gu")
    assert torch.equal(act, ops.swiglu_fwd(gu))
    check_close(act, ref.swiglu_fwd(a.float() @ w.float().t()), dt, k=5.0, name="gemm_nt_swiglu act")
