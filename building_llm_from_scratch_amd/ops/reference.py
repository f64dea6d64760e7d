"""Plain-PyTorch implementations of every fused op.

These define the numerical contract of the HIP kernels in ``csrc/`` (same signatures, fp32
internal math) and are the execution path for CPU tensors (unit tests, gloo multi-process
tests, the BASELINE config #1 CPU run).  GPU tensors never reach this module: the
dispatchers in ``ops/__init__.py`` route them to the compiled extension and fail loudly if
it is missing.

Reference ops these replace (all eager PyTorch in the reference):
  RMSNorm   Models/Llama/common_components.py:54-70
  LayerNorm Models/GPT2/GPT2.py:79-80 (nn.LayerNorm)
  RoPE      common_components.py:6-35 (rotate-half)
  attention GPT2.py:38-46, Llama3.py:131-155 (materialised [B,H,T,T] scores + softmax)
  SwiGLU    common_components.py:110-124;  GELU(erf) GPT2.py:58-62
  CE        train.py:88-92 (F.cross_entropy, ignore_index=-100)
  AdamW     torch.optim.AdamW(lr, wd=0.1) build_components.py:250-258
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

# ---------------------------------------------------------------------------
# counter-based dropout RNG (identical bit-for-bit to csrc/common.h::drop_bits16):
# one 32-bit hash per PAIR of element indices, 16 bits per element, 16-bit threshold
# ---------------------------------------------------------------------------
_M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 integer hash on int64 tensors holding uint32 values."""
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    x = x ^ (x >> 16)
    return x


def drop_threshold16(p: float) -> int:
    return min(int(p * 65536.0), 65536)


def drop_inv_keep(p: float) -> float:
    """Scale of kept elements: 1 / P(keep) for the quantised 16-bit threshold."""
    t = drop_threshold16(p)
    return 0.0 if t >= 65536 else 65536.0 / (65536.0 - t)


def drop_keep_mask(seed: int, offset: int, numel: int, p: float, device=None) -> torch.Tensor:
    """keep[i] = bits16(seed, offset + i) >= p * 2^16."""
    idx = torch.arange(numel, dtype=torch.int64, device=device) + offset
    pair = idx >> 1
    s = _mix32(torch.full_like(pair, seed & _M32) + ((pair >> 32) * 0x9E3779B9 & _M32))
    h = _mix32((pair & _M32) ^ s)
    bits = torch.where((idx & 1) == 1, h >> 16, h & 0xFFFF)
    return bits >= drop_threshold16(p)


# ---------------------------------------------------------------------------
# norms
# ---------------------------------------------------------------------------
def rmsnorm_fwd(x: torch.Tensor, w: torch.Tensor, eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    xf = x.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1) + eps)
    y = (xf * rstd[:, None] * w.float()).to(x.dtype)
    return y, rstd


def rmsnorm_bwd(dy, x, w, rstd, dx_acc: Optional[torch.Tensor] = None):
    xf, dyf, wf = x.float(), dy.float(), w.float()
    xhat = xf * rstd[:, None]
    dw = (dyf * xhat).sum(0)
    g = dyf * wf
    d = x.shape[-1]
    dx = rstd[:, None] * (g - xhat * (g * xhat).sum(-1, keepdim=True) / d)
    if dx_acc is not None:
        dx = dx + dx_acc.float()
    return dx.to(x.dtype), dw


def layernorm_fwd(x, w, b, eps: float):
    xf = x.float()
    mean = xf.mean(-1)
    var = (xf - mean[:, None]).pow(2).mean(-1)
    rstd = torch.rsqrt(var + eps)
    y = ((xf - mean[:, None]) * rstd[:, None] * w.float() + b.float()).to(x.dtype)
    return y, mean, rstd


def layernorm_bwd(dy, x, w, mean, rstd, dx_acc: Optional[torch.Tensor] = None):
    xf, dyf, wf = x.float(), dy.float(), w.float()
    xhat = (xf - mean[:, None]) * rstd[:, None]
    dw = (dyf * xhat).sum(0)
    db = dyf.sum(0)
    g = dyf * wf
    d = x.shape[-1]
    dx = rstd[:, None] * (g - g.mean(-1, keepdim=True) - xhat * (g * xhat).sum(-1, keepdim=True) / d)
    if dx_acc is not None:
        dx = dx + dx_acc.float()
    return dx.to(x.dtype), dw, db


def dropout_add(x, a, p: float, seed: int, offset: int):
    """x + dropout(a)."""
    if p <= 0.0:
        return (x.float() + a.float()).to(x.dtype)
    keep = drop_keep_mask(seed, offset, a.numel(), p, a.device).view_as(a)
    return (x.float() + a.float() * keep * drop_inv_keep(p)).to(x.dtype)


def dropout_bwd(dy, p: float, seed: int, offset: int):
    if p <= 0.0:
        return dy
    keep = drop_keep_mask(seed, offset, dy.numel(), p, dy.device).view_as(dy)
    return (dy.float() * keep * drop_inv_keep(p)).to(dy.dtype)


# ---------------------------------------------------------------------------
# RoPE (rotate-half, non-interleaved) on the packed qkv buffer [N, (H+2G)*hd]
# ---------------------------------------------------------------------------
def rope_tables(head_dim: int, context_length: int, theta_base: float, freq_config=None,
                device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 cos/sin [T, hd/2] (reference Llama3.py:74-104 incl. 3.1 smoothing)."""
    inv_freq = 1.0 / (theta_base ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if freq_config is not None:
        fc = freq_config if isinstance(freq_config, dict) else freq_config.to_dict()
        low_wl = fc["original_context_length"] / fc["low_freq_factor"]
        high_wl = fc["original_context_length"] / fc["high_freq_factor"]
        wavelen = 2 * math.pi / inv_freq
        adj = torch.where(wavelen > low_wl, inv_freq / fc["factor"], inv_freq)
        smooth = (fc["original_context_length"] / wavelen - fc["low_freq_factor"]) / (
            fc["high_freq_factor"] - fc["low_freq_factor"])
        smoothed = (1 - smooth) * (inv_freq / fc["factor"]) + smooth * inv_freq
        med = (wavelen <= low_wl) & (wavelen >= high_wl)
        inv_freq = torch.where(med, smoothed, adj)
    pos = torch.arange(context_length, dtype=torch.float64)
    ang = pos[:, None] * inv_freq[None, :]
    return torch.cos(ang).float().to(device), torch.sin(ang).float().to(device)


def rope_(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, T: int, n_heads: int,
          n_kv: int, head_dim: int, inverse: bool = False, pos_offset: int = 0) -> torch.Tensor:
    """In-place RoPE on the q and k heads of qkv [N, (H+2G)*hd]; row r has position
    (r % T) + pos_offset.  ``inverse`` applies the transpose rotation (backward)."""
    N = qkv.shape[0]
    half = head_dim // 2
    v = qkv.view(N, n_heads + 2 * n_kv, head_dim)
    qk = v[:, :n_heads + n_kv, :].float()
    pos = (torch.arange(N, device=qkv.device) % T) + pos_offset
    c = cos[pos][:, None, :]
    s = sin[pos][:, None, :]
    if inverse:
        s = -s
    x1, x2 = qk[..., :half], qk[..., half:]
    out = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)
    v[:, :n_heads + n_kv, :] = out.to(qkv.dtype)
    return qkv


# ---------------------------------------------------------------------------
# attention on the packed qkv buffer
# ---------------------------------------------------------------------------
def _split_qkv(qkv, B, T, H, G, hd):
    v = qkv.view(B, T, H + 2 * G, hd)
    q = v[:, :, :H].permute(0, 2, 1, 3).float()
    k = v[:, :, H:H + G].permute(0, 2, 1, 3).float()
    vv = v[:, :, H + G:].permute(0, 2, 1, 3).float()
    return q, k, vv


def _attn_dropout_keep(B, H, T, p, seed, offset, device):
    return drop_keep_mask(seed, offset, B * H * T * T, p, device).view(B, H, T, T)


def flash_attn_fwd(qkv, B: int, T: int, H: int, G: int, hd: int, causal: bool = True,
                   dropout_p: float = 0.0, seed: int = 0, offset: int = 0):
    """Returns o [B*T, H*hd] (qkv dtype) and lse [B, H, T] fp32 in log2 units of the
    *scaled* scores (lse2 = log2 sum_k exp2(s_k * scale * log2e))."""
    q, k, v = _split_qkv(qkv, B, T, H, G, hd)
    rep = H // G
    k = k.repeat_interleave(rep, dim=1)
    v = v.repeat_interleave(rep, dim=1)
    scale = 1.0 / math.sqrt(hd)
    s = (q @ k.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(T, T, dtype=torch.bool, device=qkv.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.exp(s - lse[..., None])
    if dropout_p > 0.0:
        keep = _attn_dropout_keep(B, H, T, dropout_p, seed, offset, qkv.device)
        p = p * keep * drop_inv_keep(dropout_p)
    o = (p @ v).permute(0, 2, 1, 3).reshape(B * T, H * hd).to(qkv.dtype)
    return o, lse * (1.0 / math.log(2.0))


def flash_attn_bwd(qkv, o, lse2, do, B: int, T: int, H: int, G: int, hd: int, causal: bool = True,
                   dropout_p: float = 0.0, seed: int = 0, offset: int = 0):
    """Returns dqkv [B*T, (H+2G)*hd] (qkv dtype); P is recomputed from lse."""
    q, k, v = _split_qkv(qkv, B, T, H, G, hd)
    rep = H // G
    kx = k.repeat_interleave(rep, dim=1)
    vx = v.repeat_interleave(rep, dim=1)
    scale = 1.0 / math.sqrt(hd)
    s = (q @ kx.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(T, T, dtype=torch.bool, device=qkv.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.exp(s - (lse2 * math.log(2.0))[..., None])
    dO = do.view(B, T, H, hd).permute(0, 2, 1, 3).float()
    O = o.view(B, T, H, hd).permute(0, 2, 1, 3).float()
    if dropout_p > 0.0:
        keep = _attn_dropout_keep(B, H, T, dropout_p, seed, offset, qkv.device)
        pd = p * keep * drop_inv_keep(dropout_p)
    else:
        keep = None
        pd = p
    dv = pd.transpose(-1, -2) @ dO
    dpd = dO @ vx.transpose(-1, -2)
    dp = dpd * keep * drop_inv_keep(dropout_p) if keep is not None else dpd
    delta = (dO * O).sum(-1, keepdim=True)          # = rowsum(P * dP) incl. dropout
    ds = p * (dp - delta) * scale
    dq = ds @ kx
    dk = ds.transpose(-1, -2) @ q
    dk = dk.view(B, G, rep, T, hd).sum(2)
    dv = dv.view(B, G, rep, T, hd).sum(2)
    out = torch.empty(B, T, H + 2 * G, hd, dtype=qkv.dtype, device=qkv.device)
    out[:, :, :H] = dq.permute(0, 2, 1, 3).to(qkv.dtype)
    out[:, :, H:H + G] = dk.permute(0, 2, 1, 3).to(qkv.dtype)
    out[:, :, H + G:] = dv.permute(0, 2, 1, 3).to(qkv.dtype)
    return out.view(B * T, (H + 2 * G) * hd)


# ---------------------------------------------------------------------------
# activations
# ---------------------------------------------------------------------------
def swiglu_fwd(gu: torch.Tensor) -> torch.Tensor:
    F = gu.shape[-1] // 2
    g, u = gu[:, :F].float(), gu[:, F:].float()
    return (g * torch.sigmoid(g) * u).to(gu.dtype)


def swiglu_bwd(gu: torch.Tensor, dact: torch.Tensor) -> torch.Tensor:
    F = gu.shape[-1] // 2
    g, u, d = gu[:, :F].float(), gu[:, F:].float(), dact.float()
    sg = torch.sigmoid(g)
    silu = g * sg
    dg = d * u * (sg * (1 + g * (1 - sg)))
    du = d * silu
    return torch.cat([dg, du], dim=-1).to(gu.dtype)


def gelu_fwd(f: torch.Tensor) -> torch.Tensor:
    x = f.float()
    return (0.5 * x * (1.0 + torch.erf(x * 0.7071067811865476))).to(f.dtype)


def gelu_bwd(f: torch.Tensor, dg: torch.Tensor) -> torch.Tensor:
    x = f.float()
    cdf = 0.5 * (1.0 + torch.erf(x * 0.7071067811865476))
    pdf = torch.exp(-0.5 * x * x) * 0.3989422804014327
    return (dg.float() * (cdf + x * pdf)).to(f.dtype)


# ---------------------------------------------------------------------------
# cross entropy over [N, V] logits (mean over targets != ignore_index)
# ---------------------------------------------------------------------------
def ce_fwd(logits: torch.Tensor, targets: torch.Tensor, ignore_index: int = -100):
    """Returns per-row loss [N] fp32 (0 for ignored rows) and lse [N] fp32 (natural log)."""
    lf = logits.float()
    lse = torch.logsumexp(lf, dim=-1)
    valid = targets != ignore_index
    t = torch.where(valid, targets, torch.zeros_like(targets))
    tgt = lf.gather(1, t[:, None]).squeeze(1)
    loss = torch.where(valid, lse - tgt, torch.zeros_like(lse))
    return loss, lse


def ce_bwd_(logits: torch.Tensor, targets: torch.Tensor, lse: torch.Tensor, scale: torch.Tensor,
            ignore_index: int = -100) -> torch.Tensor:
    """In place: logits <- (softmax(logits) - onehot(target)) * scale, rows with an ignored
    target set to 0.  ``scale`` is a 1-element fp32 tensor (dloss / n_valid)."""
    lf = logits.float()
    p = torch.exp(lf - lse[:, None])
    valid = targets != ignore_index
    t = torch.where(valid, targets, torch.zeros_like(targets))
    p[torch.arange(p.shape[0], device=p.device), t] -= 1.0
    p = p * valid[:, None].float() * scale.float()
    logits.copy_(p.to(logits.dtype))
    return logits


# ---------------------------------------------------------------------------
# embedding
# ---------------------------------------------------------------------------
def embedding_fwd(idx: torch.Tensor, wte: torch.Tensor, wpe: Optional[torch.Tensor], T: int,
                  dropout_p: float = 0.0, seed: int = 0, offset: int = 0) -> torch.Tensor:
    x = wte.index_select(0, idx.reshape(-1))
    if wpe is not None:
        pos = torch.arange(idx.numel(), device=idx.device) % T
        x = (x.float() + wpe.index_select(0, pos).float()).to(wte.dtype)
    if dropout_p > 0.0:
        keep = drop_keep_mask(seed, offset, x.numel(), dropout_p, x.device).view_as(x)
        x = (x.float() * keep * drop_inv_keep(dropout_p)).to(x.dtype)
    return x


def embedding_bwd(idx, dx, grad_wte: Optional[torch.Tensor], grad_wpe: Optional[torch.Tensor], T: int,
                  accumulate: bool = False):
    """grad_wte[idx[n]] += dx[n]; grad_wpe[n % T] += dx[n] (fp32 sums, written in grad dtype)."""
    flat = idx.reshape(-1)
    if grad_wte is not None:
        acc = torch.zeros(grad_wte.shape, dtype=torch.float32, device=dx.device)
        acc.index_add_(0, flat, dx.float())
        if accumulate:
            acc += grad_wte.float()
        grad_wte.copy_(acc.to(grad_wte.dtype))
    if grad_wpe is not None:
        pos = torch.arange(flat.numel(), device=dx.device) % T
        acc = torch.zeros(grad_wpe.shape, dtype=torch.float32, device=dx.device)
        acc.index_add_(0, pos, dx.float())
        if accumulate:
            acc += grad_wpe.float()
        grad_wpe.copy_(acc.to(grad_wpe.dtype))


# ---------------------------------------------------------------------------
# optimizer
# ---------------------------------------------------------------------------
def sq_norm(t: torch.Tensor) -> torch.Tensor:
    return t.float().pow(2).sum()


def adamw_step_(param: torch.Tensor, master: Optional[torch.Tensor], grad: torch.Tensor,
                exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, lr: float, beta1: float, beta2: float,
                eps: float, weight_decay: float, step: int, grad_scale: Optional[torch.Tensor] = None):
    """torch.optim.AdamW semantics (decoupled wd, bias correction) on one flat buffer.
    ``grad_scale`` (1-element fp32 tensor) multiplies the gradient first (clip coef and/or
    fp16 loss-scale inverse).  ``master`` is the fp32 copy when ``param`` is low precision."""
    p32 = master if master is not None else param
    g = grad.float()
    if grad_scale is not None:
        g = g * grad_scale.float()
    p32.mul_(1.0 - lr * weight_decay)
    exp_avg.mul_(beta1).add_(g, alpha=1 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
    p32.addcdiv_(exp_avg, denom, value=-lr / bc1)
    if master is not None:
        param.copy_(master.to(param.dtype))


def attn_decode(q, kcache, vcache, L: int):
    """Reference for the KV-cache decode kernel: q [B,H,hd], cache [B,G,Tmax,hd] -> [B,H*hd]."""
    B, H, hd = q.shape
    G = kcache.shape[1]
    k = kcache[:, :, :L].float().repeat_interleave(H // G, dim=1)   # [B,H,L,hd]
    v = vcache[:, :, :L].float().repeat_interleave(H // G, dim=1)
    s = torch.einsum("bhd,bhld->bhl", q.float(), k) / math.sqrt(hd)
    p = torch.softmax(s, dim=-1)
    return torch.einsum("bhl,bhld->bhd", p, v).reshape(B, H * hd).to(q.dtype)


# ------------------------------------------------------------------ LoRA (csrc/lora.hip oracle)
def lora_down(x, ws, c0, lens, ocol, R: int, scale: float = 1.0):
    """out[:, ocol_i : ocol_i + r_i] = scale * x[:, c0_i : c0_i + len_i] @ w_i[:, :len_i]^T"""
    out = torch.zeros(x.shape[0], R, dtype=torch.float32, device=x.device)
    for w, c, n, o in zip(ws, c0, lens, ocol):
        out[:, o:o + w.shape[0]] = x[:, c:c + n].float() @ w[:, :n].float().t()
    return (out * scale).to(x.dtype)


def lora_up_(y, t, us, c0, toff, scale: float, base=None, bias=None):
    """y[:, c0_i : c0_i + len_i] = base + bias + scale * t[:, toff_i : toff_i + r_i] @ u_i
    (u_i [r_i, len_i]; base / bias optional)"""
    for u, c, o in zip(us, c0, toff):
        r, n = u.shape
        v = scale * (t[:, o:o + r].float() @ u.float())
        if base is not None:
            v = v + base[:, c:c + n].float()
        if bias is not None:
            v = v + bias[c:c + n].float()
        y[:, c:c + n] = v.to(y.dtype)
    return y


def lora_wgrad(p, q, gs, pa, qb, scale: float, accumulate: bool):
    """g_i[a][b] (+)= scale * sum_n p[n][pa_i + a] q[n][qb_i + b]  (g_i [r_i, len_i], may be a view)"""
    for g, a0, b0 in zip(gs, pa, qb):
        r, n = g.shape
        v = scale * (p[:, a0:a0 + r].float().t() @ q[:, b0:b0 + n].float())
        if accumulate:
            v = v + g.float()
        g.copy_(v.to(g.dtype))


def lora_pack_t(As):
    """[sum r_i, K] = concat_i A_i^T"""
    return torch.cat([a.t() for a in As], 0).contiguous()
