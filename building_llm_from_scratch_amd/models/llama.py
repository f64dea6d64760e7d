"""Llama-2 / Llama-3 / 3.1 / 3.2 (one GQA module; MHA is GQA with n_kv_groups == n_heads).

Parity (reference, read-only):
  * module / state-dict names: ``tok_emb``, ``trf_blocks.{i}.att.W_query|W_key|W_value|out_proj``,
    ``trf_blocks.{i}.ff.fc1|fc2|fc3``, ``trf_blocks.{i}.norm1|norm2``, ``final_norm``, ``out_head``
    plus the ``att.mask|cos|sin`` buffers (Llama3.py:108-204, Llama2.py:61-190);
  * math: pre-RMSNorm (eps 1e-5, fp32 weight in checkpoints), rotate-half RoPE with the 3.1
    by-parts smoothing, causal GQA, SwiGLU ``fc3(silu(fc1 x) * fc2 x)``, untied head
    (common_components.py:6-124, Llama3.py:131-181).

MI355X execution (per block, N = B*T rows, all bf16 with fp32 accumulation):
  rmsnorm[HIP] -> QKV GEMM (fused [Wq;Wk;Wv], hipBLASLt) -> RoPE in place[HIP] ->
  flash-attention fwd (GQA-native, no repeat_interleave)[HIP MFMA] -> out-proj GEMM with
  the residual add in the epilogue (addmm beta=1) -> rmsnorm[HIP] -> gate/up GEMM (fused
  [fc1;fc2]) -> SwiGLU[HIP] -> down GEMM + residual.  Backward mirrors it and writes all
  weight gradients into the unit's flat gradient buffer.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .. import ops
from .base import BaseLM, UnitCompute, cached_attention
from .linear import FusedLinear, _dgrad_wt_ok, _weight_grad, mm_nt


# ---------------------------------------------------------------------------
# reference-named containers (parameters become views into flat unit buffers)
# ---------------------------------------------------------------------------
class RMSNorm(nn.Module):
    def __init__(self, emb_dim, eps=1e-5, dtype=None, device=None):
        super().__init__()
        self.eps = eps
        self.emb_dim = emb_dim
        self.weight = nn.Parameter(torch.ones(emb_dim, dtype=dtype, device=device))

    def reset_parameters(self):   # (seeded per-unit init of a meta-built model, base.py:init_unit_)
        with torch.no_grad():
            self.weight.fill_(1.0)

    def forward(self, x):  # reference-style eager path (used only by tests / users)
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)
        return (y * self.weight.float()).to(x.dtype)


class GroupedQueryAttention(nn.Module):
    def __init__(self, d_in, d_out, context_length, num_heads, num_kv_groups, rope_base=10_000,
                 rope_config=None, dtype=None, device=None):
        super().__init__()
        assert d_out % num_heads == 0 and num_heads % num_kv_groups == 0
        self.d_out = d_out
        self.num_heads = num_heads
        self.head_dim = d_out // num_heads
        self.num_kv_groups = num_kv_groups
        self.group_size = num_heads // num_kv_groups
        kw = dict(bias=False, dtype=dtype, device=device)
        self.W_query = nn.Linear(d_in, d_out, **kw)
        self.W_key = nn.Linear(d_in, num_kv_groups * self.head_dim, **kw)
        self.W_value = nn.Linear(d_in, num_kv_groups * self.head_dim, **kw)
        self.out_proj = nn.Linear(d_out, d_out, **kw)


# reference Llama2.py names this MultiHeadAttention
class MultiHeadAttention(GroupedQueryAttention):
    def __init__(self, d_in, d_out, context_length, num_heads, dtype=None, device=None):
        super().__init__(d_in, d_out, context_length, num_heads, num_heads, dtype=dtype, device=device)


class FeedForward(nn.Module):
    def __init__(self, cfg, device=None):
        super().__init__()
        kw = dict(bias=False, dtype=cfg["dtype"], device=device)
        self.fc1 = nn.Linear(cfg["emb_dim"], cfg["hidden_dim"], **kw)
        self.fc2 = nn.Linear(cfg["emb_dim"], cfg["hidden_dim"], **kw)
        self.fc3 = nn.Linear(cfg["hidden_dim"], cfg["emb_dim"], **kw)


class TransformerBlock(nn.Module):
    def __init__(self, cfg, device=None):
        super().__init__()
        self.att = GroupedQueryAttention(cfg["emb_dim"], cfg["emb_dim"], cfg["context_length"],
                                         cfg["n_heads"], cfg["n_kv_groups"], cfg["rope_base"],
                                         cfg["rope_freq"], dtype=cfg["dtype"], device=device)
        self.ff = FeedForward(cfg, device=device)
        self.norm1 = RMSNorm(cfg["emb_dim"], eps=1e-5, dtype=cfg["dtype"], device=device)
        self.norm2 = RMSNorm(cfg["emb_dim"], eps=1e-5, dtype=cfg["dtype"], device=device)


# ---------------------------------------------------------------------------
# unit computes
# ---------------------------------------------------------------------------
class LlamaEmbedCompute(UnitCompute):
    name = "tok_emb"

    def __init__(self, rctx, model):
        super().__init__(rctx)
        self.m = model

    def layout(self):
        return [[self.m.tok_emb.weight]]

    def forward(self, idx, save, replay=None):
        rc = self.rctx
        W = self.unit.data(self.m.tok_emb.weight)
        x = ops.embedding_fwd(idx.reshape(-1), W, None, rc.T)
        return x.view(rc.B, rc.T, -1), (idx.reshape(-1) if save else None)

    def backward(self, dx, saved):
        g = self.unit.grad(self.m.tok_emb.weight)
        if g is not None:
            ops.embedding_bwd(saved, dx.view(-1, dx.shape[-1]), g, None, self.rctx.T, self.rctx.accumulate)
        return None

    def infer(self, idx, pos):
        W = self.unit.data(self.m.tok_emb.weight)
        return ops.embedding_fwd(idx.reshape(-1).contiguous(), W, None, idx.shape[1])

    def infer_dev(self, idx, pos_t):
        W = self.unit.data(self.m.tok_emb.weight)
        return ops.embedding_fwd(idx.reshape(-1).contiguous(), W, None, 1)


class LlamaBlockCompute(UnitCompute):
    def __init__(self, rctx, block: TransformerBlock, i: int):
        super().__init__(rctx)
        self.block = block
        self.name = f"trf_blocks.{i}"
        self.index = i
        a, f = block.att, block.ff
        self.qkv = FusedLinear([a.W_query, a.W_key, a.W_value])
        self.o = FusedLinear([a.out_proj])
        self.gu = FusedLinear([f.fc1, f.fc2])
        self.down = FusedLinear([f.fc3])

    def layout(self):
        b = self.block
        return (self.qkv.layout() + self.o.layout() + self.gu.layout() + self.down.layout()
                + [[b.norm1.weight], [b.norm2.weight]])

    def bind(self, unit):
        super().bind(unit)
        for fl in (self.qkv, self.o, self.gu, self.down):
            fl.bind(unit)

    def forward(self, x, save, replay=None, recompute=False):
        """``recompute``: the activation-checkpoint re-run inside backward — the block output
        is not needed there, so the down projection GEMM (1/6 of the block's forward FLOPs) is
        skipped; only its LoRA intermediate, if any, is rebuilt."""
        rc, cfg, u, b = self.rctx, self.rctx.cfg, self.unit, self.block
        B, T = rc.B, rc.T
        N, d = B * T, cfg.emb_dim
        H, G, hd = cfg.n_heads, cfg.n_kv_groups, cfg.head_dim
        eps = cfg.norm_eps
        cos, sin = rc.rope
        x2d = x.reshape(N, d)
        keep = rc.block_mode(self.index) == "none" or recompute  # the recompute's outputs live one block
        # LoRA with a frozen base: the norms / SwiGLU write straight into the K-augmented
        # [x | s t] operand of the next projection (FusedLinear.kaug_input / forward_kaug)
        xq = self.qkv.kaug_input(x2d, d)
        if xq is not None:
            h1, r1 = ops.rmsnorm_fwd_into(x2d, u.data(b.norm1.weight), eps, xq[:, :d])
            qkv, xa_qkv = self.qkv.forward_kaug(xq, d)
            ops.rope_(qkv, cos, sin, T, H, G, hd)
        else:
            h1, r1 = ops.rmsnorm_fwd(x2d, u.data(b.norm1.weight), eps)
            qkv = self.qkv.forward_rope(h1, cos, sin, T, H, G, hd)   # K4: RoPE in the GEMM epilogue
            if qkv is not None:
                xa_qkv = None
            else:
                qkv, xa_qkv = self.qkv.forward(h1)
                ops.rope_(qkv, cos, sin, T, H, G, hd)
        o, lse = ops.flash_attn_fwd(qkv, B, T, H, G, hd, causal=True)
        x2, xa_o = self.o.forward(o, residual=x2d)
        xg = self.gu.kaug_input(x2, d)
        fused = None
        if xg is not None:
            h2, r2 = ops.rmsnorm_fwd_into(x2, u.data(b.norm2.weight), eps, xg[:, :d])
            gu, xa_gu = self.gu.forward_kaug(xg, d)
        else:
            h2, r2 = ops.rmsnorm_fwd(x2, u.data(b.norm2.weight), eps)
            if not (recompute and not self.down.has_lora and RECOMPUTE_FUSED):
                fused = self.gu.forward_swiglu(h2)     # gate/up GEMM with the SwiGLU epilogue
            if fused is not None:
                (gu, act), xa_gu = fused, None
            else:
                gu, xa_gu = self.gu.forward(h2)
        if recompute and not self.down.has_lora and RECOMPUTE_FUSED:
            # backward rebuilds act inside the SwiGLU backward kernel (swiglu_bwd_act)
            act, x3, xa_dn = None, None, None
        else:
            F = gu.shape[1] // 2
            xd = None if (fused is not None or recompute) else self.down.kaug_input(gu, F)
            if xd is not None:
                act = ops.swiglu_fwd_into(gu, xd[:, :F])
                x3, xa_dn = self.down.forward_kaug(xd, F, residual=x2)
            else:
                if fused is None:
                    act = ops.swiglu_fwd(gu)
                if recompute:
                    x3, xa_dn = None, self.down.lora_state(act)
                else:
                    x3, xa_dn = self.down.forward(act, residual=x2)
        saved = None
        if save:
            if not keep:
                # h1 / h2 are dropped (rebuilt in backward): keep only the s t columns of their
                # K-augmented buffers, not the whole [x | s t]
                xa_qkv, xa_gu = (_compact_kaug(v) for v in (xa_qkv, xa_gu))
            saved = dict(x=x2d, r1=r1, qkv=qkv, o=o, lse=lse, x2=x2, r2=r2, gu=gu,
                         xa=(xa_qkv, xa_o, xa_gu, xa_dn))
            # selective: act is rebuilt by the SwiGLU backward (swiglu_bwd_act), h1/h2 by rmsnorm
            if act is not None and (keep or self.down.has_lora or not RECOMPUTE_FUSED):
                saved["act"] = act
            if keep:
                saved.update(h1=h1, h2=h2)
        return (x3.view(B, T, d) if x3 is not None else None), saved

    def infer_dev(self, x2d, pos_t, kv):
        """Decode step with the position in device memory (RoPE reads it, the decode kernel
        appends K/V at it): capturable in a HIP graph and replayed once per generated token."""
        cfg, u, b = self.rctx.cfg, self.unit, self.block
        H, G, hd, eps = cfg.n_heads, cfg.n_kv_groups, cfg.head_dim, cfg.norm_eps
        cos, sin = self.rctx.rope
        h1, _ = ops.rmsnorm_fwd(x2d, u.data(b.norm1.weight), eps)
        qkv, _ = self.qkv.forward(h1)
        ops.rope_dev_(qkv, cos, sin, H, G, hd, pos_t)
        o = ops.attn_decode_append(qkv, kv[0], kv[1], pos_t, H, G)
        x2, _ = self.o.forward(o, residual=x2d)
        h2, _ = ops.rmsnorm_fwd(x2, u.data(b.norm2.weight), eps)
        gu, _ = self.gu.forward(h2)
        x3, _ = self.down.forward(ops.swiglu_fwd(gu), residual=x2)
        return x3

    def infer(self, x2d, B, t, pos, kv):
        cfg, u, b = self.rctx.cfg, self.unit, self.block
        H, G, hd, eps = cfg.n_heads, cfg.n_kv_groups, cfg.head_dim, cfg.norm_eps
        cos, sin = self.rctx.rope
        h1, _ = ops.rmsnorm_fwd(x2d, u.data(b.norm1.weight), eps)
        qkv, _ = self.qkv.forward(h1)
        ops.rope_(qkv, cos, sin, t, H, G, hd, pos_offset=pos)
        o = cached_attention(qkv, B, t, pos, H, G, hd, kv)
        x2, _ = self.o.forward(o, residual=x2d)
        h2, _ = ops.rmsnorm_fwd(x2, u.data(b.norm2.weight), eps)
        gu, _ = self.gu.forward(h2)
        x3, _ = self.down.forward(ops.swiglu_fwd(gu), residual=x2)
        return x3

    def _lora_swiglu_wgrad(self, xa_dn, xa_gu, F):
        """(gB_gate, gB_up, gA_down^T) when the MLP's LoRA gradients can be summed inside the
        SwiGLU backward (ops.swiglu_bwd_lowrank_wgrad: both groups K-augmented, rank 16 per
        member, the down projection's low-rank dX formed by that kernel, all three trainable),
        else None."""
        dn, gu = self.down, self.gu
        if not (LORA_SWIGLU_WGRAD and dn.has_lora and gu.has_lora):
            return None
        kaug = lambda xa: isinstance(xa, tuple) and xa[0] == "kaug"  # noqa: E731
        if not (kaug(xa_dn) and kaug(xa_gu) and dn.lora_R == 16 and gu.lora_r == [16, 16]
                and gu.lora_c0 == [0, F] and gu.lora_len == [F, F] and gu.lora_off == [0, 16]
                and ops.swiglu_bwd_lowrank_ok(16, F) and ops.swiglu_bwd_lowrank_wgrad_ok(16, F)):
            return None
        u = self.unit
        gBg, gBu = (u.grad(sp.lora_B) for sp in gu.lora_specs)
        gAd = u.grad(dn.lora_specs[0].lora_A)
        if gBg is None or gBu is None or gAd is None or not (gBg.dtype == gBu.dtype == gAd.dtype):
            return None
        return gBg, gBu, gAd.t()

    def backward(self, dy, s):
        rc, cfg, u, b = self.rctx, self.rctx.cfg, self.unit, self.block
        B, T = rc.B, rc.T
        N, d = B * T, cfg.emb_dim
        H, G, hd = cfg.n_heads, cfg.n_kv_groups, cfg.head_dim
        eps, acc = cfg.norm_eps, rc.accumulate
        cos, sin = rc.rope
        xa_qkv, xa_o, xa_gu, xa_dn = s["xa"]
        dy2 = dy.reshape(N, d)
        w1, w2 = u.data(b.norm1.weight), u.data(b.norm2.weight)
        # ---- MLP
        gu_B_done = False
        if "act" in s or self.down.has_lora:
            fuse = self._lora_swiglu_wgrad(xa_dn, xa_gu, s["gu"].shape[1] // 2)
            # the fused kernel rebuilds act itself: no SwiGLU forward for the down dA
            act = s["act"] if "act" in s else (s["gu"][:, :s["gu"].shape[1] // 2] if fuse
                                               else ops.swiglu_fwd(s["gu"]))
            d_act = self.down.backward(dy2, act, xa_dn, accumulate=acc, lowrank_dx=True, defer_lora_A=fuse is not None)
            del act
            assert fuse is None or (isinstance(d_act, tuple) and d_act[5]), "fused LoRA SwiGLU path not taken"
            if isinstance(d_act, tuple) and d_act[5]:
                # K-augmented LoRA MLP: dact = base + s u P, the gate/up dB and the down dA summed in
                # the same pass over the rows (ops.swiglu_bwd_lowrank_wgrad)
                d_gu = ops.swiglu_bwd_lowrank_wgrad(s["gu"], *d_act[1:5], xa_gu[1], *fuse, accumulate=acc)
                gu_B_done = True
            elif isinstance(d_act, tuple):   # K-augmented LoRA: dact = base + s u P inside the kernel
                d_gu = ops.swiglu_bwd_lowrank(s["gu"], *d_act[1:5])
            else:
                d_gu = ops.swiglu_bwd(s["gu"], d_act)
            del d_act
        else:
            # recompute without act: dX GEMM first, then one SwiGLU backward pass that also
            # rebuilds act in place of d_act, then the down projection's dW from it
            act = self.down.input_grad(dy2)
            d_gu = ops.swiglu_bwd_act(s["gu"], act)
            self.down.backward(dy2, act, None, need_dx=False, accumulate=acc)
            del act
        h2 = s["h2"] if "h2" in s else ops.rmsnorm_fwd(s["x2"], w2, eps)[0]
        dh2 = self.gu.backward(d_gu, h2, xa_gu, accumulate=acc, lora_B_done=gu_B_done)
        del d_gu, h2
        dx2, _ = ops.rmsnorm_bwd(dh2, s["x2"], w2, s["r2"], dy2, u.grad(b.norm2.weight), acc)
        del dh2
        # ---- attention
        d_o = self.o.backward(dx2, s["o"], xa_o, accumulate=acc)
        dqkv = ops.flash_attn_bwd(s["qkv"], s["o"], s["lse"], d_o, B, T, H, G, hd, causal=True,
                                  rope=(cos, sin))  # inverse RoPE fused into the kernels' epilogues
        del d_o
        h1 = s["h1"] if "h1" in s else ops.rmsnorm_fwd(s["x"], w1, eps)[0]
        dh1 = self.qkv.backward(dqkv, h1, xa_qkv, accumulate=acc)
        del dqkv, h1
        dx, _ = ops.rmsnorm_bwd(dh1, s["x"], w1, s["r1"], dx2, u.grad(b.norm1.weight), acc)
        return dx.view(B, T, d)


# False: the gate/up dB and down dA of a LoRA MLP as separate lora_wgrad passes (A/B)
LORA_SWIGLU_WGRAD = True


def _compact_kaug(xa):
    """A saved ("kaug", s t view, P, WaT) with the s t columns copied out of their buffer."""
    if isinstance(xa, tuple) and xa[0] == "kaug":
        return (xa[0], xa[1].contiguous(), xa[2], xa[3])
    return xa


# False: the checkpoint recompute runs its SwiGLU forward as a separate pass (A/B)
RECOMPUTE_FUSED = True

# logits chunk budget of the fused head + CE (bytes of one [rows, V] chunk)
LOGIT_CHUNK_BYTES = int(os.environ.get("BLLM_LOGIT_CHUNK_MB", "2048")) * 2 ** 20
MIN_CHUNK_ROWS = 256  # chunk rows are a multiple of this (token-major dW kernel K granule)


class HeadComputeMixin:
    """final norm + LM head + fused cross-entropy (reference train.py:88-92).

    Training forward (``forward_loss`` with ``save``): the head GEMM, CE forward, CE backward and
    both head gradient GEMMs run chunk by chunk over the tokens, so the [N, V] logits never exist
    at once (Llama-3-8B, 24k tokens: 6.3 GB of bf16 logits -> 2 GiB chunks, 3 of them; 6 chunks
    of 1 GiB measured +5 ms / step, profiles/r2_llama3_8b_fsdp_full_v3.md).  The loss
    gradient is taken for dloss = ``rctx.loss_scale`` (1, or the fp16 loss scale the trainer
    announces before the forward) and rescaled by dloss / loss_scale in backward (dh and dW, one
    pass each; exactly 1 when the announced scale is the dloss that arrives).  Taking it at the
    loss scale matters in fp16: softmax tails p / nvalid below fp16's smallest subnormal would
    round to 0 before any later scaling could lift them."""

    ignore_index = -100

    def _norm_fwd(self, x):
        raise NotImplementedError

    def _norm_bwd(self, dh, ns, dx_acc=None):
        raise NotImplementedError

    def infer(self, x2d, B, t):
        last = x2d.view(B, t, -1)[:, -1, :].contiguous()
        logits, _ = self.forward_logits(last, save=False)
        return logits

    def forward_logits(self, x, save):
        x2d = x.reshape(-1, x.shape[-1])
        h, ns = self._norm_fwd(x2d)
        logits, xa = self.head.forward(h)
        return logits, ((x2d, h, ns, xa) if save else None)

    def backward_logits(self, dlogits, saved):
        x2d, h, ns, xa = saved
        dl = dlogits.reshape(-1, dlogits.shape[-1]).to(h.dtype)
        dh = self.head.backward(dl, h, xa, accumulate=self.rctx.accumulate)
        dx = self._norm_bwd(dh, (x2d,) + ns)
        return dx.view(self.rctx.B, self.rctx.T, -1)

    def _fused_ok(self, h) -> bool:
        return not self.head.has_lora and self.head.b_params is None

    def _head_padded(self, W: torch.Tensor):
        """W with its rows padded to a multiple of 256 (zero rows), or W itself when V already is
        one.  GPT-2's V = 50,257 gives odd-leading-dimension logits, on which hipBLASLt falls back
        to slower non-K-contiguous kernels (2.2-2.6 ms per 16k-token chunk, 0.8-1 PF); the padded
        vocabulary keeps every head GEMM on the tile-aligned kernels and our dW kernel.  The buffer
        is kept across steps (its pad rows are zeroed once); the V real rows are re-copied per
        call: the optimizer moves them."""
        V, d = W.shape
        Vp = -(-V // 256) * 256
        if Vp == V or not W.is_cuda:
            return W
        buf = getattr(self, "_wpad_buf", None)
        if buf is None or buf.shape != (Vp, d) or buf.dtype != W.dtype or buf.device != W.device:
            buf = self._wpad_buf = torch.zeros(Vp, d, dtype=W.dtype, device=W.device)
        buf[:V].copy_(W)
        return buf

    def _fused_loss(self, x2d, h, ns, targets, nvalid):
        W = self.head.W()                                          # [V, d]
        N, V = h.shape[0], W.shape[0]
        Wp = self._head_padded(W)                                  # [Vp, d], rows >= V zero
        Vp = Wp.shape[0]
        rows = max(MIN_CHUNK_ROWS, LOGIT_CHUNK_BYTES // (Vp * h.element_size()) // MIN_CHUNK_ROWS * MIN_CHUNK_ROWS)
        gW = gWp = None
        if self.head.unit.trainable(self.head.W_params[0]):
            gW = torch.empty(W.shape, dtype=self.head.unit.train.grad.dtype, device=W.device)
            gWp = gW if Vp == V else torch.empty(Wp.shape, dtype=gW.dtype, device=W.device)
        dh = torch.empty_like(h)
        Wd = Wp
        if _dgrad_wt_ok(h[:rows], Wp):   # one K-contiguous copy of W for every chunk's dX GEMM
            Wd = ops.transpose2d(Wp).t()
        scale = (self.rctx.loss_scale / nvalid).reshape(1)
        total = torch.zeros(1, dtype=torch.float32, device=h.device)
        for s0 in range(0, N, rows):
            hc, tc = h[s0:s0 + rows], targets[s0:s0 + rows]
            logits = mm_nt(hc, Wp)                                 # [rows, Vp]; columns >= V are 0
            lv = logits[:, :V]
            lrow, lse = ops.ce_fwd(lv, tc, self.ignore_index)
            total += lrow.sum()
            ops.ce_bwd_(lv, tc, lse, scale, self.ignore_index)    # in place; the zero pad stays
            dl = logits
            if Wd is not Wp:
                mm_nt(dl, Wd.t(), out=dh[s0:s0 + rows])                   # dh = dl . W (W^T copy)
            else:
                torch.mm(dl, Wd, out=dh[s0:s0 + rows])
            if gWp is not None:
                _weight_grad(dl, hc, gWp, accumulate=s0 > 0)
            del logits, dl, lv
        if gWp is not None and gWp is not gW:
            gW.copy_(gWp[:V])
        return total[0] / nvalid, (x2d, ns, dh, gW, [], self.rctx.loss_scale, "fused")

    def _fused_lora_ok(self, h) -> bool:
        hd = self.head
        if not (hd.has_lora and len(hd.specs) == 1 and hd.b_params is None
                and not hd.unit.trainable(hd.W_params[0])):
            return False
        # on the GPU the rank-r parts run on csrc/lora.hip (rank % 16 <= 64, widths % 32)
        spec = hd.specs[0]
        return not h.is_cuda or ops.lora_kernel_ok_dims(h.device, h.dtype, [spec.lora_A.shape[1]],
                                                        [h.shape[1], spec.out_features])

    def _waug(self, W, Bm, rp: int):
        """[W | B^T | 0] ([V, d + rp], rp >= r pads a row to whole 128-byte lines) in a buffer kept
        across steps; W and B^T re-copied per call (FSDP may re-materialise W, the optimizer moves
        B), the pad columns zeroed once."""
        V, d = W.shape
        r = Bm.shape[0]
        buf = getattr(self, "_waug_buf", None)
        if buf is None or buf.shape != (V, d + rp) or buf.dtype != W.dtype or buf.device != W.device:
            buf = self._waug_buf = torch.zeros(V, d + rp, dtype=W.dtype, device=W.device)
        buf[:, :d].copy_(W)
        buf[:, d:d + r].copy_(Bm.t())
        return buf

    def _fused_lora_loss(self, x2d, h, ns, targets, nvalid):
        """LoRA head (the reference's replace_linear_with_lora also wraps the output head; its
        base weight is frozen) on the same chunked head + CE, with the rank-r path folded into
        the logits GEMM by augmenting K (t = h A, s = alpha / r):
            logits = [h | s t | 0] . [W | B^T | 0]^T          (rows padded to 128-byte lines)
        one GEMM per chunk instead of a separate s t B pass over the [N, V] logits plus a beta = 1
        GEMM.  The dX GEMM stays at the base width, dh_W = dl . W on the cached K-contiguous W^T
        (an augmented [N, d + r] output made hipBLASLt fall back from 1.64 to 0.66-0.75 PF at
        V = 128k, tools/bench_head_k.py); u = dl B^T is a skinny hipBLASLt GEMM over each dlogits
        chunk (355 us vs 610 us for lora_down, tools/bench_head_u.py), dB = (s t)^T dl runs on
        lora_wgrad, then dh = dh_W + s u A^T and dA = s h^T u on the LoRA kernels.  With
        ops.LORA_HEAD_FUSED (default) u and dB come from one kernel reading each dl chunk once
        (``ops.lora_head_bwd_``)."""
        hd, u_ = self.head, self.head.unit
        spec = hd.specs[0]
        A, Bm, sc = u_.data(spec.lora_A), u_.data(spec.lora_B), float(spec.scaling)   # [d, r], [r, V]
        W = hd.W()
        N, d = h.shape
        V, r = W.shape[0], A.shape[1]
        rp = -(-(d + r) // 64) * 64 - d
        Wa = self._waug(W, Bm, rp)
        P = ops.lora_pack_t([A])                                            # A^T [r, d]
        ha = torch.empty(N, d + rp, dtype=h.dtype, device=h.device)
        ha[:, :d].copy_(h)
        ops.lora_down_into(h, [P], [0], [d], [0], r, sc, ha[:, d:])         # [s h A | 0]
        st = ha[:, d:d + r]
        rows = max(MIN_CHUNK_ROWS, LOGIT_CHUNK_BYTES // (V * h.element_size()) // MIN_CHUNK_ROWS * MIN_CHUNK_ROWS)
        Wd = W
        if _dgrad_wt_ok(h[:rows], W):    # frozen: the K-contiguous W^T copy is kept across steps
            key = (W.data_ptr(), W._version, W.shape, W.dtype)
            cached = getattr(self, "_wt_cache", None)
            if cached is None or cached[0] != key:
                cached = self._wt_cache = (key, ops.transpose2d(W))
            Wd = cached[1].t()
        dh = torch.empty_like(h)
        ub = torch.empty(N, r, dtype=h.dtype, device=h.device)
        # (grad views only exist in backward: FSDP allocates the full gradient in pre_backward)
        gB = torch.empty(r, V, dtype=torch.float32, device=h.device) if u_.trainable(spec.lora_B) else None
        scale = (self.rctx.loss_scale / nvalid).reshape(1)
        total = torch.zeros(1, dtype=torch.float32, device=h.device)
        fused_bwd = ops.lora_head_bwd_ok(V, r) and Bm.is_contiguous()
        for s0 in range(0, N, rows):
            hc, tc = ha[s0:s0 + rows], targets[s0:s0 + rows]
            logits = mm_nt(hc, Wa)
            lrow, lse = ops.ce_fwd(logits, tc, self.ignore_index)
            total += lrow.sum()
            dl = ops.ce_bwd_(logits, tc, lse, scale, self.ignore_index)   # in place
            if Wd is not W:
                mm_nt(dl, Wd.t(), out=dh[s0:s0 + rows])                   # dh_W = dl . W
            else:
                torch.mm(dl, Wd, out=dh[s0:s0 + rows])
            if gB is not None and fused_bwd:                              # u and dB in one pass over dl
                ops.lora_head_bwd_(dl, st[s0:s0 + rows], Bm, ub[s0:s0 + rows], gB, accumulate=s0 > 0)
                del logits, dl
                continue
            torch.mm(dl, Bm.t(), out=ub[s0:s0 + rows])            # u = dl B^T (hipBLASLt: 5.9 TB/s here)
            if gB is not None:                                            # dB = (s t)^T dl
                ops.lora_wgrad(st[s0:s0 + rows], dl, [gB], [0], [0], 1.0, accumulate=s0 > 0)
            del logits, dl
        ops.lora_up_(dh, ub, [P], [0], [0], sc, base=dh)                  # dh_W + s u A^T
        lora = []
        if gB is not None:
            lora.append((spec.lora_B, gB))
        if u_.trainable(spec.lora_A):                                     # dA = s h^T u
            gA = torch.empty(d, r, dtype=torch.float32, device=h.device)
            ops.lora_wgrad(ub, h, [gA.t()], [0], [0], sc)
            lora.append((spec.lora_A, gA))
        del ha
        return total[0] / nvalid, (x2d, ns, dh, None, lora, self.rctx.loss_scale, "fused")

    def forward_loss(self, x, targets, save):
        x2d = x.reshape(-1, x.shape[-1])
        h, ns = self._norm_fwd(x2d)
        if save and (self._fused_ok(h) or self._fused_lora_ok(h)):
            nvalid = (targets != self.ignore_index).sum().to(torch.float32).clamp_(min=1.0)
            if not self._fused_ok(h):
                return self._fused_lora_loss(x2d, h, ns, targets, nvalid)
            return self._fused_loss(x2d, h, ns, targets, nvalid)
        logits, xa = self.head.forward(h)
        rows, lse = ops.ce_fwd(logits, targets, self.ignore_index)
        # a batch whose targets are all ignore_index (e.g. prompts longer than the context in
        # instruction finetuning) gives loss 0 and zero gradients (torch's mean CE gives NaN)
        nvalid = (targets != self.ignore_index).sum().to(torch.float32).clamp_(min=1.0)
        loss = rows.sum() / nvalid
        if not save:
            return loss, None
        return loss, (x2d, h, ns, xa, logits, lse, targets, nvalid)

    def backward_loss(self, dloss, saved):
        if saved[-1] == "fused":
            x2d, ns, dh, gW, lora, ls, _ = saved
            dls = dloss.float().reshape(1) / ls
            dh.mul_(dls)
            if gW is not None:
                g = self.head.unit.fused_grad(self.head.W_params)
                if self.rctx.accumulate:
                    g.add_(gW * dls)
                else:
                    torch.mul(gW, dls, out=g)
            for p, gp in lora:  # LoRA head: dA / dB taken for dloss = 1 in forward
                g = self.head.unit.grad(p)
                if self.rctx.accumulate:
                    g.add_(gp * dls)
                else:
                    g.copy_(gp * dls)
            dx = self._norm_bwd(dh, (x2d,) + ns)
            return dx.view(self.rctx.B, self.rctx.T, -1)
        x2d, h, ns, xa, logits, lse, targets, nvalid = saved
        scale = (dloss.float() / nvalid).reshape(1)
        dlogits = ops.ce_bwd_(logits, targets, lse, scale, self.ignore_index)  # in place
        dh = self.head.backward(dlogits, h, xa, accumulate=self.rctx.accumulate)
        del dlogits
        dx = self._norm_bwd(dh, (x2d,) + ns)
        return dx.view(self.rctx.B, self.rctx.T, -1)


class LlamaHeadCompute(HeadComputeMixin, UnitCompute):
    name = "final"

    def __init__(self, rctx, model):
        super().__init__(rctx)
        self.m = model
        self.head = FusedLinear([model.out_head])

    def layout(self):
        return [[self.m.final_norm.weight]] + self.head.layout()

    def bind(self, unit):
        super().bind(unit)
        self.head.bind(unit)

    def _norm_fwd(self, x2d):
        h, r = ops.rmsnorm_fwd(x2d, self.unit.data(self.m.final_norm.weight), self.rctx.cfg.norm_eps)
        return h, (r,)

    def _norm_bwd(self, dh, ns):
        x2d, r = ns
        w = self.m.final_norm.weight
        dx, _ = ops.rmsnorm_bwd(dh, x2d, self.unit.data(w), r, None, self.unit.grad(w), self.rctx.accumulate)
        return dx


# ---------------------------------------------------------------------------
class LlamaModel(BaseLM):
    """Llama-2 / 3 / 3.1 / 3.2 (reference Llama2Model, Llama3Model)."""

    def __init__(self, cfg, use_actv_ckpt=False, device=None):
        super().__init__(cfg, use_actv_ckpt)
        dt = cfg["dtype"]
        self.tok_emb = nn.Embedding(cfg["vocab_size"], cfg["emb_dim"], dtype=dt, device=device)
        self.trf_blocks = nn.Sequential(*[TransformerBlock(cfg, device) for _ in range(cfg["n_layers"])])
        self.final_norm = RMSNorm(cfg["emb_dim"], eps=1e-5, dtype=dt, device=device)
        self.out_head = nn.Linear(cfg["emb_dim"], cfg["vocab_size"], bias=False, dtype=dt, device=device)
        self._register_state_dict_hook(_llama_state_dict_hook)
        self._register_load_state_dict_pre_hook(_llama_load_pre_hook)
        self.include_buffers_in_state_dict = True

    def build_computes(self):
        rc = self._rctx
        return ([LlamaEmbedCompute(rc, self)]
                + [LlamaBlockCompute(rc, b, i) for i, b in enumerate(self.trf_blocks)]
                + [LlamaHeadCompute(rc, self)])

    def _after_flatten(self, device):
        cfg = self.cfg
        self._rctx.rope = ops.rope_tables(cfg.head_dim, cfg.context_length, cfg.rope_base,
                                          cfg.rope_freq, device=device)


Llama3Model = LlamaModel
Llama2Model = LlamaModel


def _llama_buffers(cfg):
    """Reference per-block buffers: mask [T,T] fp32 (triu ones), cos/sin [T, hd] (halves
    duplicated) — bf16 for Llama-3.x, fp32 for Llama-2 (Llama3.py:59-70, Llama2.py:83-88)."""
    T, hd = cfg.context_length, cfg.head_dim
    mask = torch.triu(torch.ones(T, T), diagonal=1)
    c, s = ops.rope_tables(hd, T, cfg.rope_base, cfg.rope_freq)
    cos = torch.cat([c, c], dim=1)
    sin = torch.cat([s, s], dim=1)
    if cfg.name != "llama2":
        cos, sin = cos.to(cfg.dtype), sin.to(cfg.dtype)
    return mask, cos, sin


def _llama_state_dict_hook(module, state_dict, prefix, local_metadata):
    # RMSNorm weights are fp32 in the reference's checkpoints
    for k in list(state_dict.keys()):
        if k.endswith("norm1.weight") or k.endswith("norm2.weight") or k.endswith("final_norm.weight"):
            state_dict[k] = state_dict[k].float()
    if getattr(module, "include_buffers_in_state_dict", False):
        mask, cos, sin = _llama_buffers(module.cfg)
        for i in range(module.cfg.n_layers):
            p = f"{prefix}trf_blocks.{i}.att."
            state_dict[p + "mask"] = mask
            state_dict[p + "cos"] = cos
            state_dict[p + "sin"] = sin
    return state_dict


def _llama_load_pre_hook(state_dict, prefix, *args, **kwargs):
    for k in list(state_dict.keys()):
        if k.startswith(prefix) and (k.endswith(".att.mask") or k.endswith(".att.cos") or k.endswith(".att.sin")):
            del state_dict[k]
