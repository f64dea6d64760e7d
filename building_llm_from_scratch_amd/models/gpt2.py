"""GPT-2 (reference Models/GPT2/GPT2.py:6-124).

Names / state dict: ``tok_emb``, ``pos_emb``, ``blocks.{i}.att.W_query|W_key|W_value|out_proj``
(+ ``att.mask`` buffer), ``blocks.{i}.ff.layers.0|2``, ``blocks.{i}.norm1|norm2``, ``norm``,
``output_head`` (untied).  Math: pre-LayerNorm, causal MHA with attention-probability
dropout, residual dropout, embedding dropout (p = ``drop_rate`` = 0.1), exact-erf GELU MLP.

Differences: parameters follow ``--data_type`` (the reference ignores it for GPT-2, SURVEY
§2.8 defect 5); no per-forward debug print (defect 10).  Dropout masks come from a
counter-based hash (seed, element offset) so backward and activation-checkpoint recompute
regenerate them instead of storing them; GPU kernels and the CPU path produce identical masks.

Execution per block: LayerNorm[HIP] -> QKV GEMM (+bias epilogue) -> flash attention with
in-kernel dropout[HIP MFMA] -> out-proj GEMM (+bias) -> dropout+residual[HIP] -> LayerNorm
-> fc GEMM (+bias) -> GELU[HIP] -> proj GEMM (+bias) -> dropout+residual[HIP].
"""
from __future__ import annotations


import torch
import torch.nn as nn

from .. import ops
from .base import BaseLM, UnitCompute, cached_attention
from .linear import FusedLinear
from .llama import HeadComputeMixin


class MultiHeadAttention(nn.Module):
    def __init__(self, d_in, d_out, context_length, dropout, num_heads, qkv_bias=False, dtype=None, device=None):
        super().__init__()
        assert d_out % num_heads == 0, "Output dimension must be divisible by number of heads"
        self.d_out = d_out
        self.num_heads = num_heads
        self.head_dim = d_out // num_heads
        kw = dict(dtype=dtype, device=device)
        self.W_query = nn.Linear(d_in, d_out, bias=qkv_bias, **kw)
        self.W_key = nn.Linear(d_in, d_out, bias=qkv_bias, **kw)
        self.W_value = nn.Linear(d_in, d_out, bias=qkv_bias, **kw)
        self.out_proj = nn.Linear(d_out, d_out, **kw)
        self.dropout = nn.Dropout(dropout)


class FeedForward(nn.Module):
    def __init__(self, cfg, device=None):
        super().__init__()
        d = cfg["emb_dim"]
        kw = dict(dtype=cfg["dtype"], device=device)
        self.layers = nn.Sequential(nn.Linear(d, 4 * d, **kw), nn.GELU(), nn.Linear(4 * d, d, **kw))


class TransformerBlock(nn.Module):
    def __init__(self, cfg, device=None):
        super().__init__()
        self.att = MultiHeadAttention(cfg["emb_dim"], cfg["emb_dim"], cfg["context_length"],
                                      cfg["drop_rate"], cfg["n_heads"], cfg["qkv_bias"],
                                      dtype=cfg["dtype"], device=device)
        self.ff = FeedForward(cfg, device)
        kw = dict(dtype=cfg["dtype"], device=device)
        self.norm1 = nn.LayerNorm(cfg["emb_dim"], **kw)
        self.norm2 = nn.LayerNorm(cfg["emb_dim"], **kw)
        self.dropout = nn.Dropout(cfg["drop_rate"])


# ---------------------------------------------------------------------------
class GPTEmbedCompute(UnitCompute):
    name = "embed"

    def __init__(self, rctx, model):
        super().__init__(rctx)
        self.m = model

    def layout(self):
        return [[self.m.tok_emb.weight], [self.m.pos_emb.weight]]

    def forward(self, idx, save, replay=None):
        rc = self.rctx
        p = rc.drop_p
        off = rc.reserve_offsets(idx.numel() * self.rctx.cfg.emb_dim) if p > 0 else 0
        x = ops.embedding_fwd(idx.reshape(-1), self.unit.data(self.m.tok_emb.weight),
                              self.unit.data(self.m.pos_emb.weight), rc.T, p, rc.seed, off)
        return x.view(rc.B, rc.T, -1), ((idx.reshape(-1), p, off) if save else None)

    def infer(self, idx, pos):
        B, t = idx.shape
        wte = self.unit.data(self.m.tok_emb.weight)
        wpe = self.unit.data(self.m.pos_emb.weight)
        return (wte[idx.reshape(-1)].view(B, t, -1) + wpe[pos:pos + t]).reshape(B * t, -1)

    def infer_dev(self, idx, pos_t):
        """One decode token per row, position in device memory (graph-replayable)."""
        wte = self.unit.data(self.m.tok_emb.weight)
        wpe = self.unit.data(self.m.pos_emb.weight)
        return wte.index_select(0, idx.reshape(-1)) + wpe.index_select(0, pos_t)

    def backward(self, dx, saved):
        idx, p, off = saved
        rc = self.rctx
        dx = ops.dropout_bwd(dx.view(-1, dx.shape[-1]), p, rc.seed, off)
        ops.embedding_bwd(idx, dx, self.unit.grad(self.m.tok_emb.weight),
                          self.unit.grad(self.m.pos_emb.weight), rc.T, rc.accumulate)
        return None


def _ln_bwd(unit, norm, dy, x, mean, rstd, dx_acc, acc):
    """LayerNorm backward whose dW / dB land straight in the unit's flat gradient."""
    dx, _, _ = ops.layernorm_bwd(dy, x, unit.data(norm.weight), mean, rstd, dx_acc, unit.grad(norm.weight),
                                 unit.grad(norm.bias), acc)
    return dx


# bias gradients ride along in the dropout / GELU backward passes (ops.*_bwd_bias); tests set
# this to False to check them against the separate column-sum pass
FUSED_BIAS = True
# False: the checkpoint recompute runs its GELU forward as a separate pass (A/B)
RECOMPUTE_FUSED = True
# the attention residual's dropout-add and norm2 as one row pass (ops.dropout_add_layernorm, bitwise
# the two kernels); False: separate passes (A/B, profiles/r5/ln_dropout/)
FUSED_LN_DROPOUT = True


def _drop_bwd_bias(lin, dy, p, seed, offset, acc):
    """dropout backward of ``dy`` with ``lin``'s bias gradient summed in the same pass (when it
    has a trainable bias and dropout is on); returns (d, bias_done)."""
    gb = lin.bias_grad_buf() if FUSED_BIAS else None
    if gb is not None and p > 0.0:
        return ops.dropout_bwd_bias(dy, p, seed, offset, gb, acc), True
    return ops.dropout_bwd(dy, p, seed, offset), False


class GPTBlockCompute(UnitCompute):
    def __init__(self, rctx, block: TransformerBlock, i: int):
        super().__init__(rctx)
        self.block = block
        self.name = f"blocks.{i}"
        self.index = i
        a, f = block.att, block.ff
        self.qkv = FusedLinear([a.W_query, a.W_key, a.W_value])
        self.o = FusedLinear([a.out_proj])
        self.fc = FusedLinear([f.layers[0]])
        self.proj = FusedLinear([f.layers[2]])

    def layout(self):
        b = self.block
        return (self.qkv.layout() + self.o.layout() + self.fc.layout() + self.proj.layout()
                + [[b.norm1.weight, b.norm1.bias], [b.norm2.weight, b.norm2.bias]])

    def bind(self, unit):
        super().bind(unit)
        for fl in (self.qkv, self.o, self.fc, self.proj):
            fl.bind(unit)

    def _ln(self, x, norm):
        u = self.unit
        return ops.layernorm_fwd(x, u.data(norm.weight), u.data(norm.bias), 1e-5)

    def infer_dev(self, x2d, pos_t, kv):
        """Decode step with the position in device memory: K/V appended and attended by one
        kernel (csrc/attn_decode.hip APPEND), so the step can be captured in a HIP graph."""
        cfg, b = self.rctx.cfg, self.block
        H = cfg.n_heads
        qkv, _ = self.qkv.forward(self._ln(x2d, b.norm1)[0])
        a, _ = self.o.forward(ops.attn_decode_append(qkv, kv[0], kv[1], pos_t, H, H))
        x2 = x2d + a
        f, _ = self.fc.forward(self._ln(x2, b.norm2)[0])
        m, _ = self.proj.forward(ops.gelu_fwd(f))
        return x2 + m

    def infer(self, x2d, B, t, pos, kv):
        cfg, b = self.rctx.cfg, self.block
        H, hd = cfg.n_heads, cfg.head_dim
        h1 = self._ln(x2d, b.norm1)[0]
        qkv, _ = self.qkv.forward(h1)
        a, _ = self.o.forward(cached_attention(qkv, B, t, pos, H, H, hd, kv))
        x2 = x2d + a
        f, _ = self.fc.forward(self._ln(x2, b.norm2)[0])
        m, _ = self.proj.forward(ops.gelu_fwd(f))
        return x2 + m

    def forward(self, x, save, replay=None, recompute=False):
        """``recompute`` (activation-checkpoint re-run in backward): the MLP output projection
        and the last residual are skipped — backward never reads the block output."""
        rc, cfg, b = self.rctx, self.rctx.cfg, self.block
        B, T = rc.B, rc.T
        N, d = B * T, cfg.emb_dim
        H, hd = cfg.n_heads, cfg.head_dim
        p = rc.drop_p
        if replay is not None:
            offs = replay
        elif p > 0:
            offs = (rc.reserve_offsets(B * H * T * T), rc.reserve_offsets(N * d), rc.reserve_offsets(N * d))
        else:
            offs = (0, 0, 0)
        x2d = x.reshape(N, d)
        h1, m1, r1 = self._ln(x2d, b.norm1)
        qkv, xa_qkv = self.qkv.forward(h1)
        # attention-dropout keep bits for the backward (only when this forward saves for it)
        km = ops.attn_keep_mask(qkv, B, T, H, hd, p) if save else None
        o, lse = ops.flash_attn_fwd(qkv, B, T, H, H, hd, True, p, rc.seed, offs[0], keep_mask=km)
        a, xa_o = self.o.forward(o)
        if FUSED_LN_DROPOUT:
            u = self.unit
            x2, h2, m2, r2 = ops.dropout_add_layernorm(x2d, a, u.data(b.norm2.weight), u.data(b.norm2.bias), 1e-5,
                                                       p, rc.seed, offs[1])
        else:
            x2 = ops.dropout_add(x2d, a, p, rc.seed, offs[1])
            h2, m2, r2 = self._ln(x2, b.norm2)
        del a
        rebuild_g = recompute and not self.proj.has_lora and RECOMPUTE_FUSED
        fused = None if rebuild_g else self.fc.forward_bias_gelu(h2)   # K9: bias + GELU in the epilogue
        if fused is not None:
            (f, g), xa_fc = fused, None
        else:
            f, xa_fc = self.fc.forward(h2)
            g = None
        if rebuild_g:
            # backward rebuilds g inside the GELU backward pass (ops.gelu_bwd_act)
            g, x3, xa_pr = None, None, None
        elif recompute:
            g = ops.gelu_fwd(f) if g is None else g
            x3, xa_pr = None, self.proj.lora_state(g)
        else:
            g = ops.gelu_fwd(f) if g is None else g
            m, xa_pr = self.proj.forward(g)
            x3 = ops.dropout_add(x2, m, p, rc.seed, offs[2])
        if not save:
            # full-recompute mode: _BlockFn keeps ``offs`` as the replay token so the
            # recomputed forward regenerates identical dropout masks
            return x3.view(B, T, d), offs
        saved = dict(x=x2d, m1=m1, r1=r1, qkv=qkv, o=o, lse=lse, km=km, x2=x2, m2=m2, r2=r2, f=f,
                     p=p, offs=offs, xa=(xa_qkv, xa_o, xa_fc, xa_pr))
        keep = rc.block_mode(self.index) == "none" or recompute  # the recompute's outputs live one block
        # selective: g is rebuilt by the GELU backward (gelu_bwd_act), h1/h2 by the LayerNorm
        if g is not None and (keep or self.proj.has_lora or not RECOMPUTE_FUSED):
            saved["g"] = g
        if keep:
            saved.update(h1=h1, h2=h2)
        return (x3.view(B, T, d) if x3 is not None else None), saved

    def backward(self, dy, s):
        rc, cfg, u, b = self.rctx, self.rctx.cfg, self.unit, self.block
        B, T = rc.B, rc.T
        N, d = B * T, cfg.emb_dim
        H, hd = cfg.n_heads, cfg.head_dim
        acc, p, offs = rc.accumulate, s["p"], s["offs"]
        xa_qkv, xa_o, xa_fc, xa_pr = s["xa"]
        dy2 = dy.reshape(N, d)
        # ---- MLP branch: x3 = x2 + drop(proj(gelu(fc(ln2(x2)))))
        # the bias-gradient column sums ride along in the dropout / GELU backward passes
        dm, pr_b = _drop_bwd_bias(self.proj, dy2, p, rc.seed, offs[2], acc)
        gb = self.fc.bias_grad_buf() if FUSED_BIAS else None
        if "g" in s or self.proj.has_lora:
            g = s["g"] if "g" in s else ops.gelu_fwd(s["f"])
            dg = self.proj.backward(dm, g, xa_pr, accumulate=acc, bias_done=pr_b)
            del dm, g
            if gb is not None:
                df = ops.gelu_bwd_bias(s["f"], dg, gb, acc)
            else:
                df = ops.gelu_bwd(s["f"], dg)
        else:
            # recompute without g: c_proj dX first, then one GELU backward pass that also
            # rebuilds g in place of dg (and sums the c_fc bias grad), then c_proj's dW from g
            dg = self.proj.input_grad(dm)
            df = ops.gelu_bwd_act(s["f"], dg, gb, acc)
            self.proj.backward(dm, dg, None, need_dx=False, accumulate=acc, bias_done=pr_b)
            del dm
        del dg
        h2 = s["h2"] if "h2" in s else self._ln(s["x2"], b.norm2)[0]
        dh2 = self.fc.backward(df, h2, xa_fc, accumulate=acc, bias_done=gb is not None)
        del df, h2
        dx2 = _ln_bwd(u, b.norm2, dh2, s["x2"], s["m2"], s["r2"], dy2, acc)
        # ---- attention branch: x2 = x + drop(out_proj(attn(ln1(x))))
        da, o_b = _drop_bwd_bias(self.o, dx2, p, rc.seed, offs[1], acc)
        d_o = self.o.backward(da, s["o"], xa_o, accumulate=acc, bias_done=o_b)
        del da
        dqkv = ops.flash_attn_bwd(s["qkv"], s["o"], s["lse"], d_o, B, T, H, H, hd, True, p, rc.seed, offs[0],
                                  keep_mask=s.get("km"))
        del d_o
        h1 = s["h1"] if "h1" in s else self._ln(s["x"], b.norm1)[0]
        dh1 = self.qkv.backward(dqkv, h1, xa_qkv, accumulate=acc)
        del dqkv, h1
        dx = _ln_bwd(u, b.norm1, dh1, s["x"], s["m1"], s["r1"], dx2, acc)
        return dx.view(B, T, d)


class GPTHeadCompute(HeadComputeMixin, UnitCompute):
    name = "final"

    def __init__(self, rctx, model):
        super().__init__(rctx)
        self.m = model
        self.head = FusedLinear([model.output_head])

    def layout(self):
        return [[self.m.norm.weight, self.m.norm.bias]] + self.head.layout()

    def bind(self, unit):
        super().bind(unit)
        self.head.bind(unit)

    def _norm_fwd(self, x2d):
        u, n = self.unit, self.m.norm
        h, mean, rstd = ops.layernorm_fwd(x2d, u.data(n.weight), u.data(n.bias), 1e-5)
        return h, (mean, rstd)

    def _norm_bwd(self, dh, ns):
        x2d, mean, rstd = ns
        u, n = self.unit, self.m.norm
        dx = _ln_bwd(u, n, dh, x2d, mean, rstd, None, self.rctx.accumulate)
        return dx


class GPTModel(BaseLM):
    def __init__(self, cfg, use_actv_ckpt=False, device=None):
        super().__init__(cfg, use_actv_ckpt)
        kw = dict(dtype=cfg["dtype"], device=device)
        self.tok_emb = nn.Embedding(cfg["vocab_size"], cfg["emb_dim"], **kw)
        self.pos_emb = nn.Embedding(cfg["context_length"], cfg["emb_dim"], **kw)
        self.drop_emb = nn.Dropout(cfg["drop_rate"])
        self.blocks = nn.Sequential(*[TransformerBlock(cfg, device) for _ in range(cfg["n_layers"])])
        self.norm = nn.LayerNorm(cfg["emb_dim"], **kw)
        self.output_head = nn.Linear(cfg["emb_dim"], cfg["vocab_size"], bias=False, **kw)
        self._register_state_dict_hook(_gpt_state_dict_hook)
        self._register_load_state_dict_pre_hook(_gpt_load_pre_hook)
        self.include_buffers_in_state_dict = True

    def build_computes(self):
        rc = self._rctx
        return ([GPTEmbedCompute(rc, self)]
                + [GPTBlockCompute(rc, b, i) for i, b in enumerate(self.blocks)]
                + [GPTHeadCompute(rc, self)])


def _gpt_state_dict_hook(module, state_dict, prefix, local_metadata):
    if getattr(module, "include_buffers_in_state_dict", False):
        T = module.cfg.context_length
        mask = torch.triu(torch.ones(T, T), diagonal=1)
        for i in range(module.cfg.n_layers):
            state_dict[f"{prefix}blocks.{i}.att.mask"] = mask
    return state_dict


def _gpt_load_pre_hook(state_dict, prefix, *args, **kwargs):
    for k in list(state_dict.keys()):
        if k.startswith(prefix) and k.endswith(".att.mask"):
            del state_dict[k]
