"""Unit-structured language-model base.

The reference runs every model as a plain ``nn.Module`` forward under autograd (one graph
node per eager op, ``[B,H,T,T]`` scores materialised; reference GPT2.py:108-124,
Llama3.py:196-204).  Here a model is an ordered list of *units* (embedding -> blocks ->
final norm + head) and each unit is ONE autograd node whose forward/backward is written by
hand (models/gpt2.py, models/llama.py) on top of the HIP kernels and hipBLASLt GEMMs.  That
gives exact control over:

  * what each block saves for backward (``actv_ckpt``: ``none`` | ``selective`` — recompute
    only the norm outputs and the SwiGLU / GELU activation, the cheapest memory-bound ops (the
    activation is rebuilt inside the activation-backward pass, in place of its gradient, so it
    costs no extra pass); everything a GEMM or the attention kernel produced is kept, which
    288 GB of HBM affords | ``full`` — save the block input
    only, the reference's ``checkpoint_sequential(blocks, segments=n_layers)`` semantics
    (Llama3.py:199, GPT2.py:116): every block of the first ``segments - 1`` segments is
    recomputed in backward, the last segment runs without checkpointing.  ``ckpt_segments``
    (default n_layers, exactly the reference) trades recompute for memory; the recompute is
    per block either way, so only one block's activations are ever rebuilt at a time);
  * where distributed hooks fire (``engine.pre_forward/post_forward/pre_backward/
    post_backward`` per unit — FSDP gathers and reduce-scatters, DDP bucket all-reduce);
  * fused head + cross-entropy: ``model(idx, targets)`` returns the mean loss without
    keeping fp32 logits (``model(idx)`` still returns logits like the reference).
"""
from __future__ import annotations

from contextlib import contextmanager
from typing import List, Optional

import torch
import torch.nn as nn

from .flat import FlatUnit

DEFAULT_INIT_SEED = 123   # the reference's set_seed(123) (utils.py:55)


def unit_seed(seed: int, index: int) -> int:
    """Seed of unit ``index`` in a meta-built model's per-unit initialisation."""
    return (int(seed) * 1_000_003 + 7919 * (index + 1)) % (2 ** 63)


class LocalEngine:
    """No-op distributed engine (single process)."""

    world_size = 1
    rank = 0

    def __init__(self, model=None):
        self.model = model

    def pre_forward(self, unit):
        pass

    def post_forward(self, unit):
        pass

    def pre_backward(self, unit):
        pass

    def post_backward(self, unit):
        pass

    def finish_backward(self):
        pass

    @torch.no_grad()
    def load_full_state_dict(self, sd, strict: bool = True):
        return self.model.load_state_dict(sd, strict=strict)

    @contextmanager
    def params_resident(self):
        """Inference over many forwards (KV-cache decode): every unit's full parameters stay
        available for the duration (FSDP gathers them once instead of per forward)."""
        yield


class RunCtx:
    """Per-model mutable run state shared by all unit computes."""

    def __init__(self, cfg, actv_ckpt: str = "none"):
        self.cfg = cfg
        self.actv_ckpt = actv_ckpt
        self.ckpt_segments = None      # full mode: checkpoint_sequential segments (None = n_layers)
        # explicit per-block modes (the memory planner's choice, train/memplan.py); overrides
        # actv_ckpt / ckpt_segments when set
        self.block_modes: Optional[List[str]] = None
        self.training = True
        self.engine = LocalEngine()
        self.accumulate = False        # micro-batch gradient accumulation: add into grads
        # expected dloss of the next backward (the fp16 loss scale): the fused head + CE takes the
        # logit gradient during the forward at this scale and divides it out in backward
        self.loss_scale = 1.0
        self.grad_forward = False      # whether the current model forward builds a backward
        self.seed = 1234
        self._offset = 0
        self.rope = None               # (cos, sin) fp32 [T, hd/2] on device
        self.B = 1
        self.T = 1
        self.profile_hook = None
        # unit index -> HIP event recorded after that unit's optimizer update (the update
        # runs on a side stream, overlapped with the next forward; see train/optim.py)
        self.param_ready: dict = {}

    def block_mode(self, i: int) -> str:
        """Checkpoint mode of block ``i``.  ``full`` follows torch's checkpoint_sequential:
        segment size n // s, the first s - 1 segments checkpointed, the rest (the last segment
        plus the remainder) run plainly -- with s = n_layers only the last block is not."""
        if self.block_modes is not None:
            return self.block_modes[i]
        if self.actv_ckpt != "full":
            return self.actv_ckpt
        n = self.cfg.n_layers
        s = max(1, min(int(self.ckpt_segments or n), n))
        return "full" if i < (n // s) * (s - 1) else "none"

    def wait_param_ready(self, unit_index: int):
        ev = self.param_ready.pop(unit_index, None)
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)

    def sync_all_params(self):
        for k in list(self.param_ready):
            self.wait_param_ready(k)

    def reserve_offsets(self, n: int) -> int:
        base = self._offset
        self._offset += (n + 255) // 256 * 256
        return base

    @property
    def drop_p(self) -> float:
        return float(self.cfg.drop_rate) if self.training else 0.0


class UnitCompute:
    """Hand-written forward/backward of one unit over a :class:`FlatUnit`."""

    name = "unit"
    index = -1   # block index (blocks only)

    def __init__(self, rctx: RunCtx):
        self.rctx = rctx
        self.unit: Optional[FlatUnit] = None

    def layout(self) -> List[List[nn.Parameter]]:
        raise NotImplementedError

    def bind(self, unit: FlatUnit):
        self.unit = unit

    def forward(self, x, save: bool, replay=None):
        raise NotImplementedError

    def backward(self, dy, saved):
        raise NotImplementedError

    def infer(self, *args):
        """KV-cache inference step (see BaseLM.forward_cached)."""
        raise NotImplementedError


def cached_attention(qkv, B: int, t: int, pos: int, H: int, G: int, hd: int, kv, causal: bool = True):
    """Attention of ``t`` new tokens at positions ``pos..pos+t-1`` (packed qkv rows, RoPE
    already applied) against a per-block KV cache ``kv = (k, v)`` of [B, G, Tmax, hd]; the new
    keys/values are appended to the cache first.  Prefill from position 0 runs the flash kernel
    on the packed rows; single-token decode runs the HIP decode kernel over the cache."""
    from .. import ops
    kc, vc = kv
    rows = qkv.view(B, t, H + 2 * G, hd)
    kc[:, :, pos:pos + t].copy_(rows[:, :, H:H + G].transpose(1, 2))
    vc[:, :, pos:pos + t].copy_(rows[:, :, H + G:].transpose(1, 2))
    if pos == 0:
        return ops.flash_attn_fwd(qkv, B, t, H, G, hd, causal)[0]
    if t == 1:
        return ops.attn_decode(rows[:, 0, :H], kc, vc, pos + 1)
    # chunked continuation (t > 1 after a prefix): explicit masked attention over the cache
    L = pos + t
    q = rows[:, :, :H].transpose(1, 2).float()                                   # [B,H,t,hd]
    k = kc[:, :, :L].float().repeat_interleave(H // G, dim=1)                    # [B,H,L,hd]
    v = vc[:, :, :L].float().repeat_interleave(H // G, dim=1)
    sc = (q @ k.transpose(-1, -2)) / (hd ** 0.5)
    qpos = torch.arange(pos, L, device=qkv.device)[:, None]
    kpos = torch.arange(L, device=qkv.device)[None, :]
    sc = sc.masked_fill(kpos > qpos, float("-inf"))
    o = torch.softmax(sc, dim=-1) @ v                                            # [B,H,t,hd]
    return o.transpose(1, 2).reshape(B * t, H * hd).to(qkv.dtype)


# ---------------------------------------------------------------------------
# autograd nodes
# ---------------------------------------------------------------------------
class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, anchor, comp):
        eng = comp.rctx.engine
        eng.pre_forward(comp.unit)
        x, saved = comp.forward(idx, save=True)
        eng.post_forward(comp.unit)
        ctx.comp, ctx.saved = comp, saved
        return x

    @staticmethod
    def backward(ctx, dx):
        comp = ctx.comp
        eng = comp.rctx.engine
        eng.pre_backward(comp.unit)
        comp.backward(dx.contiguous(), ctx.saved)
        ctx.saved = None
        eng.post_backward(comp.unit)
        eng.finish_backward()
        return None, None, None


class _BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, comp):
        eng = comp.rctx.engine
        eng.pre_forward(comp.unit)
        full = comp.rctx.block_mode(comp.index) == "full"
        y, saved = comp.forward(x, save=not full)
        eng.post_forward(comp.unit)
        ctx.comp = comp
        ctx.saved = ("__recompute__", x, saved) if full else saved
        return y

    @staticmethod
    def backward(ctx, dy):
        comp = ctx.comp
        eng = comp.rctx.engine
        eng.pre_backward(comp.unit)
        saved = ctx.saved
        if isinstance(saved, tuple) and len(saved) == 3 and isinstance(saved[0], str) \
                and saved[0] == "__recompute__":
            _, x, replay = saved
            _, saved = comp.forward(x, save=True, replay=replay, recompute=True)
        dx = comp.backward(dy.contiguous(), saved)
        ctx.saved = None
        eng.post_backward(comp.unit)
        return dx, None


class _HeadLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, targets, comp):
        eng = comp.rctx.engine
        eng.pre_forward(comp.unit)
        loss, saved = comp.forward_loss(x, targets, save=True)
        eng.post_forward(comp.unit)
        ctx.comp, ctx.saved = comp, saved
        return loss

    @staticmethod
    def backward(ctx, dloss):
        comp = ctx.comp
        eng = comp.rctx.engine
        eng.pre_backward(comp.unit)
        dx = comp.backward_loss(dloss, ctx.saved)
        ctx.saved = None
        eng.post_backward(comp.unit)
        return dx, None, None


class _HeadLogitsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, comp):
        eng = comp.rctx.engine
        eng.pre_forward(comp.unit)
        logits, saved = comp.forward_logits(x, save=True)
        eng.post_forward(comp.unit)
        ctx.comp, ctx.saved = comp, saved
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        comp = ctx.comp
        eng = comp.rctx.engine
        eng.pre_backward(comp.unit)
        dx = comp.backward_logits(dlogits.contiguous(), ctx.saved)
        ctx.saved = None
        eng.post_backward(comp.unit)
        return dx, None


# ---------------------------------------------------------------------------
class BaseLM(nn.Module):
    """Common machinery for GPTModel / Llama models."""

    init_seed = DEFAULT_INIT_SEED   # seed of the per-unit init of a meta-built model

    def __init__(self, cfg, use_actv_ckpt=False):
        super().__init__()
        self.cfg = cfg
        mode = use_actv_ckpt if isinstance(use_actv_ckpt, str) else ("full" if use_actv_ckpt else "none")
        assert mode in ("none", "selective", "full"), mode
        self.use_actv_ckpt = mode != "none"
        object.__setattr__(self, "_rctx", RunCtx(cfg, mode))
        object.__setattr__(self, "_comps", None)
        object.__setattr__(self, "_anchor", None)

    # -- to be provided by subclasses ------------------------------------------------
    def build_computes(self) -> List[UnitCompute]:
        raise NotImplementedError

    # -- configuration -----------------------------------------------------------------
    @property
    def rctx(self) -> RunCtx:
        return self._rctx

    def set_actv_ckpt(self, mode: str, segments=None):
        assert mode in ("none", "selective", "full")
        self._rctx.actv_ckpt = mode
        self._rctx.ckpt_segments = segments
        self._rctx.block_modes = None
        self.use_actv_ckpt = mode != "none"

    def set_block_modes(self, modes: List[str]):
        """Per-block checkpoint modes (``none`` | ``selective`` | ``full`` for each block), e.g.
        the memory planner's choice (train/memplan.py): the first k blocks fully recomputed, the
        rest selective."""
        assert len(modes) == self.cfg.n_layers and all(m in ("none", "selective", "full") for m in modes)
        self._rctx.block_modes = list(modes)
        self._rctx.actv_ckpt = "full" if "full" in modes else ("selective" if "selective" in modes else "none")
        self.use_actv_ckpt = any(m != "none" for m in modes)

    def ckpt_summary(self) -> dict:
        """How many blocks run in each checkpoint mode."""
        modes = [self._rctx.block_mode(i) for i in range(self.cfg.n_layers)]
        return {m: modes.count(m) for m in ("full", "selective", "none")}

    def set_engine(self, engine):
        self._rctx.engine = engine

    def train(self, mode: bool = True):
        super().train(mode)
        self._rctx.training = mode
        return self

    @property
    def device(self):
        return next(self.parameters()).device

    @property
    def units(self) -> List[FlatUnit]:
        self._ensure_flat()
        return [c.unit for c in self._comps]

    @property
    def computes(self) -> List[UnitCompute]:
        self._ensure_flat()
        return self._comps

    # -- flat storage ------------------------------------------------------------------
    def flatten(self, device=None, dtype=None, pad_to: int = 1, grad_dtype=None, arena=None, on_unit=None,
                init_seed: Optional[int] = None):
        """(Re)build every unit's flat buffers from the current parameters (call after
        LoRA replacement / weight loading; idempotent).  ``arena`` (optional) maps a unit
        index to ``(param_view, grad_view)`` slices of model-wide contiguous buffers that the
        trainable flat must live in (DDP / ZeRO buckets).

        A model built on the ``meta`` device has no values yet: each unit is initialised right
        after its flat is allocated, by its modules' own ``reset_parameters`` under a seed
        derived from ``init_seed`` and the unit index (``init_unit_``) — the same values on every
        rank, with no broadcast.  ``on_unit(unit)`` runs after each unit is built, BEFORE the
        next one is allocated: FSDP shards and frees the unit there, so a rank never holds
        more than one unit at full size."""
        p0 = next(self.parameters())
        meta = any(p.is_meta for p in self.parameters())
        device = torch.device(device) if device is not None else p0.device
        dtype = dtype or p0.dtype
        comps = self.build_computes()
        for i, c in enumerate(comps):
            u = FlatUnit(c.name, i)
            ts, gs = (arena[i] if arena is not None and i in arena else (None, None))
            u.flatten(c.layout(), device, dtype, pad_to=pad_to, grad_dtype=grad_dtype,
                      train_storage=ts, train_grad_storage=gs)
            c.bind(u)
            if meta and device.type != "meta":   # (meta -> meta: shape-only plans, no values)
                self.init_unit_(u, self.init_seed if init_seed is None else init_seed)
            if on_unit is not None:
                on_unit(u)
        object.__setattr__(self, "_comps", comps)
        object.__setattr__(self, "_anchor", torch.zeros((), device=device, requires_grad=True))
        self._after_flatten(device)
        return self

    def _after_flatten(self, device):
        pass

    @torch.no_grad()
    def init_unit_(self, unit: FlatUnit, seed: int = None):
        """Seeded in-place initialisation of one unit's parameters: every module owning one of
        them runs its ``reset_parameters`` (nn.Linear / nn.Embedding / nn.LayerNorm defaults,
        RMSNorm ones, LoRA kaiming A / zero B), in module order, under
        ``torch.manual_seed(unit_seed(seed, unit.index))``.  Deterministic per (seed, unit), so
        every rank computes the same values for the units it shards."""
        seed = self.init_seed if seed is None else seed
        ids = {id(p) for fb in unit.buffers() for p in fb.params}
        # the unit seed must not leak into the caller's streams (dropout, sampling, shuffling
        # continue from where they were): fork the CPU RNG and the device's own
        devs = [p.device for fb in unit.buffers() for p in fb.params if p.device.type == "cuda"][:1]
        with torch.random.fork_rng(devices=devs, device_type="cuda"):
            torch.manual_seed(unit_seed(seed, unit.index))
            for mod in self.modules():
                own = [p for p in mod.parameters(recurse=False) if id(p) in ids]
                if not own:
                    continue
                if not hasattr(mod, "reset_parameters"):
                    raise TypeError(f"{type(mod).__name__} has no reset_parameters: cannot initialise a "
                                    "meta-built model")
                mod.reset_parameters()

    def _ensure_flat(self):
        if self._comps is None:
            self.flatten()

    def _apply(self, fn, *args, **kwargs):
        # .to()/.cuda() on a flattened model: move, then rebuild flats on the new device
        was_flat = self._comps is not None
        r = super()._apply(fn, *args, **kwargs)
        if was_flat:
            object.__setattr__(self, "_comps", None)
            self.flatten()
        return r

    # -- forward -----------------------------------------------------------------------
    def forward(self, in_idx: torch.Tensor, targets: Optional[torch.Tensor] = None,
                last_only: bool = False):
        self._ensure_flat()
        comps = self._comps
        rc = self._rctx
        B, T = in_idx.shape
        rc.B, rc.T = B, T
        idx = in_idx.to(self._anchor.device, non_blocking=True)
        grad = torch.is_grad_enabled()
        rc.grad_forward = grad          # engines read this: inside autograd.Function.forward grad is off
        emb, blocks, head = comps[0], comps[1:-1], comps[-1]
        eng = rc.engine
        wait = rc.wait_param_ready if rc.param_ready else (lambda i: None)
        if grad:
            wait(emb.unit.index)
            x = _EmbedFn.apply(idx, self._anchor, emb)
            for c in blocks:
                wait(c.unit.index)
                x = _BlockFn.apply(x, c)
            wait(head.unit.index)
            if targets is not None:
                tg = targets.to(self._anchor.device, non_blocking=True).reshape(-1)
                return _HeadLossFn.apply(x, tg, head)
            logits = _HeadLogitsFn.apply(x, head)
            return logits.view(B, T, -1)
        # inference path: no autograd nodes, nothing saved
        with torch.no_grad():
            for c in comps[:-1]:
                wait(c.unit.index)
                eng.pre_forward(c.unit)
                x, _ = c.forward(idx if c is emb else x, save=False)
                eng.post_forward(c.unit)
            wait(head.unit.index)
            eng.pre_forward(head.unit)
            if targets is not None:
                tg = targets.to(self._anchor.device, non_blocking=True).reshape(-1)
                loss, _ = head.forward_loss(x, tg, save=False)
                eng.post_forward(head.unit)
                return loss
            if last_only:
                x = x.view(B, T, -1)[:, -1, :].contiguous()
                logits, _ = head.forward_logits(x, save=False)
                eng.post_forward(head.unit)
                return logits.view(B, 1, -1)
            logits, _ = head.forward_logits(x, save=False)
            eng.post_forward(head.unit)
            return logits.view(B, T, -1)

    # -- KV-cache inference -------------------------------------------------------------
    def new_kv_cache(self, B: int, max_len: int):
        """Per-block (K, V) caches [B, G, max_len, hd] in the parameter dtype."""
        self._ensure_flat()
        cfg = self.cfg
        G = cfg.n_kv_groups if cfg.is_llama else cfg.n_heads
        p = self._comps[1].unit
        dev, dt = self._anchor.device, (p.train.dtype if p.train is not None else p.frozen.dtype)
        return [(torch.empty(B, G, max_len, cfg.head_dim, device=dev, dtype=dt),
                 torch.empty(B, G, max_len, cfg.head_dim, device=dev, dtype=dt))
                for _ in range(len(self._comps) - 2)]

    @torch.no_grad()
    def forward_cached(self, idx: torch.Tensor, cache, pos: int) -> torch.Tensor:
        """Run ``idx`` [B, t] (positions ``pos..pos+t-1``) through the model, appending to
        ``cache``; returns the last position's logits [B, V].  Call inside
        ``engine.params_resident()`` (FSDP) — see train/generate.py:generate_cached."""
        self._ensure_flat()
        comps, rc = self._comps, self._rctx
        rc.sync_all_params()
        B, t = idx.shape
        idx = idx.to(self._anchor.device)
        x = comps[0].infer(idx, pos)
        for c, kv in zip(comps[1:-1], cache):
            x = c.infer(x, B, t, pos, kv)
        return comps[-1].infer(x, B, t)

    def decode_graph_ok(self, cache) -> bool:
        """Whether :meth:`forward_cached_dev` runs on this model / cache (GPU, bf16/fp16, head
        dim 64/128, cache <= 8192 positions)."""
        dev = self._anchor.device if self._anchor is not None else torch.device("cpu")
        kc = cache[0][0]
        return (dev.type == "cuda" and kc.dtype in (torch.bfloat16, torch.float16)
                and self.cfg.head_dim in (64, 128) and kc.shape[2] <= 8192)

    @torch.no_grad()
    def forward_cached_dev(self, idx: torch.Tensor, cache, pos_t: torch.Tensor) -> torch.Tensor:
        """One decode token per row (idx [B, 1]) at the position held in ``pos_t`` (int32 on the
        device): no host-side position, no host sync, so the whole step can be captured in a HIP
        graph once and replayed per token (train/generate.py)."""
        comps = self._comps
        x = comps[0].infer_dev(idx, pos_t)
        for c, kv in zip(comps[1:-1], cache):
            x = c.infer_dev(x, pos_t, kv)
        return comps[-1].infer(x, idx.shape[0], 1)

    def sync_params(self):
        """Make the current stream wait for every in-flight (overlapped) optimizer update."""
        self._rctx.sync_all_params()
        eng = self._rctx.engine
        if hasattr(eng, "sync"):
            eng.sync()

    def state_dict(self, *args, **kwargs):
        self.sync_params()
        return super().state_dict(*args, **kwargs)

    # -- parameter groups for optimizers -----------------------------------------------
    def trainable_buffers(self):
        self._ensure_flat()
        return [c.unit.train for c in self._comps if c.unit.train is not None]
