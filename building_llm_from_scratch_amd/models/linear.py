"""Fused (multi-)linear forward/backward on flat-unit views, with LoRA folded in.

A :class:`FusedLinear` covers one or more reference ``nn.Linear`` modules that share an
input (Q/K/V; gate/up) and whose weights are adjacent in the unit's flat buffer, so the
whole group is ONE GEMM ``y = x @ W_cat^T (+ b_cat) (+ residual)`` on hipBLASLt.  LoRA
members add ``scaling * (x @ A) @ B`` into their column slice of ``y`` in place.

Backward writes ``dW`` / ``db`` / ``dA`` / ``dB`` directly into the unit's flat gradient
buffer (``out=`` GEMMs; ``addmm_`` when accumulating micro-batches).

LoRA on the GPU runs on the fused kernels of csrc/lora.hip (reference lora.py:24-26,45-46),
a fixed number of launches per group however many members it has.  Two forms:
  * K-augmented (frozen, bias-free, unsharded base; ``kaug_input`` / ``forward_kaug``): the
    producer of x (RMSNorm, SwiGLU) writes it into [x | s t | 0], lora_down adds s t, and ONE
    GEMM computes y (+ residual) = [x | s t] . [W | Bd^T]^T; the dX GEMM on the cached
    [W^T ; Bd] returns [dx_W | dy B^T]; dB / dA by lora_wgrad, dx += s u P by lora_up;
  * grouped (everything else the kernels take):
      fwd  P = [A_1^T; A_2^T; ...] (pack), t = x P^T (lora_down), y[:, cols_m] += s t_m B_m (lora_up)
      bwd  u_m = dy[:, cols_m] B_m^T (lora_down), dB_m = s t_m^T dy[:, cols_m] and
           dA_m = s x^T u_m (lora_wgrad, into the flat gradient), dx += s u P (lora_up)
Groups the kernels cannot take (fp32, ranks not a multiple of 16, odd widths) use per-member
hipBLASLt GEMMs.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.nn as nn

from .. import ops

from .flat import FlatUnit
from .lora import LinearWithLoRA


@dataclass
class LinearSpec:
    module: nn.Module
    weight: nn.Parameter
    bias: Optional[nn.Parameter]
    lora_A: Optional[nn.Parameter] = None
    lora_B: Optional[nn.Parameter] = None
    scaling: float = 0.0

    @property
    def out_features(self) -> int:
        return self.weight.shape[0]


def resolve(mod: nn.Module) -> LinearSpec:
    if isinstance(mod, LinearWithLoRA):
        lin = mod.linear
        return LinearSpec(mod, lin.weight, lin.bias, mod.lora.A, mod.lora.B, mod.lora.scaling)
    assert isinstance(mod, nn.Linear), f"expected nn.Linear, got {type(mod)}"
    return LinearSpec(mod, mod.weight, mod.bias)


def layout_groups(specs: Sequence[LinearSpec]) -> List[List[nn.Parameter]]:
    """Fused layout: [all weights], [all biases], then each LoRA's A and B."""
    groups = [[s.weight for s in specs]]
    biases = [s.bias for s in specs if s.bias is not None]
    if biases:
        assert len(biases) == len(specs), "mixed bias / no-bias in a fused linear group"
        groups.append(biases)
    for s in specs:
        if s.lora_A is not None:
            groups.append([s.lora_A])
            groups.append([s.lora_B])
    return groups


def _mm_out(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, accumulate: bool):
    if accumulate:
        out.addmm_(a, b)
    else:
        torch.mm(a, b, out=out)


def weight_grad_splits(n_tokens: int, out_f: int, in_f: int) -> int:
    """Split-K factor for dW = dy^T x (K = tokens).  With 16k tokens and small projections
    (GPT-2 d=1280: 25-100 output tiles of 256x256 for 256 CUs) one GEMM leaves most of the chip
    idle for a 16k-deep K loop; splitting the tokens into S batched GEMMs and summing the
    partials measured 1.5-1.6x faster on MI355X (tools/bench_dw.py), and slower once the output
    alone fills the chip (Llama-3-8B, Llama-3.2-1B gate/up and down)."""
    tiles = -(-out_f // 256) * -(-in_f // 256)
    S = 8 if tiles <= 32 else 4 if tiles <= 128 else 1
    while S > 1 and (n_tokens % S or n_tokens // S < 1024):
        S //= 2
    return S


def _weight_grad(dy: torch.Tensor, x: torch.Tensor, gW: torch.Tensor, accumulate: bool):
    """gW[out, in] (+)= dy^T x.  Single GEMM: issued as gW^T = x^T dy into the transposed view
    (same memory; hipBLASLt then picks a kernel family that measured 3-6 % faster for the Llama
    projections, tools/bench_gemm.py).  Few output tiles: split-K over token chunks (batched
    GEMM into [S, out, in] partials + one deterministic fixed-order sum kernel)."""
    if not gW.is_cuda:
        _mm_out(dy.t(), x, gW, accumulate)
        return
    if ops.wgrad_gemm_enabled() and ops.wgrad_gemm_ok(dy, x, gW) \
            and ops.wgrad_gemm_preferred(gW.shape[0], gW.shape[1]):
        # token-major MFMA kernel (csrc/gemm_wgrad.hip): both operands consumed as stored,
        # transposed by the LDS read; split-K chosen by ops.wgrad_splits
        ops.wgrad_gemm_(dy, x, gW, accumulate)
        return
    N = x.shape[0]
    S = weight_grad_splits(N, gW.shape[0], gW.shape[1]) \
        if gW.is_contiguous() and dy.is_contiguous() and x.is_contiguous() else 1
    if S == 1:
        _mm_out(x.t(), dy, gW.t(), accumulate)
        return
    part = torch.bmm(dy.view(S, N // S, -1).transpose(1, 2), x.view(S, N // S, -1))   # [S, out, in]
    ops.sum_partials_(part, gW, accumulate)


DGRAD_WT_MIN_TOKENS = 8192  # below this the transpose costs more than the faster GEMM layout saves


def _dgrad_wt_ok(dy: torch.Tensor, W: torch.Tensor) -> bool:
    return (dy.is_cuda and ops.dgrad_wt_enabled() and W.dim() == 2 and W.dtype in (torch.bfloat16, torch.float16)
            and W.is_contiguous() and W.shape[0] % 8 == 0 and W.shape[1] % 8 == 0
            and dy.shape[0] >= DGRAD_WT_MIN_TOKENS)


# The forward-layout GEMMs (y = x W^T, dX on the transposed weight copy, the fused head's logits
# and dh).  GEMM_NT False = hipBLASLt / rocBLAS (default), True = csrc/gemm_nt.hip's persistent
# kernel wherever its shape rules hold (tests / A/B).  Round 5 measured the library GEMMs
# (TunableOp-picked per shape) 3-12 % faster on every Llama-3-8B and GPT-2 projection, and the
# epilogue fusions built on this kernel lost end to end (profiles/r5/fused_epilogues_ab.md).  A
# per-shape timed pick ("auto") was removed: a lazily timed pick differs between ranks whose
# batch shapes differ, and settling it needed a collective inside a cache miss.
GEMM_NT = False


def nt_choice(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> bool:
    """Whether mm_nt runs this call on csrc/gemm_nt.hip (else hipBLASLt)."""
    return GEMM_NT and ops.gemm_nt_ok(a, b, out)


def mm_nt(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a @ b^T for b stored [N, K] (both operands K-contiguous)."""
    if nt_choice(a, b, out):
        if out is None:
            out = torch.empty(a.shape[0], b.shape[0], dtype=a.dtype, device=a.device)
        ops.gemm_nt_(a, b, out, False)
        return out
    return torch.mm(a, b.t(), out=out) if out is not None else torch.mm(a, b.t())


def _input_grad(dy: torch.Tensor, W: torch.Tensor, dx_acc: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dx = dy @ W (+ dx_acc) [+ written into / added to ``out``].  GPU shapes the MFMA kernel
    takes (csrc/gemm_wgrad.hip, K-contiguous A) run there, else hipBLASLt."""
    nn_kernel = ops.dgrad_gemm_enabled() and ops.gemm_nn_ok(dy, W, out)
    if not nn_kernel and _dgrad_wt_ok(dy, W):
        # W^T scratch copy (HBM-bound, ~0.2 ms per Llama-3-8B layer) buys the K-contiguous
        # hipBLASLt layout for the GEMM (~1 ms per layer at 24k tokens)
        Wt = ops.transpose2d(W)
        if out is None and dx_acc is None and GEMM_NT and ops.gemm_nt_ok(dy, Wt):
            return mm_nt(dy, Wt)
        W = Wt.t()
    if out is not None:  # out += dy @ W
        if nn_kernel:
            ops.gemm_nn_(dy, W, out, True)
        else:
            out.addmm_(dy, W)
        return out
    if nn_kernel:
        if dx_acc is not None:
            dx = dx_acc.clone(memory_format=torch.contiguous_format)
            ops.gemm_nn_(dy, W, dx, True)
        else:
            dx = torch.empty(dy.shape[0], W.shape[1], dtype=dy.dtype, device=dy.device)
            ops.gemm_nn_(dy, W, dx, False)
        return dx
    return torch.addmm(dx_acc, dy, W) if dx_acc is not None else torch.mm(dy, W)


# tests set this to drive the grouped LoRA path through the CPU oracles of ops.reference
FORCE_GROUPED_LORA = False
LORA_KAUG = True   # zero-copy K-augmented LoRA projections (FusedLinear.forward_kaug)
# The forward epilogue fusions on csrc/gemm_nt.hip's persistent 4-wave kernel: gate/up GEMM +
# SwiGLU (FusedLinear.forward_swiglu), QKV GEMM + RoPE (forward_rope), GPT-2 c_fc GEMM + bias +
# GELU (forward_bias_gelu).  Off by default: the HBM pass each removes is worth less than what the
# kernel gives up against the TunableOp-picked library GEMM on MI355X (-0.8 / -0.17 / -3.8 % end
# to end, profiles/r5/fused_epilogues_ab.md).  ``use_gemm_epilogues(True)`` (CLI / bench
# ``--gemm_epilogues``) turns all three on.
FUSED_SWIGLU = False
FUSED_ROPE = False
FUSED_GELU = False


GEMM_EPILOGUES = ("swiglu", "rope", "gelu")


def use_gemm_epilogues(on=True) -> None:
    """Route the gate/up (``swiglu``), QKV (``rope``) and c_fc (``gelu``) projections through the
    fused-epilogue kernels: ``True`` / ``False`` for all three, or an iterable of names."""
    global FUSED_SWIGLU, FUSED_ROPE, FUSED_GELU
    names = set(GEMM_EPILOGUES) if on is True else set() if on is False or on is None else set(on)
    bad = names - set(GEMM_EPILOGUES)
    if bad:
        raise ValueError(f"unknown GEMM epilogue(s) {sorted(bad)}; choose from {GEMM_EPILOGUES}")
    FUSED_SWIGLU, FUSED_ROPE, FUSED_GELU = "swiglu" in names, "rope" in names, "gelu" in names


class FusedLinear:
    def __init__(self, modules: Sequence[nn.Module]):
        self.modules = list(modules)
        self.specs: List[LinearSpec] = []

    def refresh(self):
        self.specs = [resolve(m) for m in self.modules]
        return self

    def layout(self) -> List[List[nn.Parameter]]:
        self.refresh()
        return layout_groups(self.specs)

    def bind(self, unit: FlatUnit):
        self.unit = unit
        ws = [s.weight for s in self.specs]
        self.W_params = ws
        self.b_params = [s.bias for s in self.specs] if self.specs[0].bias is not None else None
        self.cols = []
        c = 0
        for s in self.specs:
            self.cols.append((c, c + s.out_features))
            c += s.out_features
        self.out_total = c
        self.has_lora = any(s.lora_A is not None for s in self.specs)
        lm = [(c, s) for c, s in zip(self.cols, self.specs) if s.lora_A is not None]
        self.lora_c0 = [c0 for (c0, _), _ in lm]
        self.lora_len = [c1 - c0 for (c0, c1), _ in lm]
        self.lora_r = [s.lora_A.shape[1] for _, s in lm]
        self.lora_off = [sum(self.lora_r[:i]) for i in range(len(lm))]
        self.lora_R = sum(self.lora_r)
        self.lora_specs = [s for _, s in lm]
        scales = {float(s.scaling) for s in self.lora_specs}
        self.lora_scale = scales.pop() if len(scales) == 1 else None

    def _grouped_lora(self, x: torch.Tensor) -> bool:
        return self._grouped_lora_dims(x.device, x.dtype, x.shape[1]) and x.dim() == 2 and x.shape[0] >= 1

    def _grouped_lora_dims(self, device, dtype, K: int) -> bool:
        if self.lora_scale is None or len(self.lora_specs) != len(self.specs):
            return False
        if FORCE_GROUPED_LORA:
            return True
        return ops.lora_kernel_ok_dims(device, dtype, self.lora_r, [K] + self.lora_len + self.lora_c0)

    def _kaug_base_ok(self) -> bool:
        """K-augmented LoRA (see forward_kaug) needs a frozen, bias-free base weight that is not
        sharded: the persistent [W | Bd^T] / [W^T ; Bd] copies would keep a full unsharded frozen
        weight per rank under a sharding FSDP engine (Llama-3-8B gate/up: ~7.5 GB regardless of
        world size) and would be rebuilt after every re-gather.  ``LORA_KAUG = False`` turns it off
        (tests / A/B)."""
        return (self.has_lora and self.b_params is None
                and not self.unit.trainable(self.W_params[0])
                and not self.unit.state.get("sharded", False)
                and LORA_KAUG)

    def kaug_input(self, like: torch.Tensor, K: int) -> Optional[torch.Tensor]:
        """An [N, K + R] buffer for a zero-copy K-augmented forward, or None: the caller's
        producer (RMSNorm, SwiGLU) writes this projection's input into its first K columns and
        ``forward_kaug`` adds the s t columns, so neither a copy of x nor a pass over y is paid."""
        if not (self._kaug_base_ok() and self._grouped_lora_dims(like.device, like.dtype, K)):
            return None
        return torch.empty(like.shape[0], K + self._kaug_pad(K), dtype=like.dtype, device=like.device)

    def _kaug_pad(self, K: int) -> int:
        """Columns after x: the R of s t, rounded up so that a row is a whole number of 128-byte
        lines (K + R = 2096 split every 64-column read of x over two lines: the dA pass ran 1.6x
        slower on it); the pad columns are zero in both operands."""
        return -(-(K + self.lora_R) // 64) * 64 - K

    def _waug(self, W: torch.Tensor, K: int):
        """([W | Bd^T] [out, K + R], [W^T ; Bd] [K + R, out]): member m's B_m^T in rows c0_m..,
        columns K + off_m.. of the first (and transposed in the second, the dX GEMM's
        K-contiguous operand).  Kept across calls: the frozen W parts are re-copied only when
        W's storage or version changed (a re-gather, a state-dict load); the B blocks (trained)
        are rewritten every call, one kernel each."""
        u = self.unit
        Rp = self._kaug_pad(K)
        key = (W.data_ptr(), W._version, W.shape, W.dtype)
        cached = getattr(self, "_wa_cache", None)
        if cached is not None and cached[0] == key:
            Wa, WaT = cached[1], cached[2]
        else:
            Wa = torch.empty(W.shape[0], K + Rp, dtype=W.dtype, device=W.device)
            Wa[:, :K].copy_(W)
            WaT = torch.empty(K + Rp, W.shape[0], dtype=W.dtype, device=W.device)
            WaT[:K].copy_(ops.transpose2d(W) if W.is_cuda else W.t())
            self._wa_cache = (key, Wa, WaT)
        Bs = [u.data(s.lora_B) for s in self.lora_specs]
        ops.lora_block_(Wa[:, K:], Bs, self.lora_c0, self.lora_off)
        ops.lora_block_(WaT[K:].t(), Bs, self.lora_c0, self.lora_off)
        return Wa, WaT

    def forward_kaug(self, xa: torch.Tensor, K: int, residual: Optional[torch.Tensor] = None):
        """K-augmented forward on ``xa`` = [x | .] (x already written by the producer):
        s t = s x A_cat goes into the last R columns, then ONE GEMM
        y (= residual +) [x | s t] . [W | Bd^T]^T — the rank-r update rides in the GEMM's K loop.
        Backward gets dy Bd = dy B^T from the dX GEMM the same way (``_kaug_lora_backward``)."""
        u = self.unit
        R = self.lora_R
        x = xa[:, :K]
        P = ops.lora_pack_t([u.data(s.lora_A) for s in self.lora_specs])          # [R, K]
        ops.lora_down_into(x, [P], [0], [K], [0], R, self.lora_scale, xa[:, K:])  # [s x A_cat | 0]
        Wa, WaT = self._waug(self.W(), K)
        y = ops.linear_residual(xa, Wa, residual) if residual is not None else mm_nt(xa, Wa)
        return y, ("kaug", xa[:, K:K + R], P, WaT)

    # views are re-fetched every call: FSDP may have re-materialised the storage
    def W(self):
        return self.unit.fused_data(self.W_params)

    def b(self):
        return self.unit.fused_data(self.b_params) if self.b_params else None

    # ------------------------------------------------------------------ fwd
    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None):
        W = self.W()
        b = self.b()
        if residual is not None:
            assert b is None
        if (residual is None and self.out_total >= 4 * x.shape[1] and self.has_lora
                and self._grouped_lora(x) and self._kaug_base_ok()):
            # an input no producer wrote into a K-augmented buffer (wide output: copying x costs
            # less than the s t B write plus the beta = 1 re-read of y it replaces)
            xa = self.kaug_input(x, x.shape[1])
            xa[:, :x.shape[1]].copy_(x)
            return self.forward_kaug(xa, x.shape[1])
        if self.has_lora and self._grouped_lora(x):
            # y = (residual | bias) + s t B, written by lora_up, then the base GEMM accumulates
            # onto it (beta = 1): the rank-r update costs no read-modify-write pass of y
            u = self.unit
            P = ops.lora_pack_t([u.data(s.lora_A) for s in self.lora_specs])          # [R, K]
            t = ops.lora_down(x, [P], [0], [x.shape[1]], [0], self.lora_R)            # x A_cat
            y = torch.empty(x.shape[0], self.out_total, dtype=x.dtype, device=x.device)
            ops.lora_up_(y, t, [u.data(s.lora_B) for s in self.lora_specs], self.lora_c0,
                         self.lora_off, self.lora_scale, base=residual, bias=b)
            y.addmm_(x, W.t())
            return y, ("grouped", t, P)
        if residual is not None:
            y = ops.linear_residual(x, W, residual)
        elif b is not None:
            y = torch.addmm(b, x, W.t())
        else:
            y = mm_nt(x, W)
        xa = None
        if self.has_lora:
            xa = []
            for (c0, c1), s in zip(self.cols, self.specs):
                if s.lora_A is None:
                    xa.append(None)
                    continue
                A = self.unit.data(s.lora_A)
                B = self.unit.data(s.lora_B)
                t = torch.mm(x, A)
                y[:, c0:c1].addmm_(t, B, alpha=s.scaling)
                xa.append(t)
        return y, xa

    def forward_swiglu(self, x: torch.Tensor):
        """Gate/up projection with the SwiGLU forward in the GEMM epilogue (``[fc1; fc2]``, no
        bias, no LoRA): returns ``(gu, act)`` or None when the fused kernel does not apply
        (csrc/gemm_nt.hip; only with ``use_gemm_epilogues(True)``)."""
        if self.has_lora or self.b_params is not None or len(self.specs) != 2 or not FUSED_SWIGLU:
            return None
        W = self.W()
        if not ops.gemm_nt_swiglu_ok(x, W):
            return None
        return ops.gemm_nt_swiglu(x, W)

    def forward_bias_gelu(self, x: torch.Tensor):
        """c_fc with its bias and the exact GELU in the GEMM epilogue (K9; no LoRA): returns
        ``(f, g)`` = (pre-activation, activation) or None when the fused kernel does not apply
        (only with ``use_gemm_epilogues(True)``) and the caller runs the GEMM + ``gelu_fwd``."""
        if self.has_lora or self.b_params is None or not FUSED_GELU:
            return None
        W, b = self.W(), self.b()
        if not ops.gemm_nt_bias_gelu_ok(x, W, b):
            return None
        return ops.gemm_nt_bias_gelu(x, W, b)

    def forward_rope(self, x: torch.Tensor, cos, sin, T: int, H: int, G: int, hd: int):
        """QKV projection with RoPE applied to the q and k heads in the GEMM epilogue (K4; no bias,
        no LoRA): returns the rotated qkv, or None when the fused kernel does not apply (head dim
        128 only; only with ``use_gemm_epilogues(True)``) and the caller runs the GEMM + ``rope_``."""
        if self.has_lora or self.b_params is not None or not FUSED_ROPE:
            return None
        W = self.W()
        if not ops.gemm_nt_rope_ok(x, W, hd) or W.shape[0] != (H + 2 * G) * hd:
            return None
        return ops.gemm_nt_rope(x, W, cos, sin, T, H, G, hd)

    def lora_state(self, x: torch.Tensor):
        """Only the LoRA intermediate ``x A`` that ``backward`` needs (what ``forward`` would
        return as its second value) without the base GEMM: the activation-checkpoint recompute
        of a block's LAST projection needs it, but never that projection's output."""
        if not self.has_lora:
            return None
        u = self.unit
        if self._grouped_lora(x):
            P = ops.lora_pack_t([u.data(s.lora_A) for s in self.lora_specs])
            return ("grouped", ops.lora_down(x, [P], [0], [x.shape[1]], [0], self.lora_R), P)
        return [torch.mm(x, u.data(s.lora_A)) if s.lora_A is not None else None for s in self.specs]

    # ------------------------------------------------------------------ bwd
    def bias_grad_buf(self) -> Optional[torch.Tensor]:
        """The flat gradient view of the fused bias (None: no bias or frozen); a caller that fills
        it itself passes ``bias_done=True`` to ``backward``."""
        return self.unit.fused_grad(self.b_params) if self.b_params is not None else None

    def backward(self, dy: torch.Tensor, x: torch.Tensor, xa, need_dx: bool = True,
                 accumulate: bool = False, dx_acc: Optional[torch.Tensor] = None, bias_done: bool = False,
                 lowrank_dx: bool = False, defer_lora_A: bool = False, lora_B_done: bool = False):
        """Returns dx (plus ``dx_acc`` if given) and writes parameter grads into the flat.
        ``lowrank_dx``: a K-augmented group may instead return ("lowrank", base, u, P, s, A_deferred)
        with dx = base + s u P left for the consumer to form (ops.swiglu_bwd_lowrank); with
        ``defer_lora_A`` that consumer also sums dA = s x^T u (A_deferred True: ops.swiglu_bwd_lowrank_wgrad).
        ``lora_B_done``: the caller already summed the K-augmented group's dB (same kernel)."""
        u = self.unit
        gW = u.fused_grad(self.W_params)
        if gW is not None:
            _weight_grad(dy, x, gW, accumulate)
        if self.b_params is not None and not bias_done:
            gb = u.fused_grad(self.b_params)
            if gb is not None:
                ops.bias_grad_(dy, gb, accumulate)
        if self.has_lora and isinstance(xa, tuple) and xa[0] == "kaug":
            return self._kaug_lora_backward(dy, x, xa[1], xa[2], xa[3], need_dx, dx_acc, accumulate, lowrank_dx,
                                            defer_lora_A, lora_B_done)
        if self.has_lora and isinstance(xa, tuple) and xa[0] == "grouped":
            return self._grouped_lora_backward(dy, x, xa[1], xa[2], need_dx, dx_acc, accumulate)
        dx = None
        if need_dx:
            dx = _input_grad(dy, self.W(), dx_acc)
        if self.has_lora:
            for (c0, c1), s, t in zip(self.cols, self.specs, xa):
                if s.lora_A is None:
                    continue
                A = u.data(s.lora_A)
                B = u.data(s.lora_B)
                dys = dy[:, c0:c1]
                dyB = torch.mm(dys, B.t())                                   # [N, r]
                gB = u.grad(s.lora_B)
                if gB is not None:
                    if accumulate:
                        gB.addmm_(t.t(), dys, alpha=s.scaling)
                    else:
                        torch.addmm(gB, t.t(), dys, beta=0, alpha=s.scaling, out=gB)
                gA = u.grad(s.lora_A)
                if gA is not None:
                    if accumulate:
                        gA.addmm_(x.t(), dyB, alpha=s.scaling)
                    else:
                        torch.addmm(gA, x.t(), dyB, beta=0, alpha=s.scaling, out=gA)
                if need_dx:
                    dx.addmm_(dyB, A.t(), alpha=s.scaling)
        return dx

    def input_grad(self, dy: torch.Tensor) -> torch.Tensor:
        """dx = dy W alone (no LoRA, no parameter grads): lets a caller run the dX GEMM before the
        dW GEMM whose input it is still producing (``backward(..., need_dx=False)`` then)."""
        assert not self.has_lora
        return _input_grad(dy, self.W())

    def _kaug_lora_backward(self, dy, x, st, P, WaT, need_dx, dx_acc, accumulate, lowrank_dx=False,
                            defer_A=False, B_done=False):
        """st = s t (the forward's augmented columns), WaT = [W^T ; Bd]."""
        u_ = self.unit
        sc = self.lora_scale
        K = x.shape[1]
        gB = [(u_.grad(s.lora_B), c0, off) for s, c0, off in zip(self.lora_specs, self.lora_c0, self.lora_off)]
        gB = [g for g in gB if g[0] is not None]
        if gB and not B_done:                                      # dB = s t^T dy = (s t)^T dy
            ops.lora_wgrad(st, dy, [g for g, _, _ in gB], [o for _, _, o in gB], [c for _, c, _ in gB], 1.0,
                           accumulate)
        dxa = mm_nt(dy, WaT)                                       # [dy W | dy Bd | 0] = [dx_W | dy B^T | 0]
        ub = dxa[:, K:K + self.lora_R]
        lowrank = need_dx and lowrank_dx and dx_acc is None and ops.swiglu_bwd_lowrank_ok(self.lora_R, K)
        defer = lowrank and defer_A
        gA = [(u_.grad(s.lora_A), off) for s, off in zip(self.lora_specs, self.lora_off)]
        gA = [g for g in gA if g[0] is not None]
        if gA and not defer:
            ops.lora_wgrad(ub, x, [g.t() for g, _ in gA], [o for _, o in gA], [0] * len(gA), sc, accumulate)
        if not need_dx:
            return None
        if lowrank:
            return ("lowrank", dxa[:, :K], ub, P, sc, defer)      # the consumer adds s u P (and dA)
        dx = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        ops.lora_up_(dx, ub, [P], [0], [0], sc, base=dxa[:, :K])  # dx_W + s (dy B^T) A_cat^T
        if dx_acc is not None:
            dx += dx_acc
        return dx

    def _grouped_lora_backward(self, dy, x, t, P, need_dx, dx_acc, accumulate):
        u_ = self.unit
        sc = self.lora_scale
        Bs = [u_.data(s.lora_B) for s in self.lora_specs]
        u = ops.lora_down(dy, Bs, self.lora_c0, self.lora_len, self.lora_off, self.lora_R)   # dy B^T
        gB = [(u_.grad(s.lora_B), c0, off) for s, c0, off in zip(self.lora_specs, self.lora_c0, self.lora_off)]
        gB = [g for g in gB if g[0] is not None]
        if gB:
            ops.lora_wgrad(t, dy, [g for g, _, _ in gB], [o for _, _, o in gB], [c for _, c, _ in gB], sc,
                           accumulate)
        gA = [(u_.grad(s.lora_A), off) for s, off in zip(self.lora_specs, self.lora_off)]
        gA = [g for g in gA if g[0] is not None]
        if gA:
            ops.lora_wgrad(u, x, [g.t() for g, _ in gA], [o for _, o in gA], [0] * len(gA), sc, accumulate)
        if not need_dx:
            return None
        # dx = dx_acc + s u A_cat^T (lora_up, write-only) then += dy W (beta = 1 GEMM)
        dx = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        ops.lora_up_(dx, u, [P], [0], [0], sc, base=dx_acc)
        return _input_grad(dy, self.W(), out=dx)
