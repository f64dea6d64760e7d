"""Op dispatch: GPU tensors -> hand-written HIP kernels (``torch.ops.bllm.*`` from the
in-tree ``_C.so``), CPU tensors -> ``ops.reference`` (plain PyTorch).

There is deliberately NO silent fallback for GPU tensors: if the extension is not built,
every op on a GPU tensor raises (fp32 attention included: csrc/attn_f32.hip).

Kernel debug mode (``BLLM_KERNEL_DEBUG=1`` with ``tools/build_ext.py --debug``): every
``torch.ops.bllm`` call is followed by a device synchronisation and a read of the kernels'
debug word, so a failed device-side check (token id / CE target / decode position out of
range, common.h ``BLLM_DASSERT``) raises at the op that caused it, like a launch-blocking run.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from . import reference as ref
from ._ext import ext_available, kernel_debug, load_ext

__all__ = [
    "rmsnorm_fwd", "rmsnorm_bwd", "layernorm_fwd", "layernorm_bwd", "dropout_add", "dropout_bwd",
    "dropout_add_layernorm",
    "rope_", "rope_tables", "flash_attn_fwd", "flash_attn_bwd", "swiglu_fwd", "swiglu_bwd", "swiglu_bwd_act",
    "swiglu_bwd_lowrank_wgrad", "swiglu_bwd_lowrank_wgrad_ok",
    "gelu_fwd", "gelu_bwd", "gelu_bwd_bias", "gelu_bwd_act", "dropout_bwd_bias", "ce_fwd", "ce_bwd_", "embedding_fwd", "embedding_bwd",
    "sq_norm_multi", "adamw_step_", "attn_decode", "bias_grad_", "ext_available", "load_ext", "attention_backend",
    "lora_down", "lora_up_", "lora_wgrad", "lora_pack_t", "lora_kernel_ok", "lora_kernel_ok_dims",
    "lora_down_into", "lora_block_", "rmsnorm_fwd_into", "swiglu_fwd_into", "sum_partials_",
    "wgrad_gemm_", "wgrad_gemm_ok", "wgrad_gemm_enabled", "wgrad_gemm_preferred", "wgrad_splits",
    "gemm_nn_", "gemm_nt_", "gemm_nn_ok", "dgrad_gemm_enabled", "transpose2d", "dgrad_wt_enabled", "attn_keep_mask",
]

rope_tables = ref.rope_tables


def _hip(t: torch.Tensor) -> bool:
    if t.device.type == "cuda":
        load_ext(required=True)
        return True
    return False


DEBUG_CODES = {1: "embedding token id outside [0, vocab)", 2: "cross-entropy target outside [0, V)",
               3: "decode cache position outside [0, Tmax)", 4: "rope device position negative"}


class _CheckedOps:
    """torch.ops.bllm with a synchronise + device-check after every call (kernel debug mode)."""

    def __getattr__(self, name):
        op = getattr(torch.ops.bllm, name)

        def call(*args, **kwargs):
            out = op(*args, **kwargs)
            torch.cuda.synchronize()
            code = torch.ops.bllm.debug_error()
            if code:
                raise RuntimeError(f"bllm kernel check failed in {name}: {DEBUG_CODES.get(code, code)}")
            return out
        return call


_CHECKED = _CheckedOps()


def _k():
    return _CHECKED if kernel_debug() else torch.ops.bllm


# --------------------------------------------------------------------------- norms
def rmsnorm_fwd(x, w, eps: float):
    if _hip(x):
        return _k().rmsnorm_fwd(x, w, eps)
    return ref.rmsnorm_fwd(x, w, eps)


def rmsnorm_fwd_into(x, w, eps: float, y):
    """rmsnorm_fwd written into ``y``, a row-strided [N, d] view (the x part of a K-augmented
    LoRA operand) -> (y, rstd)."""
    if _hip(x):
        return y, _k().rmsnorm_fwd_into_(x, w, eps, y)
    out, rstd = ref.rmsnorm_fwd(x, w, eps)
    y.copy_(out)
    return y, rstd


def _vec_into(out, g32, accumulate):
    if out is None:
        return g32
    if accumulate:
        out.add_(g32.to(out.dtype))
    else:
        out.copy_(g32)
    return out


def rmsnorm_bwd(dy, x, w, rstd, dx_acc: Optional[torch.Tensor] = None, dw_out: Optional[torch.Tensor] = None,
                accumulate: bool = False):
    """-> (dx [+ dx_acc], dW).  With ``dw_out`` the weight gradient is written (or added, when
    ``accumulate``) straight into it by the reduction kernel, in its dtype."""
    if _hip(x):
        return _k().rmsnorm_bwd(dy, x, w, rstd, dx_acc, dw_out, bool(accumulate))
    dx, dw = ref.rmsnorm_bwd(dy, x, w, rstd, dx_acc)
    return dx, _vec_into(dw_out, dw, accumulate)


def layernorm_fwd(x, w, b, eps: float):
    if _hip(x):
        return _k().layernorm_fwd(x, w, b, eps)
    return ref.layernorm_fwd(x, w, b, eps)


def layernorm_bwd(dy, x, w, mean, rstd, dx_acc: Optional[torch.Tensor] = None,
                  dw_out: Optional[torch.Tensor] = None, db_out: Optional[torch.Tensor] = None,
                  accumulate: bool = False):
    if _hip(x) and (dw_out is None) == (db_out is None):
        return _k().layernorm_bwd(dy, x, w, mean, rstd, dx_acc, dw_out, db_out, bool(accumulate))
    if _hip(x):  # only one of the two outputs requested (e.g. a frozen bias)
        dx, dw, db = _k().layernorm_bwd(dy, x, w, mean, rstd, dx_acc, None, None, False)
    else:
        dx, dw, db = ref.layernorm_bwd(dy, x, w, mean, rstd, dx_acc)
    return dx, _vec_into(dw_out, dw, accumulate), _vec_into(db_out, db, accumulate)


def dropout_add(x, a, p: float, seed: int, offset: int):
    if _hip(x):
        return _k().dropout_add(x, a, float(p), int(seed), int(offset))
    return ref.dropout_add(x, a, p, seed, offset)


def dropout_add_layernorm(x, a, w, b, eps: float, p: float, seed: int, offset: int):
    """x2 = x + dropout(a) and (y, mean, rstd) = layernorm_fwd(x2) in one pass over the rows ->
    (x2, y, mean, rstd); bitwise ``dropout_add`` followed by ``layernorm_fwd``."""
    if _hip(x):
        return _k().dropout_add_layernorm(x, a, w, b, float(eps), float(p), int(seed), int(offset))
    x2 = ref.dropout_add(x, a, p, seed, offset)
    return (x2,) + tuple(ref.layernorm_fwd(x2, w, b, eps))


def dropout_bwd(dy, p: float, seed: int, offset: int):
    if p <= 0.0:
        return dy
    if _hip(dy):
        return _k().dropout_bwd(dy, float(p), int(seed), int(offset))
    return ref.dropout_bwd(dy, p, seed, offset)


def _bwd_bias_ok(t: torch.Tensor) -> bool:
    return _hip(t) and t.dim() == 2 and t.is_contiguous() and t.shape[1] * t.element_size() % 16 == 0


def dropout_bwd_bias(dy, p: float, seed: int, offset: int, db, accumulate: bool = False):
    """``dropout_bwd(dy)`` and db (+)= its column sums, in one pass over dy (the output bitwise
    ``dropout_bwd``'s; the sums as ``bias_grad_`` of it, same bands and order)."""
    if p > 0.0 and _bwd_bias_ok(dy):
        return _k().bwd_bias_grad_(dy, None, db, bool(accumulate), 0, float(p), int(seed), int(offset), False)
    d = dropout_bwd(dy, p, seed, offset)
    bias_grad_(d, db, accumulate)
    return d


def gelu_bwd_bias(f, dg, db, accumulate: bool = False):
    """``gelu_bwd(f, dg)`` and db (+)= its column sums, in one pass."""
    if _bwd_bias_ok(dg) and f.is_contiguous():
        return _k().bwd_bias_grad_(dg, f, db, bool(accumulate), 1, 0.0, 0, 0, False)
    d = gelu_bwd(f, dg)
    bias_grad_(d, db, accumulate)
    return d


def gelu_bwd_act(f, dg, db=None, accumulate: bool = False):
    """``gelu_bwd(f, dg)`` (returned; db (+)= its column sums if given) and ``dg`` overwritten in
    place with g = gelu(f), bitwise ``gelu_fwd(f)``: the activation-checkpoint recompute of a
    GPT-2 block then runs no GELU forward for the c_proj weight gradient."""
    if _bwd_bias_ok(dg) and f.is_contiguous():
        return _k().bwd_bias_grad_(dg, f, db, bool(accumulate), 1, 0.0, 0, 0, True)
    d = gelu_bwd(f, dg)
    if db is not None:
        bias_grad_(d, db, accumulate)
    dg.copy_(gelu_fwd(f))
    return d


# --------------------------------------------------------------------------- rope / attention
def rope_(qkv, cos, sin, T: int, H: int, G: int, hd: int, inverse: bool = False, pos_offset: int = 0):
    if _hip(qkv):
        _k().rope_(qkv, cos, sin, T, H, G, hd, inverse, pos_offset)
        return qkv
    return ref.rope_(qkv, cos, sin, T, H, G, hd, inverse, pos_offset)


def attention_backend(dtype: torch.dtype, device_type: str = "cuda") -> str:
    """Every GPU dtype runs a flash kernel (bf16/fp16: attn_mfma.hip; fp32: attn_f32.hip on the
    f32 MFMA; other head dims: attn_naive.hip) -- [B,H,T,T] is never materialised."""
    if device_type != "cuda":
        return "reference"
    return "hip" if dtype in (torch.bfloat16, torch.float16, torch.float32) else "reference"


def attn_keep_mask(qkv, B: int, T: int, H: int, hd: int, dropout_p: float):
    """Buffer for the attention-dropout keep bits (int32 [B*H, ceil(T/32), T]) that the forward
    kernel fills and the backward kernels read instead of re-hashing every (query, key), or None
    where the kernels hash (no dropout, fp32, CPU, head dims without MFMA kernels)."""
    if dropout_p <= 0.0 or qkv.device.type != "cuda" or qkv.dtype not in (torch.bfloat16, torch.float16) \
            or hd not in (64, 128):
        return None
    return torch.empty(B * H, (T + 31) // 32, T, dtype=torch.int32, device=qkv.device)


def flash_attn_fwd(qkv, B, T, H, G, hd, causal=True, dropout_p=0.0, seed=0, offset=0, keep_mask=None):
    if qkv.device.type == "cuda" and qkv.dtype in (torch.bfloat16, torch.float16, torch.float32):
        load_ext(required=True)
        return _k().flash_attn_fwd(qkv, B, T, H, G, hd, causal, float(dropout_p), int(seed), int(offset),
                                   keep_mask)
    return ref.flash_attn_fwd(qkv, B, T, H, G, hd, causal, dropout_p, seed, offset)


def rope_dev_(qkv, cos, sin, H: int, G: int, hd: int, pos_t):
    """RoPE of one decode token per row at the position stored in ``pos_t`` (int32, device)."""
    load_ext(required=True)
    _k().rope_dev_(qkv, cos, sin, H, G, hd, pos_t)
    return qkv


def attn_decode_append(qkv, kc, vc, pos_t, H: int, G: int):
    """Append the rows' new K/V to the caches at ``pos_t`` and attend over pos + 1 keys."""
    load_ext(required=True)
    return _k().attn_decode_append(qkv, kc, vc, pos_t, H, G)


def bias_grad_(dy, db, accumulate: bool = False):
    """db (+)= dy.sum(0) (fp32 accumulation, deterministic)."""
    if _hip(dy) and dy.shape[1] * dy.element_size() % 16 == 0:
        _k().bias_grad_(dy.contiguous(), db, bool(accumulate))
        return db
    s = dy.sum(0, dtype=torch.float32)
    if accumulate:
        db.add_(s.to(db.dtype))
    else:
        db.copy_(s)
    return db


WGRAD_TILE, WGRAD_KGRAN = 256, 128


# weight gradients on the token-major MFMA dW kernel (1.28-1.44 PF vs hipBLASLt's 0.96-1.17 on
# that layout, profiles/r5/gemm_pmc/README.md); False routes them to hipBLASLt (tests / A/B)
WGRAD_GEMM = True


def wgrad_gemm_enabled() -> bool:
    return WGRAD_GEMM


def wgrad_gemm_ok(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor) -> bool:
    """Shapes/layouts the token-major MFMA dW kernel (csrc/gemm_wgrad.hip) takes: a [K, M],
    b [K, N], c [M, N] with M, N multiples of 256, K of 128, 16-B aligned unit-stride rows."""
    if not (a.is_cuda and a.dtype in (torch.bfloat16, torch.float16) and b.dtype == a.dtype):
        return False
    K, M = a.shape
    N = b.shape[1]
    return (M % WGRAD_TILE == 0 and N % WGRAD_TILE == 0 and K % WGRAD_KGRAN == 0 and K >= WGRAD_KGRAN
            and a.stride(1) == 1 and b.stride(1) == 1 and c.stride(1) == 1
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)


WGRAD_MAX_TILES = 1 << 30


def wgrad_gemm_preferred(M: int, N: int) -> bool:
    """Whether the MFMA dW kernel beats hipBLASLt for an [M, N] weight gradient.  Measured on
    MI355X at 16k tokens, interleaved in one process (tools/bench_wgrad.py,
    profiles/r1_wgrad_kernel.md), default schedule: 1.28-1.40 PF on the Llama-3-8B projections
    and 1.34 PF on the 128k-vocab LM head (1.09-1.33x hipBLASLt), 1.06-1.42 PF on Llama-3.2-1B
    (1.15-1.44x) and 0.85-1.16 PF with split-K on GPT-2 (1.9-2.3x) — every measured shape, so the
    cap only exists as a knob for future shapes."""
    return (M // WGRAD_TILE) * (N // WGRAD_TILE) <= WGRAD_MAX_TILES


def wgrad_splits(M: int, N: int, K: int, n_cu: int = 256) -> int:
    """Split-K factor for the dW kernel: one 256x256 tile per CU at a time, so a GEMM with few
    tiles (GPT-2: 25-100) or a ragged last wave leaves CUs idle.  Pick S minimising
    compute / wave-utilisation + the fp32 partial round trip (S * M * N * 8 B through HBM)."""
    tiles = (M // WGRAD_TILE) * (N // WGRAD_TILE)
    best, best_t = 1, None
    for S in range(1, 9):
        if S > K // WGRAD_KGRAN or (S > 1 and K // S < 1024):
            break
        work = tiles * S
        util = work / (n_cu * -(-work // n_cu))
        t = 2.0 * M * N * K / (1.3e15 * util)
        if S > 1:
            t += (S * M * N * 8 + M * N * 4) / 4.5e12 + 6e-6
        if best_t is None or t < best_t * 0.97:
            best, best_t = S, t
    return best


# False: a ragged last wave is always handled by splitting every tile (A/B only)
WGRAD_TAIL = True


def wgrad_plan(M: int, N: int, K: int, n_cu: int = 256):
    """("split", S) or ("tail", full, St) for the dW kernel.  Splitting EVERY tile S ways evens out a
    ragged last wave but round-trips S fp32 copies of the whole [M, N] through HBM (Llama-3-8B
    down projection: 896 tiles = 3.5 waves, S = 2 moves 1.2 GB).  The tail plan runs the whole
    waves [0, full) at full K straight into the output and splits only the ragged tail St ways into
    compact fp32 partials: the same wave count, 1/7 of the partial traffic there."""
    tiles = (M // WGRAD_TILE) * (N // WGRAD_TILE)
    S = wgrad_splits(M, N, K, n_cu)
    if S == 1 or not WGRAD_TAIL:
        return ("split", S)
    base = 2.0 * M * N * K / 1.3e15                         # s, every CU busy
    wave_t = base * n_cu / tiles                            # one wave of whole-K tiles
    util = tiles * S / (n_cu * -(-(tiles * S) // n_cu))
    best, best_t = ("split", S), base / util + (S * M * N * 8 + M * N * 4) / 4.5e12 + 6e-6
    full = tiles // n_cu * n_cu
    tail = tiles - full
    if full == 0 or tail == 0:
        return best
    for St in range(2, 9):
        if St > K // WGRAD_KGRAN or K // St < 1024:
            break
        t = (full // n_cu) * wave_t + -(-(tail * St) // n_cu) * wave_t / St
        t += (St * tail * WGRAD_TILE * WGRAD_TILE * 8 + tail * WGRAD_TILE * WGRAD_TILE * 4) / 4.5e12 + 12e-6
        if t < best_t * 0.99:
            best, best_t = ("tail", full, St), t
    return best


def wgrad_gemm_(a, b, c, accumulate: bool = False, splits: Optional[int] = None):
    """c (+)= a^T b with a [K, M], b [K, N] token-major (dW = dY^T X), fp32 accumulation."""
    if _hip(a):
        plan = wgrad_plan(a.shape[1], b.shape[1], a.shape[0]) if splits is None else ("split", int(splits))
        if plan[0] == "tail" and c.stride(1) == 1 and c.stride(0) % 8 == 0 and c.data_ptr() % 16 == 0:
            _k().wgrad_gemm_tail_(a, b, c, bool(accumulate), plan[1], plan[2])
        else:
            S = plan[1] if plan[0] == "split" else wgrad_splits(a.shape[1], b.shape[1], a.shape[0])
            _k().wgrad_gemm_(a, b, c, bool(accumulate), S)
        return c
    r = a.float().t() @ b.float()
    if accumulate:
        r += c.float()
    c.copy_(r)
    return c


# input gradients (dX = dY W) on the MFMA kernel (``gemm_nn_``) instead of hipBLASLt: off, measured
# at parity on the benchmark shapes (0.95-1.05x, tools/bench_dgrad.py, profiles/r1_wgrad_kernel.md)
# -- hipBLASLt's dX family is already at 1.25-1.38 PF, unlike its dW family the kernel was written
# for.  The kernel stays a public op (``gemm_nn_``); tests flip this to route the backward through it.
DGRAD_GEMM = False


def dgrad_gemm_enabled() -> bool:
    return DGRAD_GEMM


_LT_RESIDUAL = True   # False: torch.addmm instead of the C != D hipBLASLt epilogue (tests / A/B)


def linear_residual(x: torch.Tensor, W: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
    """``C + x @ W^T`` as one hipBLASLt matmul that reads C in its epilogue and writes a new D
    (csrc/binding.cpp linear_residual).  ``torch.addmm(C, x, W.t())`` copies C into the output
    first (one extra HBM pass of C)."""
    if (_LT_RESIDUAL and _hip(x) and x.dtype in (torch.bfloat16, torch.float16) and W.dtype == x.dtype
            and C.dtype == x.dtype and x.is_contiguous() and W.is_contiguous() and C.is_contiguous()):
        return _k().linear_residual(x, W, C)
    return torch.addmm(C, x, W.t())


def transpose2d(a: torch.Tensor) -> torch.Tensor:
    """Contiguous a^T for a 2-D 16-bit tensor (csrc/elementwise.hip transpose16_k: 64x64 LDS
    tiles, 16-byte loads and stores); dims must be multiples of 8."""
    if _hip(a):
        return _k().transpose2d(a)
    return a.t().contiguous()


# large input-gradient GEMMs dX = dY W first transpose W into a scratch copy so hipBLASLt runs
# dX = dY (W^T)^T with both operands K-contiguous -- the same fast layout as the forward x W^T
# (tools/bench_gemm.py: 1.52-1.59 PF vs 1.30-1.38 PF for the dY W layout)
DGRAD_WT = True


def dgrad_wt_enabled() -> bool:
    return DGRAD_WT


def gemm_nn_ok(a: torch.Tensor, b: torch.Tensor, c: Optional[torch.Tensor] = None) -> bool:
    """Shapes/layouts the MFMA kernel takes for c [M, N] (+)= a [M, K] b [K, N] (row-major):
    M, N multiples of 256, K of 128, 16-B aligned unit-stride rows."""
    if not (a.is_cuda and a.dtype in (torch.bfloat16, torch.float16) and b.dtype == a.dtype and a.dim() == 2
            and b.dim() == 2):
        return False
    M, K = a.shape
    N = b.shape[1]
    ok = (M % WGRAD_TILE == 0 and N % WGRAD_TILE == 0 and K % WGRAD_KGRAN == 0 and K >= WGRAD_KGRAN
          and b.shape[0] == K and a.stride(1) == 1 and b.stride(1) == 1
          and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
          and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)
    return ok and (c is None or c.stride(1) == 1)


def gemm_nn_(a, b, c, accumulate: bool = False):
    """c (+)= a @ b with a [M, K], b [K, N] row-major, fp32 accumulation (csrc/gemm_wgrad.hip,
    K-contiguous A images read with ds_read_b128, B images with transposed reads)."""
    if _hip(a):
        _k().gemm_nn_(a, b, c, bool(accumulate))
        return c
    r = a.float() @ b.float()
    if accumulate:
        r += c.float()
    c.copy_(r)
    return c


def gemm_nt_ok(a: torch.Tensor, b: torch.Tensor, c: Optional[torch.Tensor] = None) -> bool:
    """Shapes the 64-deep-K-tile kernel (csrc/gemm_nt.hip) takes for c [M, N] = a [M, K] b [N, K]^T:
    bf16/fp16, M, N multiples of 256, K of 128, 16-B aligned unit-stride rows."""
    if not (a.is_cuda and a.dtype in (torch.bfloat16, torch.float16) and b.dtype == a.dtype and a.dim() == 2
            and b.dim() == 2):
        return False
    M, K = a.shape
    N = b.shape[0]
    return (b.shape[1] == K and M % 256 == 0 and N % 256 == 0 and K % 128 == 0 and a.stride(1) == 1
            and b.stride(1) == 1 and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0
            and b.data_ptr() % 16 == 0 and 256 * a.stride(0) * 2 < 2 ** 31 and 256 * b.stride(0) * 2 < 2 ** 31
            and (c is None or (c.stride(1) == 1 and c.stride(0) % 8 == 0 and c.data_ptr() % 16 == 0)))


def gemm_nt_swiglu_ok(a: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes the gate/up + SwiGLU kernel (csrc/gemm_nt.hip) takes: a [M, K], w = [Wg; Wu] [2F, K],
    bf16/fp16, M % 256, F % 128, K % 128, 16-B aligned unit-stride rows."""
    if not (a.is_cuda and a.dtype in (torch.bfloat16, torch.float16) and w.dtype == a.dtype and a.dim() == 2
            and w.dim() == 2):
        return False
    M, K = a.shape
    F = w.shape[0] // 2
    return (w.shape[0] == 2 * F and w.shape[1] == K and M % 256 == 0 and F % 128 == 0 and K % 128 == 0
            and a.stride(1) == 1 and w.stride(1) == 1 and a.stride(0) % 8 == 0 and w.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0
            and 256 * a.stride(0) * 2 < 2 ** 31 and 256 * w.stride(0) * 2 < 2 ** 31)


def gemm_nt_rope_ok(a: torch.Tensor, w: torch.Tensor, hd: int) -> bool:
    """Shapes the QKV + RoPE-epilogue kernel (csrc/gemm_nt.hip, persistent 4-wave) takes: head dim
    128, bf16/fp16, M, N multiples of 256, K of 128, 16-B aligned unit-stride rows."""
    return hd == 128 and gemm_nt_ok(a, w)


def gemm_nt_rope(a, w, cos, sin, T: int, H: int, G: int, hd: int):
    """qkv = a . w^T ([N, (H + 2G) hd]) with RoPE applied to its q and k heads (the first
    (H + G) hd columns) at position row % T — the QKV projection with the rotation in the GEMM
    epilogue (K4); on CPU the matmul + ``rope_`` oracle (same rounding: the GEMM output first)."""
    if _hip(a):
        qkv = torch.empty(a.shape[0], w.shape[0], dtype=a.dtype, device=a.device)
        _k().gemm_nt_rope_(a, w, qkv, cos, sin, int(T), int((H + G) * hd), int(hd))
        return qkv
    qkv = (a.float() @ w.float().t()).to(a.dtype)
    return ref.rope_(qkv, cos, sin, T, H, G, hd)


def gemm_nt_bias_gelu_ok(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor]) -> bool:
    """Shapes the c_fc + bias + GELU-epilogue kernel takes (persistent 4-wave GEMM)."""
    return bias is not None and bias.dtype == a.dtype and bias.numel() == w.shape[0] and gemm_nt_ok(a, w)


def gemm_nt_bias_gelu(a, w, bias):
    """(f, g) = (a . w^T + bias, gelu(f)) — GPT-2's c_fc with the bias and the exact-erf GELU in
    the GEMM epilogue (K9); on CPU the matmul + ``gelu_fwd`` oracle (f rounded first)."""
    if _hip(a):
        f = torch.empty(a.shape[0], w.shape[0], dtype=a.dtype, device=a.device)
        g = torch.empty_like(f)
        _k().gemm_nt_bias_gelu_(a, w, bias.contiguous(), f, g)
        return f, g
    f = (a.float() @ w.float().t() + bias.float()).to(a.dtype)
    return f, gelu_fwd(f)


def gemm_nt_swiglu(a, w):
    """(gu, act) = (a . w^T, silu(gu[:, :F]) * gu[:, F:]) for w = [W_gate; W_up] — the gate/up
    projection with the SwiGLU forward in its epilogue (csrc/gemm_nt.hip, GPU); on CPU the
    matmul + ``swiglu_fwd`` oracle."""
    F = w.shape[0] // 2
    if _hip(a):
        gu = torch.empty(a.shape[0], 2 * F, dtype=a.dtype, device=a.device)
        act = torch.empty(a.shape[0], F, dtype=a.dtype, device=a.device)
        _k().gemm_nt_swiglu_(a, w, gu, act)
        return gu, act
    gu = (a.float() @ w.float().t()).to(a.dtype)
    return gu, swiglu_fwd(gu)


def gemm_nt_(a, b, c, accumulate: bool = False):
    """c (+)= a @ b^T with a [M, K], b [N, K] (both K-contiguous, a Linear's forward y = x W^T),
    fp32 accumulation on the persistent kernel of csrc/gemm_nt.hip or, for shapes it does not
    take, csrc/gemm_wgrad.hip."""
    if _hip(a):
        _k().gemm_nt_(a, b, c, bool(accumulate))
        return c
    r = a.float() @ b.float().t()
    if accumulate:
        r += c.float()
    c.copy_(r)
    return c


def sum_partials_(part, out, accumulate: bool = False):
    """out (+)= part.sum(0) in fp32, fixed order (split-K reduction); ``out`` contiguous."""
    if _hip(part) and out.numel() % 8 == 0:
        _k().sum_partials_(part, out, bool(accumulate))
        return out
    s = part.float().sum(0).view(out.shape)
    if accumulate:
        s = s + out.float()
    out.copy_(s)
    return out


def attn_decode(q, kcache, vcache, L: int):
    """One new query per sequence against the first ``L`` cached positions.
    q [B, H, hd]; kcache / vcache [B, G, Tmax, hd] -> [B, H*hd]."""
    if q.device.type == "cuda" and q.dtype in (torch.bfloat16, torch.float16):
        load_ext(required=True)
        return _k().attn_decode(q.contiguous(), kcache, vcache, int(L))
    return ref.attn_decode(q, kcache, vcache, L)


def flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, causal=True, dropout_p=0.0, seed=0, offset=0,
                   keep_mask=None, rope=None):
    """``keep_mask``: the buffer the matching forward filled (``attn_keep_mask``), or None to
    regenerate the dropout bits from the counter hash (identical result).  ``rope``: the
    (cos, sin) tables the forward rotated q/k with; the returned dq/dk are then already
    un-rotated (``rope_(..., inverse=True)`` fused into the MFMA kernels' epilogues)."""
    if qkv.device.type == "cuda" and qkv.dtype in (torch.bfloat16, torch.float16, torch.float32):
        load_ext(required=True)
        rc, rs = rope if rope is not None else (None, None)
        return _k().flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, causal, float(dropout_p),
                                   int(seed), int(offset), keep_mask, rc, rs)
    dqkv = ref.flash_attn_bwd(qkv, o, lse, do, B, T, H, G, hd, causal, dropout_p, seed, offset)
    if rope is not None:
        ref.rope_(dqkv, rope[0], rope[1], T, H, G, hd, inverse=True)
    return dqkv


# --------------------------------------------------------------------------- activations
def swiglu_fwd(gu):
    if _hip(gu):
        return _k().swiglu_fwd(gu)
    return ref.swiglu_fwd(gu)


def swiglu_fwd_into(gu, act):
    """swiglu_fwd written into ``act``, a row-strided [N, F] view -> act."""
    if _hip(gu):
        _k().swiglu_fwd_into_(gu, act)
        return act
    act.copy_(ref.swiglu_fwd(gu))
    return act


def swiglu_bwd(gu, dact):
    if _hip(gu):
        return _k().swiglu_bwd(gu, dact)
    return ref.swiglu_bwd(gu, dact)


def swiglu_bwd_lowrank_ok(r: int, F: int) -> bool:
    return r == 16 and F % 8 == 0


def swiglu_bwd_lowrank(gu, base, u, P, scale: float):
    """swiglu_bwd(gu, dact) with dact = base + scale * u @ P formed inside the kernel (the down
    projection's K-augmented LoRA dX: base = dy W, u = dy B^T [N, r], P = A^T [r, F])."""
    if _hip(gu):
        return _k().swiglu_bwd_lowrank(gu, base, u, P, float(scale))
    dact = (base.float() + scale * (u.float() @ P.float())).to(gu.dtype)
    return ref.swiglu_bwd(gu, dact)


def swiglu_bwd_lowrank_wgrad_ok(r: int, F: int) -> bool:
    return r == 16 and F % 64 == 0


def swiglu_bwd_lowrank_wgrad(gu, base, u, P, scale: float, st, gB_gate, gB_up, gA_down_t, accumulate: bool = False):
    """``swiglu_bwd_lowrank`` that also sums, over the same rows, the LoRA gradients that read them:
    gB_gate (+)= st[:, :16]^T dg, gB_up (+)= st[:, 16:32]^T du (the K-augmented gate/up group's dB;
    st = s t) and gA_down_t (+)= scale u^T act (the down projection's dA^T, act = swiglu_fwd(gu),
    u = dy B^T of the down LoRA)."""
    if _hip(gu):
        return _k().swiglu_bwd_lowrank_wgrad(gu, base, u, P, float(scale), st, gB_gate, gB_up, gA_down_t,
                                             bool(accumulate))
    dgu = swiglu_bwd_lowrank(gu, base, u, P, scale)
    F = gu.shape[1] // 2
    act = ref.swiglu_fwd(gu)
    for g, L, R, sc in ((gB_gate, st[:, :16], dgu[:, :F], 1.0), (gB_up, st[:, 16:32], dgu[:, F:], 1.0),
                        (gA_down_t, u[:, :16], act, scale)):
        _vec_into(g, sc * (L.float().t() @ R.float()), accumulate)
    return dgu


def swiglu_bwd_act(gu, dact):
    """``swiglu_bwd`` that also overwrites ``dact`` in place with act = silu(g) * u (what
    ``swiglu_fwd`` returns): the checkpoint recompute skips its SwiGLU forward pass."""
    if _hip(gu):
        return _k().swiglu_bwd_act(gu, dact)
    dgu = ref.swiglu_bwd(gu, dact)
    dact.copy_(ref.swiglu_fwd(gu))
    return dgu


def gelu_fwd(f):
    if _hip(f):
        return _k().gelu_fwd(f)
    return ref.gelu_fwd(f)


def gelu_bwd(f, dg):
    if _hip(f):
        return _k().gelu_bwd(f, dg)
    return ref.gelu_bwd(f, dg)


# --------------------------------------------------------------------------- loss
def ce_fwd(logits, targets, ignore_index: int = -100):
    if _hip(logits):
        return _k().ce_fwd(logits, targets, ignore_index)
    return ref.ce_fwd(logits, targets, ignore_index)


def ce_bwd_(logits, targets, lse, scale, ignore_index: int = -100):
    if _hip(logits):
        _k().ce_bwd_(logits, targets, lse, scale, ignore_index)
        return logits
    return ref.ce_bwd_(logits, targets, lse, scale, ignore_index)


# --------------------------------------------------------------------------- embedding
def embedding_fwd(idx, wte, wpe, T: int, dropout_p: float = 0.0, seed: int = 0, offset: int = 0):
    if _hip(wte):
        return _k().embedding_fwd(idx, wte, wpe, T, float(dropout_p), int(seed), int(offset))
    return ref.embedding_fwd(idx, wte, wpe, T, dropout_p, seed, offset)


def embedding_bwd(idx, dx, grad_wte, grad_wpe, T: int, accumulate: bool = False):
    if _hip(dx):
        _k().embedding_bwd(idx, dx, grad_wte, grad_wpe, T, accumulate)
        return
    ref.embedding_bwd(idx, dx, grad_wte, grad_wpe, T, accumulate)


# --------------------------------------------------------------------------- LoRA
def lora_kernel_ok(x: torch.Tensor, ranks, widths) -> bool:
    """Whether the fused LoRA kernels (csrc/lora.hip) take a group: bf16/fp16 on the GPU, any
    token count (row tails are bounds-checked: variable-length instruction batches), every rank
    a multiple of 16 (<= 64) and every column width (input and member outputs) a multiple of 32.
    Otherwise the caller uses the hipBLASLt GEMM path."""
    if x.dim() != 2 or x.shape[0] < 1:
        return False
    return lora_kernel_ok_dims(x.device, x.dtype, ranks, widths) and x.shape[1] % 32 == 0


def lora_kernel_ok_dims(device, dtype, ranks, widths) -> bool:
    if torch.device(device).type != "cuda" or dtype not in (torch.bfloat16, torch.float16):
        return False
    return all(r % 16 == 0 and 0 < r <= 64 for r in ranks) and all(w % 32 == 0 for w in widths)


def lora_down(x, ws, c0, lens, ocol, R: int, scale: float = 1.0):
    """out[:, ocol_i : +r_i] = scale * x[:, c0_i : +len_i] @ w_i^T  -> [N, R]"""
    if _hip(x):
        return _k().lora_down(x, list(ws), list(c0), list(lens), list(ocol), int(R), float(scale))
    return ref.lora_down(x, ws, c0, lens, ocol, R, scale)


def lora_down_into(x, ws, c0, lens, ocol, R: int, scale: float, out):
    """lora_down written into ``out``, a row-strided [N, >= R] view (the s t columns of
    [x | s t | 0]); columns past R are zeroed (the row-alignment pad)."""
    if _hip(x):
        _k().lora_down_into_(x, list(ws), list(c0), list(lens), list(ocol), int(R), float(scale), out)
        return out
    out[:, :R].copy_(ref.lora_down(x, ws, c0, lens, ocol, R, scale))
    out[:, R:].zero_()
    return out


def lora_block_(dst, Bs, c0, off):
    """dst [rows, R]: B_i^T at rows c0_i.., columns off_i.., zeros elsewhere (the B block of a
    K-augmented weight; ``dst`` may be a transposed view)."""
    if _hip(dst):
        _k().lora_block_(dst, list(Bs), list(c0), list(off))
        return dst
    dst.zero_()
    for b, c, o in zip(Bs, c0, off):
        dst[c:c + b.shape[1], o:o + b.shape[0]].copy_(b.t())
    return dst


def lora_up_(y, t, us, c0, toff, scale: float, base=None, bias=None):
    """y[:, c0_i : +len_i] = base + bias + scale * t[:, toff_i : +r_i] @ u_i  (u_i [r_i, len_i], any
    strides; ``base`` [N, M] and ``bias`` [M] optional, ``base`` may be ``y`` itself)."""
    if _hip(y):
        _k().lora_up_(y, t, list(us), list(c0), list(toff), float(scale), base, bias)
        return y
    return ref.lora_up_(y, t, us, c0, toff, scale, base, bias)


def lora_wgrad(p, q, gs, pa, qb, scale: float, accumulate: bool = False):
    """g_i[a][b] (+)= scale * sum_n p[n][pa_i + a] q[n][qb_i + b], written into g_i in its dtype."""
    if _hip(p):
        _k().lora_wgrad(p, q, list(gs), list(pa), list(qb), float(scale), bool(accumulate))
        return
    ref.lora_wgrad(p, q, gs, pa, qb, scale, accumulate)


LORA_HEAD_FUSED = True   # the LoRA head's u and dB in one pass over each dlogits chunk


def lora_head_bwd_ok(V: int, r: int) -> bool:
    return LORA_HEAD_FUSED and r == 16 and V % 64 == 0


def lora_head_bwd_(dl, st, B, u, gB, accumulate: bool = False):
    """The LoRA head's two rank-16 products of a logits-gradient chunk dl [R, V] in one pass over
    it: u = dl B^T (into u [R, 16]) and gB (+)= st^T dl (st [R, 16], B and gB [16, V])."""
    if _hip(dl):
        _k().lora_head_bwd_(dl, st, B, u, gB, bool(accumulate))
        return
    u.copy_((dl.float() @ B.float().t()).to(u.dtype))
    _vec_into(gB, st.float().t() @ dl.float(), accumulate)


def lora_pack_t(As):
    """[sum r_i, K] = concat_i A_i^T (A_i [K, r_i])"""
    if _hip(As[0]):
        return _k().lora_pack_t(list(As))
    return ref.lora_pack_t(As)


# --------------------------------------------------------------------------- optimizer
def sq_norm_multi(tensors: List[torch.Tensor]) -> torch.Tensor:
    """Sum of squares over all tensors -> 1-element fp32 tensor (no host sync)."""
    tensors = [t for t in tensors if t is not None and t.numel() > 0]
    if not tensors:
        return torch.zeros(1, dtype=torch.float32)
    if _hip(tensors[0]):
        return _k().sq_norm_multi(tensors)
    return sum(ref.sq_norm(t) for t in tensors).reshape(1)


def adamw_step_(param, master, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay,
                step, grad_scale=None):
    if _hip(param):
        _k().adamw_step_(param, master, grad, exp_avg, exp_avg_sq, float(lr), float(beta1),
                         float(beta2), float(eps), float(weight_decay), int(step), grad_scale)
        return
    ref.adamw_step_(param, master, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay,
                    step, grad_scale)
