"""Closeness checks for kernel-vs-oracle tests, tied to the oracle's own rounding.

``check_close(out, ref, dt, k)`` — ``ref`` is the fp32 (or fp64) oracle of the op, ``dt`` the
kernel's output dtype.  The unit of error is what rounding the EXACT oracle result to ``dt``
costs, ``eps = ||round_dt(ref) - ref|| / ||ref||``: no kernel that writes ``dt`` can do better.
Two conditions, both at ``k`` units:

  * global: ``||out - ref|| / ||ref|| <= k * eps``;
  * per magnitude band: the elements are split into deciles of ``|ref|`` and in each band the
    RMS error, relative to the RMS of the whole ``ref``, must be within ``k`` times the larger
    of ``eps`` and that band's own rounding error.  A global norm is dominated by the largest
    elements; the bands make an error confined to small-magnitude elements (a wrong GQA
    partial, a masked-tile edge, a mis-scaled tail) visible: a 1 % (of RMS) perturbation of
    the smallest 10 % of elements is ~6x the bf16 allowance at k = 1, so every bf16 / fp16
    kernel test keeps k <= 5 (tests/test_numerics_check.py).

``check_elem(out, ref, rtol, atol)`` — elementwise ``|out - ref| <= atol + rtol * |ref|`` for
per-row statistics (log-sum-exp, CE rows, norm rstd), where every element matters on its own.

``BLLM_NUMERICS_REPORT=<file>``: append ``{name, ratio}`` records (the measured error in units
of the allowance: <= 1 passes); with ``BLLM_NUMERICS_CALIBRATE=1`` nothing asserts (a
calibration run of the whole suite).
"""
from __future__ import annotations

import json
import math
import os

import torch

# fp32 outputs: rounding to fp32 is exact, so the unit is a small multiple of fp32's epsilon
# (summation-order differences between the kernel and the oracle)
FP32_FLOOR = 2.0e-6


# relative RMS rounding error of a normally distributed value rounded to the dtype; the floor
# of the unit when ``ref`` happens to be exactly representable (e.g. a round trip of dt data)
NOMINAL = {torch.bfloat16: 1.67e-3, torch.float16: 2.1e-4, torch.float32: FP32_FLOOR}


def _eps(r: torch.Tensor, dt: torch.dtype) -> float:
    nr = r.norm().item()
    if nr == 0.0:
        return FP32_FLOOR
    rd = (r.to(dt).double() - r).norm().item() / nr if dt != torch.float32 else 0.0
    return max(rd, 0.5 * NOMINAL.get(dt, FP32_FLOOR), FP32_FLOOR)


def close_ratio(out: torch.Tensor, ref: torch.Tensor, dt: torch.dtype, bands: int = 10) -> float:
    """Worst condition of check_close in units of k (<= k passes)."""
    dev = out.device if out.is_cuda else ref.device      # evaluate on the GPU when there is one
    a = out.detach().to(dev, torch.float64).flatten()
    r = ref.detach().to(dev, torch.float64).flatten()
    assert a.numel() == r.numel(), (a.shape, r.shape)
    if not torch.isfinite(a).all():
        return math.inf
    n = r.numel()
    nr = r.norm().item()
    if nr == 0.0:
        return a.abs().max().item() / FP32_FLOOR if n else 0.0
    eps = _eps(r, dt)
    err = a - r
    worst = err.norm().item() / nr / eps
    rms_r = nr / math.sqrt(n)
    if n >= 2 * bands:
        order = r.abs().argsort()
        rr = r.to(dt).double() - r if dt != torch.float32 else torch.zeros_like(r)
        for idx in order.chunk(bands):
            m = idx.numel()
            band_err = err[idx].norm().item() / math.sqrt(m) / rms_r
            band_round = rr[idx].norm().item() / math.sqrt(m) / rms_r
            worst = max(worst, band_err / max(eps, band_round))
    return worst


def _report(name, ratio):
    path = os.environ.get("BLLM_NUMERICS_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"name": name, "ratio": ratio, "test": os.environ.get("PYTEST_CURRENT_TEST", "")})
                    + "\n")


def _calibrating() -> bool:
    return os.environ.get("BLLM_NUMERICS_CALIBRATE", "0") == "1"


def check_close(out, ref, dt, k: float = 2.0, name: str = ""):
    ratio = close_ratio(out, ref, dt)
    _report(name, ratio / k)
    if _calibrating():
        return
    assert ratio <= k, f"{name}: error {ratio:.2f} x the {dt} rounding unit (allowed {k})"


def check_elem(out, ref, rtol: float, atol: float, name: str = ""):
    a = out.detach().double().cpu().flatten()
    r = ref.detach().double().cpu().flatten()
    tol = atol + rtol * r.abs()
    bad = (a - r).abs() > tol
    bad |= ~torch.isfinite(a)
    _report(name + " (elem)", float(((a - r).abs() / tol).max().item()) if a.numel() else 0.0)
    if _calibrating():
        return
    if bad.any():
        i = int(bad.nonzero()[0])
        raise AssertionError(f"{name}: {int(bad.sum())} of {a.numel()} elements outside atol {atol} + rtol {rtol}; "
                             f"first at {i}: {a[i].item()} vs {r[i].item()}")
