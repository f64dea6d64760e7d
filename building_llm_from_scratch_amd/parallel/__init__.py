"""Distributed engines (one process per GPU, RCCL over xGMI via torch.distributed "nccl").

* ``local``  — single process (no collectives).
* ``ddp``    — replicated params, bucketed gradient all-reduce overlapped with backward
               (reference: torch DDP, build_components.py:176).
* ``zero1``  — DDP + optimizer-state sharding: reduce-scatter grads, shard-local AdamW,
               all-gather params (reference: ZeroRedundancyOptimizer, :250-256).
* ``fsdp``   — full sharding of params / grads / optimizer state per unit with prefetched
               all-gathers and reduce-scatters on a comm stream (reference: FSDP FULL_SHARD,
               :155-174).
"""
from __future__ import annotations

import os

import torch

from ..models.base import LocalEngine


def nccl_pg_options(timeout=None):
    """RCCL process-group options: collectives on HIGH-priority HIP streams, so a prefetched
    all-gather / reduce-scatter kernel is scheduled ahead of queued compute kernels instead of
    waiting behind them (the overlap FSDP / DDP rely on).  ``timeout`` (the same timedelta
    passed to ``init_process_group``) is stored in the options too: torch warns on every RCCL
    init when the two differ."""
    import torch.distributed as dist
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        if timeout is not None:
            opts._timeout = timeout
        return opts
    except (AttributeError, RuntimeError):  # torch built without NCCL/RCCL
        return None


def force_comm() -> bool:
    """``BLLM_FORCE_COMM=1``: engines run their collective path even at world size 1 (every
    all-gather / reduce-scatter / all-reduce issued on RCCL's stream, shards freed and re-gathered)
    instead of the world-1 shortcut — the N>1 code path rehearsed on a single GPU, where RCCL
    cannot put two ranks (tests/test_engines_gpu.py, bench.py --force_comm)."""
    return os.environ.get("BLLM_FORCE_COMM", "0") not in ("", "0")


def setup_engine(model, kind: str = "local", device=None, reduce_dtype=None, bucket_mb: float = 256.0,
                 reshard_after_forward: bool = True, process_group=None, prefetch: int = 0):
    """Flatten ``model`` onto ``device`` and attach the requested engine; returns it."""
    device = torch.device(device) if device is not None else model.device
    if kind in ("local", "single", "single_gpu"):
        model.flatten(device=device)
        eng = LocalEngine(model)
        model.set_engine(eng)
        return eng
    if kind == "ddp":
        from .ddp import DDPEngine
        return DDPEngine(model, device, reduce_dtype=reduce_dtype, bucket_mb=bucket_mb, pg=process_group)
    if kind == "zero1":
        from .zero import ZeroEngine
        return ZeroEngine(model, device, reduce_dtype=reduce_dtype, bucket_mb=bucket_mb, pg=process_group)
    if kind == "fsdp":
        from .fsdp import FSDPEngine
        return FSDPEngine(model, device, reduce_dtype=reduce_dtype,
                          reshard_after_forward=reshard_after_forward, pg=process_group, prefetch=prefetch)
    raise ValueError(f"unknown parallel engine '{kind}'")
