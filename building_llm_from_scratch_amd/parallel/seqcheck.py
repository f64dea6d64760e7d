"""Run-time check that every rank issues the same collectives in the same order.

The engines are built so that the collective order is identical on every rank (FSDP's unit
order, DDP / ZeRO's bucket order, warm-up adaptation decided on the MAX over ranks:
``parallel/fsdp.py``, ``ddp.py``, ``commstats.max_over_ranks``), and ``tests/test_comm_plan.py``
checks that order against the engines' plans on a fake process group.  Nothing checked it while a
real job runs: a divergent order on the first multi-GPU run (a rank-dependent branch, a skipped
bucket, an extra all-reduce) would pair unrelated collectives on RCCL and show up only as the
process group's timeout tens of minutes later, with no hint of which call diverged.

``CollectiveSequence`` records, while active, every collective issued through
``torch.distributed`` (op, bytes, dtype; the same entry points ``commplan.Recorder`` wraps) and
``verify(tag)`` compares the ranks' records **over the rendezvous store, not over the process
group**: a mismatched collective may already have wedged the group's stream, and the check must
not pair with it.  It runs on the host right after a warm-up step has been *issued* (before any
host synchronisation that would wait on those collectives), so a divergence raises
``CollectiveOrderError`` naming the first differing call on every rank within seconds.  The
steady-state steps are not recorded (zero overhead in the timed loop).

Reference: the reference relies on torch DDP / FSDP for a consistent order and has no such check
(``/root/reference/main.py:22-29,191``)."""
from __future__ import annotations

import json
import time
from contextlib import contextmanager
from datetime import timedelta
from typing import Dict, List, Optional

import torch.distributed as dist

_OPS = ("all_reduce", "all_gather_into_tensor", "reduce_scatter_tensor", "broadcast", "all_gather",
        "reduce_scatter", "all_to_all_single", "barrier")
_NAMES = {"all_gather_into_tensor": "all_gather", "reduce_scatter_tensor": "reduce_scatter"}


class CollectiveOrderError(RuntimeError):
    pass


def _describe(op: str, args, kw) -> Dict:
    """(op, bytes, dtype) of one call: the full tensor (all-gather output, reduce-scatter input)."""
    t = None
    if op == "reduce_scatter_tensor":
        t = args[1] if len(args) > 1 else kw.get("input")
    elif op in ("all_gather", "reduce_scatter"):
        lst = args[0] if args else kw.get("tensor_list") or kw.get("output")
        if isinstance(lst, (list, tuple)) and lst:
            n = sum(x.numel() for x in lst)
            return {"op": _NAMES.get(op, op), "bytes": n * lst[0].element_size(),
                    "dtype": str(lst[0].dtype).replace("torch.", "")}
    elif op != "barrier":
        t = args[0] if args else (kw.get("tensor") or kw.get("output_tensor") or kw.get("output"))
    if t is None:
        return {"op": _NAMES.get(op, op), "bytes": 0, "dtype": "-"}
    return {"op": _NAMES.get(op, op), "bytes": int(t.numel() * t.element_size()),
            "dtype": str(t.dtype).replace("torch.", "")}


def _fmt(e: Optional[Dict]) -> str:
    return "nothing" if e is None else f"{e['op']}({e['bytes']} B, {e['dtype']})"


def first_divergence(seqs: List[List[Dict]]):
    """Index of the first position where the ranks' records differ (None if all equal)."""
    n = max(len(s) for s in seqs)
    for i in range(n):
        col = [(s[i]["op"], s[i]["bytes"], s[i]["dtype"]) if i < len(s) else None for s in seqs]
        if any(c != col[0] for c in col):
            return i
    return None


class CollectiveSequence:
    def __init__(self, pg=None, store=None, timeout_s: float = 120.0, enabled: Optional[bool] = None):
        self.pg = pg
        self.active = False
        self.log: List[Dict] = []
        self.timeout_s = timeout_s
        ok = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(pg) if ok else 1
        self.rank = dist.get_rank(pg) if ok else 0
        self.enabled = (ok and self.world > 1) if enabled is None else (bool(enabled) and ok)
        self.store = store
        if self.enabled and self.store is None:
            from torch.distributed import distributed_c10d as c10d
            self.store = c10d._get_default_store()
        self.checks = 0

    @contextmanager
    def recording(self, phase: str = ""):
        """Record the collectives issued inside the block (wraps the torch.distributed entry
        points; the calls themselves run unchanged)."""
        if not self.enabled:
            yield self
            return
        saved = {n: getattr(dist, n) for n in _OPS if hasattr(dist, n)}

        def wrap(name, fn):
            def inner(*args, **kw):
                e = _describe(name, args, kw)
                e["phase"] = phase
                self.log.append(e)
                return fn(*args, **kw)
            return inner

        for n, fn in saved.items():
            setattr(dist, n, wrap(n, fn))
        self.active = True
        try:
            yield self
        finally:
            for n, fn in saved.items():
                setattr(dist, n, fn)
            self.active = False

    def verify(self, tag: str) -> int:
        """Compare this rank's record since the last verify with every other rank's (rendezvous
        store, host only).  Raises ``CollectiveOrderError`` naming the first divergent call, or
        the ranks that never reported within ``timeout_s``.  Returns the number of calls checked."""
        mine, self.log = self.log, []
        if not self.enabled:
            return len(mine)
        key = f"bllm_collseq/{tag}/{self.checks}"
        self.checks += 1
        self.store.set(f"{key}/{self.rank}", json.dumps(mine))
        keys = [f"{key}/{r}" for r in range(self.world)]
        t0 = time.time()
        try:
            self.store.wait(keys, timedelta(seconds=self.timeout_s))
        except Exception:
            missing = [r for r in range(self.world) if not self.store.check([f"{key}/{r}"])]
            raise CollectiveOrderError(
                f"collective-order check '{tag}': rank(s) {missing} did not finish issuing the step's "
                f"collectives within {self.timeout_s:.0f} s (rank {self.rank} issued {len(mine)}: "
                f"last {_fmt(mine[-1] if mine else None)}); a rank is stuck or took another code path")
        seqs = [json.loads(self.store.get(k)) for k in keys]
        i = first_divergence(seqs)
        if i is not None:
            per = "; ".join(f"rank {r}: {_fmt(s[i] if i < len(s) else None)}"
                            + (f" [{s[i]['phase']}]" if i < len(s) and s[i].get("phase") else "")
                            for r, s in enumerate(seqs))
            counts = ", ".join(f"r{r}={len(s)}" for r, s in enumerate(seqs))
            raise CollectiveOrderError(
                f"collective-order check '{tag}': ranks diverge at collective #{i} -- {per} "
                f"(calls per rank: {counts}); RCCL would pair unrelated collectives from here on")
        self.waited_s = time.time() - t0
        return len(mine)
