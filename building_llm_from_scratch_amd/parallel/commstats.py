"""Exposed-collective accounting: how long each rank's compute stream was held up by a collective.

Every point where an engine makes compute wait for a collective (FSDP: the all-gather of the unit
about to run, the retire of an older reduce-scatter, the grad-norm all-reduce; DDP / ZeRO-1: the
end-of-backward wait for the bucket all-reduces / reduce-scatters, ZeRO's per-bucket parameter
all-gather before a forward) is bracketed by ``CommStats.waiting(kind)``:

* on a GPU, one timing event is recorded on the current HIP stream before the wait and one
  after it.  The first completes when the compute queued ahead of the wait is done, the second
  when the collective has finished too, so their distance is the time the stream sat idle on
  RCCL: 0 when the collective was fully hidden behind compute (nothing is synchronised on the
  host; events are read once, in ``summary``);
* on the CPU (gloo), ``wait()`` blocks the host, so the host time inside the bracket is used.

A rank that waits long is communication-bound; a multi-GPU bench line that shows tok/s falling
with N and ``comm_exposed_ms`` rising says why, where a bare tok/s would not.

Achieved bandwidth: every collective an engine issues is registered with ``issued(kind, work,
nbytes)``.  Its duration is RCCL's own issue-to-complete time on the collective's stream
(``Work._get_duration()``, filled when ``TORCH_NCCL_ENABLE_TIMING=1`` — bench.py and the CLI
set it before the process group exists); on gloo it is the host time from issue to the
return of its wait.  ``bandwidth()`` gives per kind the bytes, the time, the algorithm
bandwidth (bytes / time) and the bus bandwidth (x (W-1)/W for all-gather / reduce-scatter,
x 2(W-1)/W for all-reduce: the per-link figure to hold against xGMI's ~150 GB/s per link).

``BLLM_COMM_DELAY_MS`` (tests only): sleep that long inside every exposed-wait bracket of the
ranks listed in ``BLLM_COMM_DELAY_RANKS`` — a slow link, to drive the engines' adaptation."""
from __future__ import annotations

import os
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List

import torch

_BUS = {"all_gather": lambda w: (w - 1) / w, "reduce_scatter": lambda w: (w - 1) / w,
        "all_reduce": lambda w: 2.0 * (w - 1) / w, "broadcast": lambda w: 1.0}


def _delay_s() -> float:
    ms = float(os.environ.get("BLLM_COMM_DELAY_MS", "0") or 0)
    if ms <= 0:
        return 0.0
    ranks = os.environ.get("BLLM_COMM_DELAY_RANKS", "")
    if ranks:
        import torch.distributed as dist
        r = dist.get_rank() if dist.is_initialized() else 0
        if str(r) not in ranks.split(","):
            return 0.0
    return ms / 1e3


class CommStats:
    def __init__(self, device=None, world: int = 1):
        dev = torch.device(device) if device is not None else torch.device("cpu")
        self.cuda = dev.type == "cuda"
        self.world = world
        self.enabled = False
        self._events = []                       # (kind, start, end) HIP events
        self._host: Dict[str, float] = defaultdict(float)
        self._count: Dict[str, int] = defaultdict(int)
        self._issued: List[list] = []           # [kind, work, nbytes, host t0, host t1]
        self._by_work: Dict[int, list] = {}
        self._delay = _delay_s()

    def reset(self, enabled: bool = True):
        self._events, self._host, self._count = [], defaultdict(float), defaultdict(int)
        self._issued, self._by_work = [], {}
        self.enabled = enabled

    def issued(self, kind: str, work, nbytes: int):
        """Register one collective (its async work handle) for the bandwidth account."""
        if not self.enabled or work is None:
            return
        rec = [kind, work, int(nbytes), time.perf_counter(), None]
        self._issued.append(rec)
        self._by_work[id(work)] = rec

    def completed(self, work):
        rec = self._by_work.pop(id(work), None)
        if rec is not None:
            rec[4] = time.perf_counter()

    @contextmanager
    def waiting(self, kind: str):
        if not self.enabled:
            yield
            return
        self._count[kind] += 1
        if self.cuda:
            s = torch.cuda.Event(enable_timing=True)
            s.record()
            yield
            if self._delay:
                torch.cuda._sleep(int(self._delay * 2e9))
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events.append((kind, s, e))
        else:
            t0 = time.perf_counter()
            yield
            if self._delay:
                time.sleep(self._delay)
            self._host[kind] += time.perf_counter() - t0

    def bandwidth(self) -> Dict[str, Dict[str, float]]:
        """{kind: {"count", "bytes", "ms", "algbw_gbps", "busbw_gbps", "timing"}} of the
        collectives registered since the last reset."""
        if self.cuda and self._issued:
            torch.cuda.synchronize()
        acc: Dict[str, Dict[str, float]] = {}
        for kind, work, nbytes, t0, t1 in self._issued:
            ms, how = None, None
            try:
                d = float(work._get_duration())
                if d > 0:
                    ms, how = d, "rccl events"
            except Exception:
                pass
            if ms is None and t1 is not None:
                ms, how = 1e3 * (t1 - t0), "host issue-to-wait"
            if ms is None:
                continue
            a = acc.setdefault(kind, {"count": 0, "bytes": 0, "ms": 0.0, "timing": how})
            a["count"] += 1
            a["bytes"] += nbytes
            a["ms"] += ms
        for kind, a in acc.items():
            alg = a["bytes"] / (a["ms"] / 1e3) / 1e9 if a["ms"] > 0 else 0.0
            a["algbw_gbps"] = float(f"{alg:.4g}")
            a["busbw_gbps"] = float(f"{alg * _BUS.get(kind, lambda w: 1.0)(max(self.world, 2)):.4g}")
            a["ms"] = round(a["ms"], 3)
        return acc

    def summary(self) -> Dict[str, Dict[str, float]]:
        """{kind: {"ms": total exposed ms, "waits": count}} since the last reset."""
        ms: Dict[str, float] = defaultdict(float)
        if self._events:
            self._events[-1][2].synchronize()
            for kind, s, e in self._events:
                ms[kind] += s.elapsed_time(e)
        for kind, sec in self._host.items():
            ms[kind] += 1e3 * sec
        return {k: {"ms": round(ms.get(k, 0.0), 3), "waits": self._count[k]} for k in self._count}

    def total_ms(self) -> float:
        return float(sum(v["ms"] for v in self.summary().values()))


# share of the step an exposed collective wait may take before the engine adapts (warm-up)
ADAPT_FRAC = 0.02


def max_over_ranks(values, pg=None, device=None):
    """Element-wise MAX over the ranks of a small list of floats (one all-reduce): every rank
    then takes the same adaptation decision, so the collective order stays identical."""
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64,
                     device=device if device is not None and torch.device(device).type == "cuda" else "cpu")
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(pg) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=pg)
    return [float(x) for x in t.cpu().tolist()]
