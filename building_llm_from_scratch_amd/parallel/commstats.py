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
with N and ``comm_exposed_ms`` rising says why, where a bare tok/s would not."""
from __future__ import annotations

import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict

import torch


class CommStats:
    def __init__(self, device=None):
        dev = torch.device(device) if device is not None else torch.device("cpu")
        self.cuda = dev.type == "cuda"
        self.enabled = False
        self._events = []                       # (kind, start, end) HIP events
        self._host: Dict[str, float] = defaultdict(float)
        self._count: Dict[str, int] = defaultdict(int)

    def reset(self, enabled: bool = True):
        self._events, self._host, self._count = [], defaultdict(float), defaultdict(int)
        self.enabled = enabled

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
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events.append((kind, s, e))
        else:
            t0 = time.perf_counter()
            yield
            self._host[kind] += time.perf_counter() - t0

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
