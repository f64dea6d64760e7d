#!/usr/bin/env python3
"""Summarise a torch.profiler chrome trace: total time per (category, name) for host-side events
(cpu_op, cuda_runtime / hip runtime calls, user annotations), top N, plus the wall span and the
device-kernel busy time.  Usage: python tools/trace_top.py trace.json [--top 30]"""
import argparse
import collections
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    ev = json.load(open(a.trace))
    ev = ev["traceEvents"] if isinstance(ev, dict) else ev
    agg = collections.defaultdict(lambda: [0.0, 0])
    t0, t1, kbusy = None, None, 0.0
    for e in ev:
        if e.get("ph") != "X":
            continue
        cat, name, dur, ts = e.get("cat", ""), e.get("name", ""), float(e.get("dur", 0)), float(e.get("ts", 0))
        t0 = ts if t0 is None else min(t0, ts)
        t1 = ts + dur if t1 is None else max(t1, ts + dur)
        if cat == "kernel":
            kbusy += dur
            continue
        a_ = agg[(cat, name[:80])]
        a_[0] += dur
        a_[1] += 1
    print(f"span {(t1 - t0) / 1e3:.1f} ms, device kernels {kbusy / 1e3:.1f} ms")
    for (cat, name), (d, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"{d / 1e3:10.1f} ms  x{n:<6d} {cat:16s} {name}")


if __name__ == "__main__":
    main()
