#!/usr/bin/env python3
"""Per-kernel time summary from a rocprofv3 SQLite output (``-d DIR -o run`` -> run_results.db),
for runs where the CSV stats are not written.  Usage: python tools/kstats.py DB [--grep SUBSTR]
[--seq] (``--seq``: also print dispatches in order, name and duration, for the matching kernels)."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--grep", default="")
    ap.add_argument("--seq", action="store_true")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    agg = {}
    for name, s, e in rows:
        if a.grep and a.grep not in name:
            continue
        t = agg.setdefault(name, [0, 0.0])
        t[0] += 1
        t[1] += (e - s) / 1e3
    for name, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{us / n:10.1f} us  x{n:<5d} {name[:150]}")
    if a.seq:
        for name, s, e in rows:
            if not a.grep or a.grep in name:
                print(f"{(e - s) / 1e3:10.1f}  {name[:100]}")


if __name__ == "__main__":
    main()
