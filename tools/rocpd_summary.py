#!/usr/bin/env python3
"""Summarise a rocprofv3 (ROCm 7.2) SQLite database: per-kernel total time, calls, share.
Usage: python tools/rocpd_summary.py path/to/results.db [--top 40] [--md out.md]"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "")
    return name[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
    rows = con.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        k = short(n)
        t, c = agg.get(k, (0, 0))
        agg[k] = (t + (e - s), c + 1)
    total = sum(t for t, _ in agg.values())
    lines = [f"total kernel time: {total / 1e6:.2f} ms over {len(rows)} dispatches", "",
             "| kernel | calls | total ms | avg us | share |", "|---|---|---|---|---|"]
    for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[: a.top]:
        lines.append(f"| `{k}` | {c} | {t / 1e6:.3f} | {t / c / 1e3:.1f} | {100 * t / total:.1f}% |")
    out = "\n".join(lines)
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out + "\n")


if __name__ == "__main__":
    main()
