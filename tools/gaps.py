#!/usr/bin/env python3
"""GPU idle gaps in a rocprofv3 kernel-trace database: the largest gaps between consecutive
dispatches (end of one to start of the next) with the kernels around them, and the idle total
between the first and last dispatch.  Usage: python tools/gaps.py results.db [--top 25]"""
import argparse
import re
import sqlite3


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--min_us", type=float, default=50.0)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    nc = "kernel_name" if "kernel_name" in cols else "name"
    rows = sorted(con.execute(f"select start, end, {nc} from kernels").fetchall())
    gaps, idle, t_end = [], 0.0, rows[0][1]
    steps = 0   # emb_fwd dispatches seen so far: the forward pass index the gap falls in
    for (s, e, n), (ps, pe, pn) in zip(rows[1:], rows[:-1]):
        if "emb_fwd" in pn:
            steps += 1
        g = s - max(t_end, pe)
        if g > 0:
            idle += g
            if g / 1e3 >= a.min_us:
                gaps.append((g, pn, n, s, steps))
        t_end = max(t_end, e)
    span = rows[-1][1] - rows[0][0]
    print(f"{len(rows)} dispatches, span {span / 1e6:.1f} ms, idle {idle / 1e6:.1f} ms "
          f"({100 * idle / span:.1f} %), gaps >= {a.min_us} us: {len(gaps)} totalling "
          f"{sum(g[0] for g in gaps) / 1e6:.1f} ms")
    for g, pn, n, s, st in sorted(gaps, reverse=True)[:a.top]:
        print(f"{g / 1e3:10.1f} us  at {(s - rows[0][0]) / 1e6:9.1f} ms  fwd#{st:<3d} after {short(pn):60s} "
              f"before {short(n)}")


if __name__ == "__main__":
    main()
