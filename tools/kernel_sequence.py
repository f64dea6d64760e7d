#!/usr/bin/env python3
"""Print the kernel sequence (name, duration) of the last training step in a rocprofv3
kernel-trace database, starting at the last dispatch matching --marker.
Usage: python tools/kernel_sequence.py run_results.db [--marker emb_fwd] [--skip 0] [--count 80]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="emb_fwd")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--count", type=int, default=80)
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select name,start,end,grid_x from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
    seq = rows[idx[-1]:]
    t0 = seq[0][1]
    for n, s, e, g in seq[a.skip:a.skip + a.count]:
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f}us g{g:<9d} {n[:100]}")


if __name__ == "__main__":
    main()
