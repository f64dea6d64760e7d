#!/usr/bin/env python3
"""Per-kernel sums of the PMC counters in a rocprofv3 SQLite database (ROCm 7.2 rocpd schema:
view ``pmc_events``), with a few derived ratios.
Usage: python tools/pmc_db_summary.py results.db [more.db ...] [--filter attn]"""
import argparse
import collections
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    rows = collections.defaultdict(lambda: collections.defaultdict(int))
    for path in a.db:
        con = sqlite3.connect(path)
        for name, cname, val in con.execute("select name, counter_name, counter_value from pmc_events"):
            if a.filter and a.filter not in name:
                continue
            k = re.sub(r"\(.*", "", name)[:100]
            agg[k][cname] += float(val)
            rows[k][cname] += 1
    for k, d in agg.items():
        print(k)
        for c, v in sorted(d.items()):
            # rows: pmc_events records of this counter (one per dispatch for a derived counter)
            print(f"    {c:32s} {v:12.4g}   rows {rows[k][c]}")
        wc = d.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if c in d:
                    print(f"    {c + '/WAVE_CYCLES':32s} {d[c] / wc:12.3f}")
        if d.get("SQ_BUSY_CYCLES") and d.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            # MFMA_BUSY is summed over SIMDs; BUSY_CYCLES over SEs/XCDs: report both raw
            print(f"    {'MFMA_BUSY/BUSY_CYCLES':32s} {d['SQ_VALU_MFMA_BUSY_CYCLES'] / d['SQ_BUSY_CYCLES']:12.3f}")


if __name__ == "__main__":
    main()
