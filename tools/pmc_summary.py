#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output per kernel (sums over dispatches), with a few derived
ratios.  Usage: python tools/pmc_summary.py DIR/..._counter_collection.csv [--filter attn]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for path in a.csv:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            if a.filter not in k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[k] = (r.get("VGPR_Count"), r.get("Accum_VGPR_Count"), r.get("LDS_Block_Size"))
    for k, d in agg.items():
        print(k[:90], "vgpr/agpr/lds", meta[k])
        for c, v in sorted(d.items()):
            print(f"    {c:28s} {v:16.4g}")
        if "SQ_WAVE_CYCLES" in d:
            wc = d["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
                if c in d:
                    print(f"    {c + '/WAVE_CYCLES':40s} {d[c] / wc:.3f}")
        if "SQ_INSTS_MFMA" in d and "SQ_INSTS_VALU" in d:
            print(f"    VALU per MFMA {d['SQ_INSTS_VALU'] / max(d['SQ_INSTS_MFMA'], 1):.2f}   "
                  f"LDS per MFMA {d.get('SQ_INSTS_LDS', 0) / max(d['SQ_INSTS_MFMA'], 1):.2f}   "
                  f"SALU per MFMA {d.get('SQ_INSTS_SALU', 0) / max(d['SQ_INSTS_MFMA'], 1):.2f}")


if __name__ == "__main__":
    main()
