#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table from hipcc's -Rpass-analysis=kernel-resource-usage
remarks.  Usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [SUBSTR]"""
import re
import sys

want = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = int(m.group(2))
print(f"{'VGPR':>5} {'AGPR':>5} {'spill':>5} {'occ':>3}  kernel")
for r in rows:
    if want in r["name"]:
        print(f"{r.get('VGPRs', 0):5d} {r.get('AGPRs', 0):5d} {r.get('VGPRs Spill', 0):5d} "
              f"{r.get('Occupancy [waves/SIMD]', 0):3d}  {r['name']}")
