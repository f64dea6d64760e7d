#!/usr/bin/env python3
"""Communication / compute overlap from a rocprofv3 kernel trace (SQLite, ROCm 7.2).

Every RCCL kernel (name starting with ``nccl``/``rccl``) is a *comm* interval, rocclr device copies
are their own class (at world 1 under ``BLLM_FORCE_COMM=1`` RCCL's collectives run as such copies),
every other kernel is *compute*.  For each comm
interval the tool measures how much of it ran while at least one compute kernel was running,
and reports per class the total comm time, the overlapped part and the exposed part (comm time
with the matrix cores idle) -- the evidence that FSDP's all-gathers / reduce-scatters and DDP's
bucket all-reduces run under the backward / forward GEMMs instead of between them.

Usage: python tools/overlap.py run_results.db [--md out.md]
"""
import argparse
import re
import sqlite3


def _union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _covered(s, e, merged, lo):
    """Length of [s, e) covered by the merged interval list, scanning from index lo."""
    tot = 0
    i = lo
    while i < len(merged) and merged[i][1] <= s:
        i += 1
    j = i
    while j < len(merged) and merged[j][0] < e:
        tot += min(e, merged[j][1]) - max(s, merged[j][0])
        j += 1
    return tot, i


def classify(name: str) -> str:
    n = name.lower()
    if n.startswith("nccl") or n.startswith("rccl") or "nccldevkernel" in n or "ncclkernel" in n:
        m = re.search(r"(allgather|reducescatter|allreduce|broadcast|sendrecv|reduce)", n)
        return "rccl:" + (m.group(1) if m else "other")
    if "rocclr_copybuffer" in n:  # device copies; at world 1 (BLLM_FORCE_COMM) RCCL's collectives are these
        return "copy"
    return "compute"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = con.execute(f"select {name_col}, start, end from kernels").fetchall()
    comp, comm = [], {}
    for n, s, e in rows:
        c = classify(n)
        if c == "compute":
            comp.append((s, e))
        else:
            comm.setdefault(c, []).append((s, e))
    merged = _union(comp)
    lines = ["| comm class | dispatches | total ms | overlapped with compute ms | exposed ms | overlapped % |",
             "|---|---|---|---|---|---|"]
    for c, iv in sorted(comm.items()):
        iv.sort()
        tot = cov = 0
        lo = 0
        for s, e in iv:
            t, lo = _covered(s, e, merged, lo)
            tot += e - s
            cov += t
        lines.append(f"| {c} | {len(iv)} | {tot / 1e6:.2f} | {cov / 1e6:.2f} | {(tot - cov) / 1e6:.2f} | "
                     f"{100 * cov / max(tot, 1):.1f} |")
    if not comm:
        lines.append("| (no RCCL kernels in this trace) | 0 | 0 | 0 | 0 | - |")
    busy = sum(e - s for s, e in merged)
    span = (max(r[2] for r in rows) - min(r[1] for r in rows)) if rows else 0
    lines += ["", f"trace span {span / 1e6:.1f} ms, compute busy {busy / 1e6:.1f} ms "
                  f"({100 * busy / max(span, 1):.1f} %), {len(rows)} dispatches"]
    out = "\n".join(lines)
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out + "\n")


if __name__ == "__main__":
    main()
