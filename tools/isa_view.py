#!/usr/bin/env python3
"""Condensed view of a kernel's instruction stream from a hipcc -S .s file: MFMA, LDS,
global/DMA loads, waits, barriers and branches kept; other instructions collapsed to '.'.
Usage: python tools/isa_view.py file.s KERNEL_SUBSTRING [--from s_barrier] [--chars 4000]"""
import argparse


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("s")
    ap.add_argument("kernel")
    ap.add_argument("--from_", "--from", dest="frm", default=None)
    ap.add_argument("--chars", type=int, default=4000)
    a = ap.parse_args()
    lines = open(a.s).read().split("\n")
    starts = [i for i, l in enumerate(lines) if l.split(":")[0].find(a.kernel) >= 0 and l.startswith("_Z")
              and ":" in l]
    i0 = starts[0]
    out = []
    for l in lines[i0 + 1:]:
        t = l.strip()
        if t.startswith(".Lfunc_end"):
            break
        if not t or t.startswith(";"):
            continue
        if t.startswith("."):
            if t.startswith(".LBB"):
                out.append(t.split()[0])
            continue
        op = t.split()[0]
        keep = (op.startswith(("s_waitcnt", "v_mfma", "ds_", "s_barrier", "s_cbranch", "v_exp", "s_setprio"))
                or "load" in op or "store" in op or "atomic" in op)
        out.append((t[:48] if op.startswith("s_waitcnt") else op) if keep else ".")
    comp, prev, n = [], None, 0
    for o in out:
        if o == prev:
            n += 1
        else:
            if prev is not None:
                comp.append(f"{prev} x{n}" if n > 1 else prev)
            prev, n = o, 1
    comp.append(prev)
    txt = "\n".join(comp)
    if a.frm and a.frm in txt:
        txt = txt[txt.index(a.frm):]
    print(txt[:a.chars])


if __name__ == "__main__":
    main()
