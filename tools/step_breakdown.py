#!/usr/bin/env python3
"""Per-kernel-class breakdown of ONE training step from a rocprofv3 kernel-trace database:
takes the dispatches from the last embedding-forward launch to the end of the trace.
Usage: python tools/step_breakdown.py run_results.db [--marker emb_fwd]"""
import argparse
import collections
import sqlite3


def classify(n):
    if n.startswith(("Cijk", "Custom_Cijk")):
        return "gemm (hipBLASLt)"
    if "wgrad_gemm_k" in n or "wgrad4_k" in n or "wgrad4p_k" in n:
        return "wgrad_mfma (dW GEMM, csrc/gemm_wgrad.hip)"
    if "gemm_nt" in n:
        return "gemm_nt (forward-layout GEMM, csrc/gemm_nt.hip)"
    if "sum_partials" in n:
        return "sum_partials (split-K)"
    if "transpose16" in n:
        return "weight transpose (dX operand, csrc/elementwise.hip)"
    for k in ("adamw", "sqsum", "attn_bwd_mfma", "attn_bwd_dq", "attn_fwd", "attn_delta", "kv_reduce", "swiglu_fwd",
              "swiglu_bwd", "gelu", "rope", "norm_fwd", "norm_bwd", "col_reduce", "ce_fwd", "ce_bwd", "emb_",
              "copyBuffer", "dropout"):
        if k in n:
            return k
    return "torch:" + n.split("<")[0][-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="emb_fwd")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = db.execute("select name,start,end from kernels order by start").fetchall()
    # rocpd may truncate or demangle kernel names differently per table: prefer the full symbol
    try:
        full = dict(db.execute("select id,kernel_name from rocpd_info_kernel_symbol").fetchall())
        ids = db.execute("select kernel_id from kernels order by start").fetchall()
        rows = [(full.get(k[0], r[0]) or r[0], r[1], r[2]) for r, k in zip(rows, ids)]
    except sqlite3.Error:
        pass
    idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
    seq = rows[idx[-1]:]
    span = (seq[-1][2] - seq[0][1]) / 1e6
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e in seq:
        k = classify(n)
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e6
    busy = sum(v[1] for v in agg.values())
    print(f"step span {span:.2f} ms, kernel-busy {busy:.2f} ms, {len(seq)} dispatches\n")
    print("| kernel class | calls | ms/step | share |\n|---|---|---|---|")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| {k} | {c} | {t:.2f} | {100 * t / busy:.1f}% |")


if __name__ == "__main__":
    main()
