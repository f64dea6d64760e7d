#!/usr/bin/env python3
"""Per-kernel-class breakdown of ONE training step from a rocprofv3 kernel-trace database:
takes the dispatches from the last embedding-forward launch to the end of the trace.
Usage: python tools/step_breakdown.py run_results.db [--marker emb_fwd]"""
import argparse
import collections
import sqlite3


import re

# every in-house kernel (namespace bllm, csrc/*.hip) -> its class; a bllm kernel missing here is
# still labelled "bllm:<name>", never "torch:"
BLLM_CLASSES = {
    "wgrad_gemm_k": "wgrad_mfma (dW GEMM, csrc/gemm_wgrad.hip)", "wgrad4_k": "wgrad_mfma (dW GEMM, csrc/gemm_wgrad.hip)",
    "wgrad4p_k": "wgrad_mfma (dW GEMM, csrc/gemm_wgrad.hip)",
    "gemm_nt_k": "gemm_nt (forward-layout GEMM, csrc/gemm_nt.hip)", "gemm_nt4_k": "gemm_nt (forward-layout GEMM, csrc/gemm_nt.hip)",
    "gemm_nt4p_k": "gemm_nt (forward-layout GEMM, csrc/gemm_nt.hip)", "gemm_nt_pp_k": "gemm_nt (forward-layout GEMM, csrc/gemm_nt.hip)",
    "sum_partials_k": "sum_partials (split-K)", "transpose16_k": "weight transpose (dX operand, csrc/elementwise.hip)",
    "adamw_k": "adamw", "sqsum_partial_k": "sqsum", "sum_k": "sqsum",
    "attn_bwd_mfma_k": "attn_bwd_mfma", "attn_bwd_dq_k": "attn_bwd_dq", "attn_fwd_mfma_k": "attn_fwd",
    "attn_delta_k": "attn_delta", "attn_bwd_kv_reduce_k": "kv_reduce", "attn_decode_k": "attn_decode",
    "attn_fwd_f32_k": "attn (fp32 path)", "attn_bwd_dkv_f32_k": "attn (fp32 path)", "attn_bwd_dq_f32_k": "attn (fp32 path)",
    "attn_fwd_naive_k": "attn (naive path)", "attn_bwd_dkv_naive_k": "attn (naive path)", "attn_bwd_dq_naive_k": "attn (naive path)",
    "swiglu_fwd_k": "swiglu_fwd", "swiglu_fwd_rows_k": "swiglu_fwd", "swiglu_bwd_k": "swiglu_bwd", "swiglu_bwd_rows_k": "swiglu_bwd",
    "swiglu_bwd_lr_k": "swiglu_bwd (+ LoRA dX of the down projection)",
    "swiglu_bwd_lr_wg_k": "swiglu_bwd (+ LoRA dX of the down projection, gate/up dB, down dA)",
    "gelu_fwd_k": "gelu_fwd", "gelu_bwd_k": "gelu_bwd",
    "bwd_colsum_k": "bwd_colsum (GELU / dropout backward + bias column sums, csrc/elementwise.hip)",
    "col_reduce_k": "col_reduce",
    "dropout_add_k": "dropout", "rope_k": "rope", "rope_scalar_k": "rope",
    "norm_fwd_k": "norm_fwd", "norm_bwd_k": "norm_bwd", "norm_bwd_wave_k": "norm_bwd",
    "ce_fwd_k": "ce_fwd", "ce_bwd_k": "ce_bwd",
    "emb_fwd_k": "emb_", "emb_bwd_tok_k": "emb_", "emb_bwd_pos_k": "emb_",
    "lora_down_k": "lora (csrc/lora.hip)", "lora_down4_k": "lora (csrc/lora.hip)", "lora_head_bwd_k": "lora (csrc/lora.hip)", "lhb_usum_k": "lora (csrc/lora.hip)", "lora_up_k": "lora (csrc/lora.hip)", "lora_wgrad_k": "lora (csrc/lora.hip)",
    "lora_reduce_k": "lora (csrc/lora.hip)", "lora_pack_t_k": "lora (csrc/lora.hip)",
}
_MANGLED = re.compile(r"_ZN4bllm(?:12_GLOBAL__N_1)?(\d+)([A-Za-z_][A-Za-z0-9_]*)")
_DEMANGLED = re.compile(r"bllm::(?:\(anonymous namespace\)::)?([A-Za-z_][A-Za-z0-9_]*)")


def bllm_kernel(n):
    """Base name of an in-house kernel (mangled or demangled symbol), else None."""
    m = _MANGLED.search(n)
    if m:
        return m.group(2)[:int(m.group(1))]
    m = _DEMANGLED.search(n)
    return m.group(1) if m else None


def classify(n):
    if n.startswith(("Cijk", "Custom_Cijk")):
        return "gemm (hipBLASLt)"
    k = bllm_kernel(n)
    if k is not None:
        return BLLM_CLASSES.get(k, "bllm:" + k)
    if "copyBuffer" in n:
        return "copyBuffer"
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
