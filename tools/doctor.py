#!/usr/bin/env python3
"""Environment check (reference req_libraries.py:1-55, extended for the MI355X stack).

Reports, without installing anything: Python deps used by the framework, the ROCm toolchain
(hipcc, rocprofv3, RCCL), the GPU architecture (gfx950 expected), the in-tree HIP extension
(built? loadable? its kernels registered?) and the torch.distributed backends.
Exit status 1 if a REQUIRED item is missing.
Usage: python tools/doctor.py [--json]"""
import argparse
import importlib
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REQUIRED_PY = ["torch", "numpy"]
OPTIONAL_PY = {"sentencepiece": "Llama-2 tokenizer", "safetensors": "HF weight loading",
               "tiktoken": "tiktoken BPE files (a built-in BPE reader is used when absent)",
               "transformers": "HF GPT-2 checkpoints in .bin form", "matplotlib": "losses.pdf plot",
               "hypothesis": "property tests", "pytest": "test suite", "tqdm": "progress bars"}


def _ver(mod):
    try:
        m = importlib.import_module(mod)
        return getattr(m, "__version__", "ok")
    except Exception as e:  # noqa: BLE001
        return None if isinstance(e, ImportError) else f"error: {e}"


def _run(cmd):
    try:
        return subprocess.run(cmd, capture_output=True, text=True, timeout=60).stdout
    except Exception:  # noqa: BLE001
        return ""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    rep, missing = {}, []
    for m in REQUIRED_PY:
        rep[m] = _ver(m)
        if not rep[m]:
            missing.append(m)
    rep["optional"] = {m: (_ver(m) or f"absent ({why})") for m, why in OPTIONAL_PY.items()}
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    rep["hipcc"] = shutil.which("hipcc") or (os.path.join(rocm, "bin/hipcc") if os.path.exists(os.path.join(rocm, "bin/hipcc")) else None)
    rep["rocprofv3"] = shutil.which("rocprofv3") or (os.path.join(rocm, "bin/rocprofv3") if os.path.exists(os.path.join(rocm, "bin/rocprofv3")) else None)
    rccl = [p for p in (os.path.join(rocm, "lib/librccl.so"), os.path.join(rocm, "lib/librccl.so.1")) if os.path.exists(p)]
    rep["rccl"] = rccl[0] if rccl else None
    if not rep["hipcc"]:
        missing.append("hipcc")
    import torch
    rep["torch_hip"] = getattr(torch.version, "hip", None)
    rep["gpu_count"] = torch.cuda.device_count()
    archs = []
    if rep["gpu_count"]:
        for i in range(rep["gpu_count"]):
            p = torch.cuda.get_device_properties(i)
            archs.append(getattr(p, "gcnArchName", p.name))
    rep["gpu_arch"] = archs
    rep["gfx950"] = all("gfx950" in x for x in archs) if archs else None
    import torch.distributed as dist
    rep["dist_backends"] = {b: getattr(dist, f"is_{b}_available", lambda: False)() for b in ("nccl", "gloo")}
    so = os.path.join(ROOT, "building_llm_from_scratch_amd", "_C.so")
    rep["extension_built"] = os.path.exists(so)
    try:
        from building_llm_from_scratch_amd.ops import _ext
        _ext.load_ext(required=True)
        rep["extension_loaded"] = True
        rep["extension_ops"] = [n for n in ("rmsnorm_fwd", "flash_attn_fwd", "flash_attn_bwd", "adamw_step", "ce_fwd") if hasattr(torch.ops.bllm, n)]
    except Exception as e:  # noqa: BLE001
        rep["extension_loaded"] = f"no: {e}"
    if a.json:
        print(json.dumps(rep, indent=1, default=str))
    else:
        for k, v in rep.items():
            print(f"{k:18s} {v}")
        print("\nmissing required:", missing or "none")
    sys.exit(1 if missing else 0)


if __name__ == "__main__":
    main()
