#!/usr/bin/env python3
"""Build the gfx950 kernel library in-tree: ``building_llm_from_scratch_amd/_C.so``.

* every ``csrc/*.hip`` is compiled with ``hipcc --offload-arch=gfx950`` WITHOUT PyTorch
  headers (fast, ~seconds per file);
* ``csrc/binding.cpp`` (TORCH_LIBRARY registration) is compiled against the PyTorch ROCm
  headers;
* everything is linked against PyTorch's own HIP runtime (``torch/lib/libamdhip64.so``,
  same SONAME as /opt/rocm's) so one runtime instance is used in-process.

Incremental (mtime + flags hash), parallel (``-j``).  No hipify, no CUDA sources.
``--debug`` builds the kernel-debug variant ``_C_debug.so`` instead (-O1 -g and
-DBLLM_KERNEL_DEBUG: device-side bounds checks, common.h ``BLLM_DASSERT``), loaded in place of
``_C.so`` when ``BLLM_KERNEL_DEBUG=1`` (ops then synchronise and check after every call).
Usage: ``python tools/build_ext.py [-j N] [--clean] [--debug]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
OUT = os.path.join(ROOT, "building_llm_from_scratch_amd", "_C.so")
OUT_DEBUG = os.path.join(ROOT, "building_llm_from_scratch_amd", "_C_debug.so")
ARCH = os.environ.get("BLLM_ARCH", "gfx950")


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required)")


def _needs(src: str, obj: str, flags: str, deps) -> bool:
    stamp = obj + ".flags"
    if not os.path.exists(obj) or not os.path.exists(stamp):
        return True
    if open(stamp).read() != hashlib.sha1(flags.encode()).hexdigest():
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def _run(cmd, obj, flags):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(obj + ".flags", "w") as f:
        f.write(hashlib.sha1(flags.encode()).hexdigest())
    return obj, r.stderr


def build(jobs: int = 8, clean: bool = False, debug: bool = False, verbose: bool = False) -> str:
    hipcc = _hipcc()
    tdir, tinc, tlib, abi = _torch_paths()
    bdir = BUILD + "_debug" if debug else BUILD
    out = OUT_DEBUG if debug else OUT
    if clean and os.path.isdir(bdir):
        shutil.rmtree(bdir)
    os.makedirs(bdir, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    opt = ["-O1", "-DBLLM_KERNEL_DEBUG=1"] if debug else ["-O3"]
    common = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
              "-Wno-unused-result", f"-I{CSRC}"] + opt
    jobs_list = []
    objs = []
    for f in sorted(os.listdir(CSRC)):
        src = os.path.join(CSRC, f)
        if f.endswith(".hip"):
            obj = os.path.join(bdir, f + ".o")
            cmd = [hipcc] + common + ["-c", src, "-o", obj]
        elif f.endswith(".cpp"):
            obj = os.path.join(bdir, f + ".o")
            py_inc = sysconfig.get_paths()["include"]
            cmd = [hipcc, "-std=c++17", "-fPIC", "-O2", f"-I{CSRC}", f"-I{py_inc}"] + (
                ["-DBLLM_KERNEL_DEBUG=1"] if debug else []) + [f"-I{i}" for i in tinc] + [
                f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
                "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_C", "-Wno-deprecated-declarations",
                "-c", src, "-o", obj]
        else:
            continue
        objs.append(obj)
        flags = " ".join(cmd)
        if _needs(src, obj, flags, headers):
            jobs_list.append((cmd, obj, flags))
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = [ex.submit(_run, c, o, fl) for c, o, fl in jobs_list]
            for fu in cf.as_completed(futs):
                obj, err = fu.result()
                if verbose:
                    print(f"[build] {os.path.basename(obj)}" + (f"\n{err}" if err.strip() else ""))
    link_needed = not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs)
    if link_needed:
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + [
            f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch", "-lamdhip64", "-lhipblaslt",
            f"-Wl,-rpath,{tlib}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[build] linked {out}")
    build_host(verbose=verbose)
    return out


def build_host(verbose: bool = False):
    """Host-side native modules (csrc/host/*.cpp, pybind11, g++ -O3): the BPE tokenizer core."""
    import pybind11
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    hdir = os.path.join(CSRC, "host")
    outs = []
    for f in sorted(os.listdir(hdir)) if os.path.isdir(hdir) else []:
        if not f.endswith(".cpp"):
            continue
        src = os.path.join(hdir, f)
        out = os.path.join(ROOT, "building_llm_from_scratch_amd", "_" + f[:-4] + suffix)
        cmd = [os.environ.get("CXX", "g++"), "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
               f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", src, "-o", out]
        deps = [src] + [os.path.join(hdir, h) for h in os.listdir(hdir) if h.endswith(".h")]
        if not os.path.exists(out) or max(os.path.getmtime(d) for d in deps) > os.path.getmtime(out):
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"host build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
            if verbose:
                print(f"[build] host {os.path.basename(out)}")
        outs.append(out)
    return outs


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args()
    try:
        print(build(a.jobs, a.clean, a.debug, verbose=True))
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
