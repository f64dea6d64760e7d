"""Loader for the in-tree HIP extension ``building_llm_from_scratch_amd/_C.so``.

The library registers ``torch.ops.bllm.*`` (TORCH_LIBRARY in csrc/binding.cpp) and is built
for gfx950 by ``tools/build_ext.py`` (``python setup.py build_ext`` / ``__graft_entry__.build``).
With ``BLLM_KERNEL_DEBUG=1`` the kernel-debug build ``_C_debug.so`` (``tools/build_ext.py
--debug``: device-side bounds checks) is loaded instead.
"""
from __future__ import annotations

import os
import threading

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_debug() -> bool:
    return os.environ.get("BLLM_KERNEL_DEBUG", "0") not in ("", "0")


_LIB_PATH = os.path.join(_PKG, "_C_debug.so" if kernel_debug() else "_C.so")
_lock = threading.Lock()
_state = {"loaded": False, "error": None}


def lib_path() -> str:
    return _LIB_PATH


def load_ext(required: bool = False) -> bool:
    if _state["loaded"]:
        return True
    with _lock:
        if _state["loaded"]:
            return True
        if not os.path.isfile(_LIB_PATH):
            _state["error"] = (f"HIP extension not built: {_LIB_PATH} missing (run `python tools/build_ext.py"
                               + (" --debug`)" if kernel_debug() else "` or `python setup.py build_ext`)"))
        else:
            try:
                torch.ops.load_library(_LIB_PATH)
                _state["loaded"] = True
                _state["error"] = None
            except Exception as e:  # pragma: no cover - depends on the box
                _state["error"] = f"failed to load {_LIB_PATH}: {e}"
    if not _state["loaded"] and required:
        raise RuntimeError(_state["error"] + " — GPU ops have no fallback.")
    return _state["loaded"]


def ext_available() -> bool:
    return load_ext(required=False)
