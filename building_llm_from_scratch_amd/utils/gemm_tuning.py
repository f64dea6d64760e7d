"""Per-shape GEMM selection tables (PyTorch TunableOp) shared by ``bench.py`` and the CLI.

The library GEMMs (hipBLASLt / rocBLAS) pick a kernel per shape with a heuristic; for the
shipped presets a one-off tuning run on an MI355X recorded the fastest solution per shape in
``configs/tunableop_*_mi355x.csv`` (the headline's table routes gate/up to rocBLAS at 1.72 PF,
``profiles/r5/fused_epilogues_ab.md``).  A run that loads the table in read-only mode
(``PYTORCH_TUNABLEOP_TUNING=0``) uses the recorded solution for every shape in it and the
heuristic for every other shape, so a table is harmless for a batch it was not tuned for.

TunableOp reads ``PYTORCH_TUNABLEOP_*`` when the first GEMM runs, so ``install_table`` must be
called before the model is built.
"""
from __future__ import annotations

import os
import shutil
import tempfile
import warnings
from typing import Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (model, size) -> table tuned on one MI355X for that preset's shapes
TABLES = {
    ("llama3", "8B"): "configs/tunableop_llama3_8b_b40_mi355x.csv",
    ("GPT2", "774M"): "configs/tunableop_gpt2_774m_b64_mi355x.csv",
}


def resolve_table(spec: Optional[str], model: str = "", size: str = "") -> Optional[str]:
    """``spec``: a CSV path (relative to the repo root or absolute), ``"auto"`` (the shipped
    table of ``(model, size)`` if there is one) or ``"none"`` / ``""`` / None.  Returns an
    absolute path to an existing file, or None."""
    if not spec or spec == "none":
        return None
    if spec == "auto":
        spec = TABLES.get((model, str(size)))
        if spec is None:
            return None
    path = spec if os.path.isabs(spec) else os.path.join(ROOT, spec)
    if not os.path.exists(path):
        warnings.warn(f"TunableOp table {spec!r} not found: GEMMs use the libraries' heuristics")
        return None
    return path


def install_table(path: Optional[str], local_rank: int = 0) -> Optional[str]:
    """Point TunableOp at a private copy of ``path`` (read-only lookups, no tuning).  A copy and
    not a symlink: whatever TunableOp writes back at exit can never reach the shipped table.
    Returns the directory holding the copy (None when ``path`` is None)."""
    if not path:
        return None
    d = tempfile.mkdtemp(prefix="bllm_tunableop_")
    # TunableOp reads <FILENAME with %d -> device ordinal>
    shutil.copyfile(path, os.path.join(d, f"results{local_rank}.csv"))
    os.environ.update(PYTORCH_TUNABLEOP_ENABLED="1", PYTORCH_TUNABLEOP_TUNING="0",
                      PYTORCH_TUNABLEOP_FILENAME=os.path.join(d, "results%d.csv"))
    return d
