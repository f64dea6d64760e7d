"""Kernel debug mode (SURVEY §5 'race detection / sanitizers': debug build with bounds checks,
launch-blocking execution).  ``tools/build_ext.py --debug`` builds ``_C_debug.so`` with
device-side checks (csrc/common.h BLLM_DASSERT); ``BLLM_KERNEL_DEBUG=1`` loads it and makes
every op synchronise and raise at the op whose kernel failed a check.  The checked kernels
clamp the bad index after recording it, so the debug run itself never touches memory out of
bounds.  Run in a child process: the two builds register the same op library."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import torch
from building_llm_from_scratch_amd import ops
ops.load_ext(required=True)
assert torch.ops.bllm.kernel_debug_build()
dev = "cuda"
wte = torch.randn(100, 64, device=dev, dtype=torch.bfloat16)
ok = torch.randint(0, 100, (2, 8), device=dev)
ops.embedding_fwd(ok, wte, None, 8)
bad = ok.clone(); bad[1, 3] = 105
try:
    ops.embedding_fwd(bad, wte, None, 8)
    raise SystemExit("embedding: no error")
except RuntimeError as e:
    assert "embedding token id" in str(e), e
ops.embedding_fwd(ok, wte, None, 8)          # the word was reset
logits = torch.randn(16, 50, device=dev, dtype=torch.bfloat16)
tgt = torch.randint(0, 50, (16,), device=dev)
tgt[2] = -100
ops.ce_fwd(logits, tgt)
tgt[5] = 50
try:
    ops.ce_fwd(logits, tgt)
    raise SystemExit("ce: no error")
except RuntimeError as e:
    assert "cross-entropy target" in str(e), e
print("DEBUG-MODE-OK")
"""


@pytest.mark.gpu
def test_kernel_debug_mode_reports_out_of_range_indices():
    lib = os.path.join(ROOT, "building_llm_from_scratch_amd", "_C_debug.so")
    assert os.path.isfile(lib), "build it with: python tools/build_ext.py --debug"
    env = dict(os.environ, BLLM_KERNEL_DEBUG="1")
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "DEBUG-MODE-OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.gpu
def test_release_build_has_no_checks():
    import torch
    from building_llm_from_scratch_amd import ops
    ops.load_ext(required=True)
    if os.environ.get("BLLM_KERNEL_DEBUG", "0") in ("", "0"):
        assert not torch.ops.bllm.kernel_debug_build()
        assert torch.ops.bllm.debug_error() == 0
