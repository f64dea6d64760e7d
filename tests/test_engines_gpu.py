"""The N>1 engine code path on one GPU (RCCL world 1 + BLLM_FORCE_COMM=1, see
tests/_rehearse_engines.py): FSDP / ZeRO-1 / DDP with real RCCL collectives must train exactly
like the local engine.  Subprocess-isolated (own process group)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_engines_forced_comm_match_local_on_rccl():
    r = subprocess.run([sys.executable, os.path.join(HERE, "_rehearse_engines.py"), "fsdp,zero1,ddp"],
                       capture_output=True, text=True, timeout=300,
                       env={**os.environ, "BLLM_FORCE_COMM": "0"})
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for kind in ("fsdp", "zero1", "ddp"):
        k = res[kind]
        assert k["keys_match"]
        assert k["no_shard"] is False or k["no_comm"] is False, k   # the collective path ran
        # world-1 collectives are copies / sums of one: same arithmetic as the local engine
        assert k["losses"] == pytest.approx(res["ref_losses"], abs=1e-3), (kind, k["losses"], res["ref_losses"])
        assert k["max_param_diff"] < 1e-2, (kind, k["max_param_diff"])


def test_engines_world2_gloo_on_one_gpu():
    """Two ranks sharing cuda:0 over gloo (tests/_world2_one_gpu.py): real shards, gathers of the
    other rank's half, reduce-scatters of two different gradients and the cross-rank clip norm,
    all on the HIP kernels, train like one process on the whole batch."""
    r = subprocess.run([sys.executable, os.path.join(HERE, "_world2_one_gpu.py"), "fsdp,zero1,ddp"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    res = json.loads(lines[-2])
    for kind in ("fsdp", "zero1", "ddp"):
        k = res[kind]
        assert k["keys_match"], kind
        # bf16 weights, a different reduction order (two half-batch gradients averaged) than the
        # one-process reference: agreement to bf16 rounding over 3 AdamW steps
        assert k["losses"] == pytest.approx(res["ref_losses"], rel=2e-2), (kind, k["losses"], res["ref_losses"])
        assert k["max_rel_diff"] < 5e-2, (kind, k["max_rel_diff"])
