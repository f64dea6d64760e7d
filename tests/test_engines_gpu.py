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
