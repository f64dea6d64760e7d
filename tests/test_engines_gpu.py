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


BENCH = os.path.join(os.path.dirname(HERE), "bench.py")
# the headline path at 2 layers: Llama-3-8B dims, FSDP, bf16, --actv_ckpt auto, meta-built init
SMALL = ["--preset", "llama3_8b_fsdp", "--layers", "2", "--seq_len", "256", "--steps", "3", "--warmup", "1",
         "--actv_ckpt", "auto", "--data", "fixed_ids"]


def _bench(extra, timeout=420):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, BENCH] + SMALL + extra, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_headline_path_world2_one_gpu_matches_world1():
    """bench.py's own FSDP path, two ranks on cuda:0 over gloo (--one_device) at B=1 each, against
    world 1 at B=2 on the same global batches (--data fixed_ids); also: the forced world-1
    collective path reports a nonzero exposed-collective time."""
    one = _bench(["--gpus", "1", "--batch_size", "2"])
    two = _bench(["--gpus", "2", "--batch_size", "1", "--one_device"])
    forced = _bench(["--gpus", "1", "--batch_size", "2", "--force_comm"])
    assert "INVALID" in two["config"]["model"] and two["rccl_world"] == 2 and two["backend"] == "gloo"
    assert two["comm"]["deferred_init"] and one["comm"]["deferred_init"]
    a, b, c = one["loss_trace"], two["loss_trace"], forced["loss_trace"]
    assert len(a) == len(b) == len(c) == 4
    # bf16 weights; world 2 averages two half-batch gradients (another reduction order)
    assert b == pytest.approx(a, rel=2e-2), (a, b)
    assert c == pytest.approx(a, abs=1e-3), (a, c)       # world-1 collectives: copies, same arithmetic
    assert len(set(a)) == len(a)                         # four different batches, weights moving
    assert two["comm_exposed_ms"] > 0 and forced["comm_exposed_ms"] > 0, (two["comm"], forced["comm"])
    assert set(forced["comm"]["by_kind_rank0"]) >= {"all_gather", "reduce_scatter"}, forced["comm"]
    # achieved bandwidth per collective kind from RCCL's own start / end events
    bw = forced["comm"]["gbps_by_kind"]
    for kind in ("all_gather", "reduce_scatter"):
        assert bw[kind]["count"] > 0 and bw[kind]["algbw_gbps"] > 0, bw
        assert bw[kind]["timing"] == "rccl events", bw
    # warm-up collectives compared across ranks (parallel/seqcheck.py): the gloo pair and the
    # forced RCCL path both checked something; RCCL's init-time choices are in the JSON
    assert two["comm"]["order_check"]["enabled"] and two["comm"]["order_check"]["calls_checked_rank0"] > 0
    assert forced["comm"]["order_check"]["calls_checked_rank0"] > 0, forced["comm"]
    topo = forced["rccl_topology"]
    assert topo is not None and topo["lines"] > 0, topo
    assert topo.get("n_ranks") in (None, 1), topo
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "bench_world2_one_gpu.json"), "w") as f:
        json.dump({"world1": one, "world2_one_gpu": two, "world1_forced_comm": forced}, f, indent=1)
