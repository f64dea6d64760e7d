"""bench.py's distributed branch, executed on gloo (``--device cpu`` tiny config) for every engine
and preset, checking the driver's JSON-line contract: under torchrun at world 2 and 4, and
self-launched (``python bench.py --gpus N``, no torchrun: bench.py spawns the N ranks itself) at
world 2, 4 and 8.  On the GPU node the same code path runs with RCCL; only the backend and the
model size differ."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(n, extra, timeout=600, spawn=False):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    if n == 1 or spawn:
        cmd = [sys.executable, BENCH]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", f"--master-port={_port()}", BENCH]
    cmd += ["--gpus", str(n), "--device", "cpu", "--steps", "2", "--warmup", "1"] + extra
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd="/tmp")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # exactly one JSON line, from rank 0
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    warm = int(extra[extra.index("--warmup") + 1]) if "--warmup" in extra else 1
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == warm and out["value"] > 0
    assert out["rccl_world"] == n                # the process group really had N ranks
    assert len(out["per_rank"]["ms_per_step"]) == n
    assert out["per_rank"]["ms_per_step_max"] == out["ms_per_step"]
    assert out["launcher"] == ("spawn" if spawn and n > 1 else ("single" if n == 1 else "torchrun"))
    assert "INVALID" in out["config"]["model"]  # a CPU run can never pass for a measurement
    # box telemetry fields are always present; on CPU they are empty / null
    tel = out["telemetry"]
    assert tel["rank0"]["source"] is None and tel["rank0"]["samples"] == 0
    assert len(tel["sclk_mhz_avg_per_rank"]) == n and all(v is None for v in tel["sclk_mhz_avg_per_rank"])
    assert "torch" in out["versions"] and "hip" in out["versions"]
    assert out["tunableop"] is None
    return out


@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("parallel", ["fsdp", "ddp", "zero1"])
def test_bench_torchrun_gloo(n, parallel):
    out = _run(n, ["--parallel", parallel])
    assert out["config"]["parallelism"] == f"{parallel}{n}"
    assert out["config"]["global_batch"] == 2 * n
    assert out["config"]["actv_ckpt"] == "auto"
    assert out["ckpt_plan"]["full"] + out["ckpt_plan"]["selective"] == 2   # checkpointing stays on


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("parallel", ["fsdp", "ddp", "zero1"])
def test_bench_self_spawn(n, parallel):
    """``python bench.py --gpus N`` without torchrun: bench.py starts the N ranks itself."""
    out = _run(n, ["--parallel", parallel], spawn=True)
    assert out["config"]["parallelism"] == f"{parallel}{n}"
    assert out["config"]["global_batch"] == 2 * n


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("preset", ["llama32_1b_lora_alpaca", "llama2_7b_fsdp_mp", "gpt2_774m_ddp"])
def test_bench_self_spawn_presets(preset, n):
    out = _run(n, ["--preset", preset], spawn=True)
    assert out["config"]["parallelism"].endswith(str(n))


def test_bench_reference_ckpt():
    """``--actv_ckpt full`` is the reference's checkpoint_sequential(segments=n_layers)."""
    out = _run(1, ["--actv_ckpt", "full"])
    assert out["config"]["ckpt_blocks"].startswith("1/2 recomputed")


def test_bench_torchrun_gloo_world8_fsdp():
    """The driver's largest scaling point (8 ranks, FSDP full-shard + full checkpointing)."""
    test_bench_torchrun_gloo(8, "fsdp")


def test_bench_world1_uses_fsdp_engine():
    out = _run(1, [])
    assert out["config"]["engine"].startswith("FSDPEngine")
    assert out["config"]["parallelism"] == "fsdp1"


@pytest.mark.parametrize("preset,n", [("llama32_1b_lora_alpaca", 2), ("llama2_7b_fsdp_mp", 2), ("gpt2_774m_ddp", 2)])
def test_bench_presets(preset, n):
    out = _run(n, ["--preset", preset])
    if preset == "llama32_1b_lora_alpaca":
        assert out["config"]["lora"] == {"rank": 16, "alpha": 32}
        assert str(out["config"]["seq_len"]).startswith("variable")
    if preset == "llama2_7b_fsdp_mp":
        assert out["config"]["mixed_precision"] == "bf16"


@pytest.mark.parametrize("parallel", ["fsdp", "ddp", "zero1"])
def test_bench_world8_self_diagnosing_fields(parallel):
    """World 8 (gloo): the line carries what a first multi-GPU run needs to be read —
    every rank's exposed collective wait per step, the prefetch depth / bucket size the engine
    chose, a meta-built (no broadcast) init — and the headline's data path is the reference's
    (DataloaderPT windows through a DistributedSampler) with disjoint windows per rank."""
    out = _run(8, ["--parallel", parallel], spawn=True)
    assert len(out["per_rank"]["comm_exposed_ms"]) == 8
    assert out["comm_exposed_ms"] == max(out["per_rank"]["comm_exposed_ms"]) and out["comm_exposed_ms"] > 0
    kinds = out["comm"]["by_kind_rank0"]
    if parallel == "fsdp":
        assert out["comm"]["fsdp_prefetch"] >= 1 and kinds["all_gather"]["waits"] > 0
        assert kinds["reduce_scatter"]["waits"] > 0 and kinds["all_reduce"]["waits"] == 2   # clip, per step
    else:
        assert out["comm"]["bucket_mib"] == 256.0
    assert out["comm"]["deferred_init"] is True
    assert "DataloaderPT" in out["data"] and "DistributedSampler over 8 ranks" in out["data"]
    dc = out["data_check"]
    assert dc["sampler"] == "DistributedSampler" and dc["disjoint_across_ranks"] is True
    assert dc["windows_per_rank_used"] == 2 * 3    # micro-batch 2 x (1 warm-up + 2 timed steps)
    # the warm-up step's collectives were compared across the 8 ranks (parallel/seqcheck.py)
    oc = out["comm"]["order_check"]
    assert oc["enabled"] and oc["calls_checked_rank0"] > 0 and oc["steps"] == 1
    assert "rccl_topology" not in out       # gloo: nothing to capture


def test_bench_random_ids_arm():
    """``--data random_ids``: the A/B arm with device-resident random token ids."""
    out = _run(1, ["--data", "random_ids"])
    assert out["data"].startswith("synthetic random token ids") and "data_check" not in out


@pytest.mark.parametrize("parallel", ["fsdp", "ddp", "zero1"])
def test_bench_world2_matches_world1_on_the_global_batch(parallel):
    """``--data fixed_ids``: world 2 at B=1 per rank trains the same global batches as world 1 at
    B=2, so the engines' sharded path (real shards, cross-rank reduce-scatter / all-gather, clip
    norm over ranks) must reproduce the world-1 loss trace."""
    one = _run(1, ["--parallel", parallel, "--data", "fixed_ids", "--batch_size", "2"])
    two = _run(2, ["--parallel", parallel, "--data", "fixed_ids", "--batch_size", "1"], spawn=True)
    assert one["config"]["global_batch"] == two["config"]["global_batch"] == 2
    a, b = one["loss_trace"], two["loss_trace"]
    assert len(a) == len(b) == 3
    assert max(abs(x - y) for x, y in zip(a, b)) < 1e-4, (a, b)
    assert a[-1] != a[0]                          # the optimizer really moved the weights


def test_telemetry_summary_math():
    """GpuTelemetry's reductions on canned SMU samples (no GPU): averages, residency fractions
    from accumulator deltas, N/A sentinels ignored."""
    from building_llm_from_scratch_amd.utils.telemetry import GpuTelemetry, tunableop_status
    t = GpuTelemetry.__new__(GpuTelemetry)
    t.smi, t.h, t.interval = None, None, 0.25
    t.samples = [{"sclk": 2000.0, "mclk": 1900.0, "power": 1300.0, "hotspot": 80.0, "hbm": 70.0, "throttle": 0,
                  "indep": 0},
                 {"sclk": 1800.0, "mclk": 1900.0, "power": 1400.0, "hotspot": 90.0, "hbm": 72.0, "throttle": 4,
                  "indep": 0}]
    t._m0 = {"accumulation_counter": 100, "ppt_residency_acc": 10, "socket_thm_residency_acc": 0,
             "xgmi_read_data_acc": [0, 5, 0xFFFFFFFFFFFFFFFF]}
    t._m1 = {"accumulation_counter": 300, "ppt_residency_acc": 110, "socket_thm_residency_acc": 0,
             "xgmi_read_data_acc": [7, 9, 0xFFFFFFFFFFFFFFFF]}
    s = t.summary()
    assert s["sclk_mhz_avg"] == 1900.0 and s["sclk_mhz_min"] == 1800.0 and s["power_w_max"] == 1400.0
    assert s["throttle_status_nonzero_frac"] == 0.5
    assert s["limit_residency"] == {"ppt": 0.5, "socket_thm": 0.0}
    assert s["xgmi"]["xgmi_read_kb"] == 11
    assert tunableop_status(None) is None
    st = tunableop_status(os.path.join(ROOT, "configs", "tunableop_llama3_8b_b40_mi355x.csv"))
    assert st["file_rows"] >= 5    # validators compared on a GPU box only


@pytest.mark.parametrize("parallel", ["fsdp", "ddp"])
def test_bench_warmup_comm_adaptation_world4(parallel, monkeypatch):
    """A slow link on rank 1 only (injected wait, BLLM_COMM_DELAY_MS) makes the exposed
    collective wait exceed 2 % of the step; the warm-up adaptation then grows the FSDP prefetch
    depth / the DDP bucket size.  The decision uses the MAX over ranks, so every rank ends on
    the same value (same collective order), and the JSON carries the achieved bandwidth."""
    monkeypatch.setenv("BLLM_COMM_DELAY_MS", "40")
    monkeypatch.setenv("BLLM_COMM_DELAY_RANKS", "1")
    extra = ["--parallel", parallel, "--warmup", "4"] + (["--fsdp_prefetch", "1"] if parallel == "fsdp" else [])
    if parallel == "ddp":
        extra += ["--bucket_mb", "0.02", "--actv_ckpt", "none"]
    # (--warmup given twice: argparse keeps the last)
    out = _run(4, extra)
    c = out["comm"]
    assert len(c["adapted"]) == 3                      # warm-up steps 1..3 (step 0 is cold)
    if parallel == "fsdp":
        assert c["fsdp_prefetch"] > 1 and any("prefetch_new" in r for r in c["adapted"])
        assert len(set(c["per_rank_fsdp_prefetch"])) == 1 and c["per_rank_fsdp_prefetch"][0] == c["fsdp_prefetch"]
        assert c["gbps_by_kind"]["all_gather"]["count"] > 0 and c["gbps_by_kind"]["all_gather"]["algbw_gbps"] > 0
    else:
        assert c["bucket_mib"] > 0.02 and any("bucket_mib_new" in r for r in c["adapted"])
        assert len(set(c["per_rank_bucket_mib"])) == 1
        assert c["gbps_by_kind"]["all_reduce"]["busbw_gbps"] > 0
