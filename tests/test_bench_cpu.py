"""bench.py's distributed branch, executed: torchrun at world 2, 4 (and 8 for FSDP) on gloo (``--device cpu``
tiny config) for every engine and preset, checking the driver's JSON-line contract.  On the GPU
node the same code path runs with RCCL; only the backend and the model size differ."""
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


def _run(n, extra, timeout=600):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    if n == 1:
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
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == 1 and out["value"] > 0
    assert "INVALID" in out["config"]["model"]  # a CPU run can never pass for a measurement
    return out


@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("parallel", ["fsdp", "ddp", "zero1"])
def test_bench_torchrun_gloo(n, parallel):
    out = _run(n, ["--parallel", parallel])
    assert out["config"]["parallelism"] == f"{parallel}{n}"
    assert out["config"]["global_batch"] == 2 * n
    assert out["config"]["actv_ckpt"] == "full"


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
