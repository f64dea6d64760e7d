"""Checkpoint / resume (the reference saves weights only and has no resume path;
this framework adds ``--save_resume_state`` / ``--resume``).

Done criterion: train N steps, save, resume, train to 2N — must equal an uninterrupted 2N-step
run (params and per-step losses), for the single-process path (GPT-2 with dropout: the
dropout RNG counter is part of the state) and for DDP / ZeRO-1 / FSDP at gloo world 2."""
import json
import os
import subprocess
import sys
from types import SimpleNamespace

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, cwd, timeout=900):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONUNBUFFERED="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "main.py")] + args, cwd=cwd, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _losses(path):
    return {r["step"]: r["batch_loss"] for r in map(json.loads, open(path))}


def _roundtrip(tmp_path, model_args, extra=(), steps=8, half=4):
    data = tmp_path / "data"
    common = model_args + ["--data_dir", str(data), "--synthetic_data", "--n_epochs", "1", "--eval_freq", "1",
                           "--print_sample_iter", "3", "--batch_size", "2", "--device", "cpu", "--no_plot",
                           "--sample_tokens", "2", "--save_resume_state", "--max_steps", str(steps),
                           "--save_ckpt_freq", str(half), "--num_workers", "0"] + list(extra)
    a, b = tmp_path / "a", tmp_path / "b"
    _run(common + ["--output_dir", str(a), "--metrics_file", str(tmp_path / "a.jsonl")], tmp_path)
    ck = a / f"model_pg_{half}.pth"
    assert ck.exists() and any(p.name.startswith(f"model_pg_{half}.state") for p in a.iterdir())
    _run(common + ["--output_dir", str(b), "--metrics_file", str(tmp_path / "b.jsonl"), "--resume", str(ck)],
         tmp_path)
    la, lb = _losses(tmp_path / "a.jsonl"), _losses(tmp_path / "b.jsonl")
    assert sorted(lb) == list(range(half + 1, steps)), sorted(lb)
    for s in lb:
        assert abs(la[s] - lb[s]) <= 1e-6, (s, la[s], lb[s])
    sa = torch.load(a / "model_pg_final.pth", weights_only=True)
    sb = torch.load(b / "model_pg_final.pth", weights_only=True)
    assert set(sa) == set(sb)
    for k in sa:
        assert torch.allclose(sa[k].float(), sb[k].float(), atol=1e-6, rtol=0), (k, (sa[k] - sb[k]).abs().max())


def test_resume_single_process_gpt2_dropout(tmp_path):
    _roundtrip(tmp_path, ["--model", "GPT2", "--num_params", "124M", "--debug"])


@pytest.mark.parametrize("mode", [[], ["--use_zero_opt"], ["--use_fsdp"]], ids=["ddp", "zero1", "fsdp"])
def test_resume_gloo_world2(tmp_path, mode):
    os.environ["MASTER_PORT"] = str(_free_port())
    try:
        _roundtrip(tmp_path, ["--model", "llama3_2", "--num_params", "1B", "--debug", "--run_type", "multi_gpu",
                              "--backend", "gloo", "--nprocs", "2"], extra=mode)
    finally:
        os.environ.pop("MASTER_PORT", None)


@pytest.mark.parametrize("ckpt_name", ["model_pg_3_interrupted.pth", "model_pg_final.pth"])
def test_bf16_resume_weights_survive_first_step(tmp_path, ckpt_name):
    """a bf16 resume from an ``_interrupted`` / ``final`` checkpoint (no state
    file) must not be reverted by the optimizer's stale fp32 master at the next step."""
    from building_llm_from_scratch_amd.builder import build_components
    from building_llm_from_scratch_amd.cli import build_parser

    args = build_parser().parse_args(["--model", "llama3_2", "--num_params", "1B", "--debug", "--data_type", "bf16",
                                      "--device", "cpu", "--data_dir", str(tmp_path)])
    args.world_size = 1
    torch.manual_seed(5)
    _, m0, _, _, _ = build_components(0, torch.device("cpu"), args)
    sd = {k: (v + 0.25 * torch.randn_like(v.float()).to(v.dtype)) if v.is_floating_point() else v
          for k, v in m0.state_dict().items()}
    torch.save(sd, tmp_path / ckpt_name)
    args.resume = str(tmp_path / ckpt_name)
    torch.manual_seed(6)   # a different random init: only the load can make them equal
    _, m, opt, _, _ = build_components(0, torch.device("cpu"), args)
    for g in opt.param_groups:
        g["lr"] = 0.0
    idx = torch.randint(0, 100, (2, 8))
    m(idx, idx).backward()
    opt.clip_grad_norm_(1.0)
    opt.step()
    cur = m.state_dict()
    for k, v in sd.items():
        if k.endswith((".mask", ".cos", ".sin")):
            continue
        assert torch.equal(cur[k].float(), v.to(torch.bfloat16).float()), k   # params are bf16
