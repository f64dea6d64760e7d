"""The reference CLI (``main.py``) end to end on the GPU: GPT-2 in the reference's default fp32
and in bf16, Llama-3 through the self-spawned multi_gpu path on an RCCL process group with FSDP,
activation checkpointing and --mixed_precision bf16 (the headline configuration's CLI form,
world 1), and a LoRA instruction finetune.  Tiny ``--debug`` models, a few steps each; the
checkpoint / plot contract is checked as in test_cli_e2e.py."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _run(args, tmp_path, timeout=300):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONUNBUFFERED="1")
    cmd = [sys.executable, os.path.join(ROOT, "main.py")] + args
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_cli_gpt2_pretrain_gpu(tmp_path, dtype):
    out = tmp_path / "ckpt"
    _run(["--model", "GPT2", "--num_params", "124M", "--debug", "--data_dir", str(tmp_path / "data"),
          "--synthetic_data", "--output_dir", str(out), "--n_epochs", "1", "--max_steps", "4", "--eval_freq", "2",
          "--save_ckpt_freq", "2", "--print_sample_iter", "2", "--batch_size", "4", "--data_type", dtype,
          "--sample_tokens", "4", "--no_plot"], tmp_path)
    for n in ("model_pg_0.pth", "model_pg_2.pth", "model_pg_final.pth"):
        assert (out / n).exists(), n
    sd = torch.load(out / "model_pg_final.pth", weights_only=True)
    assert all(torch.isfinite(v.float()).all() for v in sd.values() if v.is_floating_point())


def test_cli_llama3_fsdp_ckpt_mixed_precision_rccl(tmp_path):
    out = tmp_path / "ckpt"
    _run(["--model", "llama3", "--num_params", "8B", "--debug", "--run_type", "multi_gpu", "--use_fsdp",
          "--use_actv_ckpt", "--mixed_precision", "bf16", "--nprocs", "1", "--data_dir", str(tmp_path / "data"),
          "--synthetic_data", "--output_dir", str(out), "--n_epochs", "1", "--max_steps", "3", "--eval_freq", "2",
          "--save_ckpt_freq", "100", "--print_sample_iter", "100", "--batch_size", "2", "--no_plot",
          "--sample_tokens", "2"], tmp_path)
    sd = torch.load(out / "model_pg_final.pth", weights_only=True)
    assert "trf_blocks.0.norm1.weight" in sd and "out_head.weight" in sd


def test_cli_llama32_lora_finetune_gpu(tmp_path):
    out = tmp_path / "ckpt"
    _run(["--model", "llama3_2", "--num_params", "1B", "--debug", "--finetune", "--dataset", "alpaca",
          "--data_dir", str(tmp_path / "alpaca"), "--synthetic_data", "--use_lora", "--lora_rank", "4",
          "--data_type", "bf16", "--output_dir", str(out), "--n_epochs", "1", "--max_steps", "3", "--eval_freq", "2",
          "--save_ckpt_freq", "100", "--print_sample_iter", "100", "--batch_size", "2", "--no_plot",
          "--sample_tokens", "2"], tmp_path)
    sd = torch.load(out / "model_pg_final.pth", weights_only=True)
    assert "trf_blocks.0.att.W_query.lora.A" in sd


def test_cli_sample_mid_epoch_with_workers_gpu(tmp_path):
    """The sample print's HIP-graph decode is captured mid-epoch while DataLoader workers and
    the pin-memory thread are alive (num_workers 2, pin_memory on the GPU): the capture runs in
    thread_local mode so their allocator / event calls cannot invalidate it."""
    out = tmp_path / "ckpt"
    r = _run(["--model", "GPT2", "--num_params", "124M", "--debug", "--data_dir", str(tmp_path / "data"),
              "--synthetic_data", "--output_dir", str(out), "--n_epochs", "1", "--max_steps", "6", "--eval_freq", "3",
              "--save_ckpt_freq", "100", "--print_sample_iter", "2", "--batch_size", "2", "--data_type", "bf16",
              "--num_workers", "2", "--sample_tokens", "8", "--no_plot"], tmp_path)
    text = r.stdout + r.stderr
    assert text.count("Generated Sample:") >= 3, text[-3000:]   # start-up sample + mid-epoch samples
