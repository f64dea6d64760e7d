"""End-to-end CLI runs on CPU (BASELINE config #1 plumbing): ``main.py`` pretraining, LoRA
instruction finetuning, resume, and the self-spawned multi-process path over gloo.
Checks the reference's output contract: model_pg_{step}.pth (incl. step 0), model_pg_final.pth,
losses.pdf, plain prefix-free state dicts."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, tmp_path, timeout=600):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONUNBUFFERED="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, os.path.join(ROOT, "main.py")] + args
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_pretrain_gpt2_debug(tmp_path):
    out = tmp_path / "ckpt"
    _run(["--model", "GPT2", "--num_params", "124M", "--debug", "--data_dir", str(tmp_path / "data"),
          "--synthetic_data", "--output_dir", str(out), "--n_epochs", "1", "--max_steps", "7", "--eval_freq", "2",
          "--save_ckpt_freq", "3", "--print_sample_iter", "3", "--batch_size", "2", "--device", "cpu",
          "--metrics_file", str(tmp_path / "m.jsonl"), "--sample_tokens", "5", "--profile_steps", "2:3"], tmp_path)
    assert (out / "trace_steps2-3_rank0.json").exists()
    for n in ("model_pg_0.pth", "model_pg_3.pth", "model_pg_6.pth", "model_pg_final.pth", "losses.pdf"):
        assert (out / n).exists(), n
    sd = torch.load(out / "model_pg_final.pth", weights_only=True)
    assert "tok_emb.weight" in sd and "blocks.0.att.mask" in sd and not any(k.startswith("module.") for k in sd)
    rows = [json.loads(line) for line in open(tmp_path / "m.jsonl")]
    assert rows and all("train_loss" in r and "lr" in r for r in rows)


def test_finetune_llama_lora_debug(tmp_path):
    out = tmp_path / "ckpt"
    _run(["--model", "llama3_2", "--num_params", "1B", "--debug", "--finetune", "--dataset", "alpaca",
          "--data_dir", str(tmp_path / "alpaca"), "--synthetic_data", "--use_lora", "--lora_rank", "4",
          "--output_dir", str(out), "--n_epochs", "1", "--max_steps", "4", "--eval_freq", "2",
          "--save_ckpt_freq", "100", "--print_sample_iter", "100", "--batch_size", "2", "--device", "cpu",
          "--no_plot", "--sample_tokens", "3"], tmp_path)
    sd = torch.load(out / "model_pg_final.pth", weights_only=True)
    assert "trf_blocks.0.att.W_query.lora.A" in sd and "out_head.lora.B" in sd


@pytest.mark.parametrize("mode", [["--use_fsdp"], ["--use_zero_opt"], []])
def test_multi_process_spawn_gloo(tmp_path, mode):
    """--run_type multi_gpu self-spawns (reference mp.spawn path) — here 2 CPU ranks on gloo."""
    out = tmp_path / "ckpt"
    env_port = str(_free_port())
    os.environ["MASTER_PORT"] = env_port
    try:
        _run(["--model", "llama3_2", "--num_params", "1B", "--debug", "--run_type", "multi_gpu", "--backend", "gloo",
              "--nprocs", "2", "--device", "cpu", "--data_dir", str(tmp_path / "data"), "--synthetic_data",
              "--output_dir", str(out), "--n_epochs", "1", "--max_steps", "3", "--eval_freq", "2",
              "--save_ckpt_freq", "100", "--print_sample_iter", "100", "--batch_size", "2", "--no_plot",
              "--sample_tokens", "2"] + mode, tmp_path)
    finally:
        os.environ.pop("MASTER_PORT", None)
    sd = torch.load(out / "model_pg_final.pth", weights_only=True)
    assert "trf_blocks.0.norm1.weight" in sd and sd["trf_blocks.0.norm1.weight"].dtype == torch.float32


@pytest.mark.parametrize("budget,full", [(None, 0), ("0.000001", 2)])
def test_actv_ckpt_auto_planner(tmp_path, budget, full):
    """``--actv_ckpt_mode auto`` (bench.py's headline policy) through the CLI: the memory planner
    picks per-block modes for this engine and batch; a tiny budget forces every block to full
    recompute.  Runs under FSDP on 2 gloo ranks."""
    out = tmp_path / "ckpt"
    os.environ["MASTER_PORT"] = str(_free_port())
    extra = ["--ckpt_budget_gib", budget] if budget else []
    try:
        r = _run(["--model", "llama3_2", "--num_params", "1B", "--debug", "--run_type", "multi_gpu", "--backend",
                  "gloo", "--nprocs", "2", "--device", "cpu", "--use_fsdp", "--use_actv_ckpt", "--actv_ckpt_mode",
                  "auto", "--data_dir", str(tmp_path / "data"), "--synthetic_data", "--output_dir", str(out),
                  "--n_epochs", "1", "--max_steps", "5", "--eval_freq", "2", "--save_ckpt_freq", "100",
                  "--print_sample_iter", "100", "--batch_size", "2", "--no_plot", "--sample_tokens", "2",
                  "--metrics_file", str(tmp_path / "m.jsonl")] + extra, tmp_path)
    finally:
        os.environ.pop("MASTER_PORT", None)
    log = r.stdout + r.stderr
    assert f"Activation checkpointing (auto): {full} blocks fully recomputed, {2 - full} selective" in log, log[-3000:]
    rows = [json.loads(line) for line in open(tmp_path / "m.jsonl")]
    # throughput is reported from the second eval point on, eval / sample / checkpoint excluded
    assert rows[0]["tokens_per_s"] is None and all(r["tokens_per_s"] > 0 for r in rows[1:])
