"""Shared utilities (reference utils.py:55-212).

set_seed, token<->text helpers, file readers, parameter / memory accounting, loss plot and
the (offline) Hugging Face login. GPU memory statistics come from the HIP caching
allocator through ``torch.cuda`` (which *is* HIP on ROCm builds).
"""
from __future__ import annotations

import json
import os
import random
from pathlib import Path

import numpy as np
import torch

from ..config import datasize_mapping, datatype_mapping, model_params_mapping  # noqa: F401
from ..logger import setup_logger

logger = setup_logger("utils")


def set_seed(seed: int = 123) -> None:
    """Seed python / numpy / torch RNGs (reference utils.py:55-66)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def text_to_token_ids(text: str, tokenizer, cfg) -> torch.Tensor:
    """reference utils.py:71-77: encode with the eos text allowed, add batch dim."""
    encoded = tokenizer.encode(text, allowed_special={cfg["eos_text"]})
    return torch.tensor(encoded, dtype=torch.long).unsqueeze(0)


def token_ids_to_text(token_ids: torch.Tensor, tokenizer) -> str:
    return tokenizer.decode(token_ids.squeeze(0).tolist())


def read_text_file(file_path) -> str:
    with open(file_path, "r", encoding="utf-8") as f:
        return f.read()


def read_json_file(file_path):
    with open(file_path, "r", encoding="utf-8") as f:
        return json.load(f)


def get_num_params(model: torch.nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


def get_total_size(num_params: int, data_type: str) -> float:
    """Adam "4N" estimate (reference utils.py:112-129)."""
    assert data_type in datasize_mapping, f"Unsupported data type: {data_type}"
    total_gb = 4 * num_params * datasize_mapping[data_type] / 1024 ** 3
    logger.info(f"Estimated model memory size: {total_gb:.2f} GB (excluding activations).")
    return total_gb


def model_memory_size(model: torch.nn.Module, input_dtype: torch.dtype = torch.float32) -> float:
    """params + grads + buffers in ``input_dtype`` (reference utils.py:131-144)."""
    total_params = sum(p.numel() for p in model.parameters())
    total_grads = sum(p.numel() for p in model.parameters() if p.requires_grad)
    total_buffers = sum(b.numel() for b in model.buffers())
    elem = torch.tensor(0, dtype=input_dtype).element_size()
    gb = (total_params + total_grads + total_buffers) * elem / 1024 ** 3
    logger.info(f"Estimated runtime model memory: {gb:.2f} GB (includes grads and buffers).")
    return gb


def start_memory_tracking() -> None:
    if torch.cuda.is_available():
        torch.cuda.reset_peak_memory_stats()


def print_memory_usage() -> float:
    if torch.cuda.is_available():
        gb = torch.cuda.max_memory_allocated() / 1024 ** 3
        logger.info(f"Max GPU memory used: {gb:.2f} GB")
        return gb
    return 0.0


def plot_losses(epochs_seen, tokens_seen, train_losses, val_losses, output_dir) -> None:
    """Loss plot with a tokens-seen secondary x axis -> ``losses.pdf`` (reference utils.py:171-191)."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        from matplotlib.ticker import MaxNLocator
    except Exception as e:  # pragma: no cover - matplotlib is installed in this image
        logger.warning(f"matplotlib unavailable, skipping loss plot: {e}")
        return
    fig, ax1 = plt.subplots()
    ax1.plot(epochs_seen, train_losses, label="Training Loss", color="blue")
    ax1.plot(epochs_seen, val_losses, linestyle="--", label="Validation Loss", color="orange")
    ax1.set_xlabel("Epochs")
    ax1.set_ylabel("Loss")
    ax1.legend(loc="upper right")
    ax1.xaxis.set_major_locator(MaxNLocator(integer=True))
    ax2 = ax1.twiny()
    ax2.plot(tokens_seen, train_losses, alpha=0)
    ax2.set_xlabel("Tokens Seen")
    fig.tight_layout()
    plt.savefig(Path(output_dir) / "losses.pdf")
    plt.close(fig)


def login_hf(config_path: str = "config_hf.json") -> bool:
    """Offline-safe HF login (reference utils.py:196-212). Returns False (and logs) when no
    token or no network is available; never raises."""
    try:
        with open(config_path, "r", encoding="utf-8") as f:
            token = json.load(f).get("HF_ACCESS_TOKEN")
    except FileNotFoundError:
        logger.info(f"'{config_path}' not found; running offline.")
        return False
    if not token or os.environ.get("HF_HUB_OFFLINE", "1") == "1":
        return False
    try:
        from huggingface_hub import login
        login(token=token)
        return True
    except Exception as e:  # no network
        logger.warning(f"Hugging Face login failed ({e}); continuing offline.")
        return False
