"""Pretraining / instruction datasets and collate.

* :class:`DatasetPT` — sliding windows over a token stream (reference datautils/dataset.py:6-40:
  ``range(0, len - max_len, stride)``, input = window, target = window shifted by one).  The
  token stream is held as ONE int32 tensor (windows are views) instead of a Python list of
  per-window tensors, and tokenisation results are cached per text so the step count pass
  (reference dataloader.py:87-103) does not re-tokenise.
* :func:`format_input` / :class:`InstructionDataset` — Alpaca prompt format and
  ``(prompt_len, full_ids)`` items (reference dataset_instruction_finetune.py:6-76).
* :func:`custom_collate_fn` — eos-append, pad, shift, ``-100`` masking of every pad but the
  first and of the prompt (reference dataloader_instruction_finetune.py:10-50).
"""
from __future__ import annotations

import hashlib
import os
import warnings
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

_TOKEN_CACHE: Dict[Tuple[str, int, str], torch.Tensor] = {}


def _tokenizer_tag(tokenizer) -> str:
    return f"{type(tokenizer).__name__}-{getattr(tokenizer, 'n_vocab', getattr(tokenizer, 'vocab_size', 0))}"


def token_cache_path(text: str, tokenizer, allowed_special, cache_dir: str) -> str:
    h = hashlib.sha1(text.encode("utf-8", errors="ignore"))
    h.update(("|" + _tokenizer_tag(tokenizer) + "|" + ",".join(sorted(allowed_special))).encode())
    return os.path.join(cache_dir, h.hexdigest() + ".u32")


def tokenize_cached(text: str, tokenizer, allowed_special=frozenset({"<|endoftext|>"}),
                    cache_dir: Optional[str] = None) -> torch.Tensor:
    """Token ids of ``text`` as one int32 tensor.  With ``cache_dir`` the stream is tokenised
    once into a flat uint32 file (written atomically) and every later call — other ranks,
    later epochs, a resumed run — memory-maps it instead of re-tokenising (reference
    dataset.py:26 re-tokenises every file every epoch, plus once more to count steps)."""
    key = (hashlib.sha1(text.encode("utf-8", errors="ignore")).hexdigest(), id(tokenizer),
           ",".join(sorted(allowed_special)))
    hit = _TOKEN_CACHE.get(key)
    if hit is not None:
        return hit
    path = token_cache_path(text, tokenizer, allowed_special, cache_dir) if cache_dir else None
    if path and os.path.exists(path):
        arr = np.memmap(path, dtype=np.uint32, mode="r")
        with warnings.catch_warnings():       # read-only memmap: windows are only ever read
            warnings.simplefilter("ignore")
            hit = torch.from_numpy(arr.view(np.int32)) if arr.size else torch.zeros(0, dtype=torch.int32)
    else:
        ids = tokenizer.encode(text, allowed_special=set(allowed_special))
        hit = torch.tensor(ids, dtype=torch.int32)
        if path:
            os.makedirs(cache_dir, exist_ok=True)
            tmp = f"{path}.{os.getpid()}.tmp"
            hit.numpy().astype(np.uint32).tofile(tmp)
            os.replace(tmp, path)
    if len(_TOKEN_CACHE) > 64:
        _TOKEN_CACHE.clear()
    _TOKEN_CACHE[key] = hit
    return hit


class DatasetPT(Dataset):
    def __init__(self, txt: str, tokenizer, max_length: int, stride: int,
                 allowed_special=frozenset({"<|endoftext|>"}), token_ids: Optional[torch.Tensor] = None,
                 cache_dir: Optional[str] = None):
        self.max_length = max_length
        self.stride = stride
        self.tokens = token_ids if token_ids is not None else \
            tokenize_cached(txt, tokenizer, allowed_special, cache_dir)
        n = self.tokens.numel()
        self.starts = list(range(0, max(n - max_length, 0), stride))

    def __len__(self):
        return len(self.starts)

    def __getitem__(self, idx):
        s = self.starts[idx]
        w = self.tokens[s:s + self.max_length + 1].long()
        return w[:-1], w[1:]


def format_input(entry: dict) -> str:
    instruction_text = (
        "Below is an instruction that describes a task. "
        "Write a response that appropriately completes the request."
        f"\n\n### Instruction:\n{entry['instruction']}"
    )
    input_text = f"\n\n### Input:\n{entry['input']}" if entry.get("input") else ""
    return instruction_text + input_text


class InstructionDataset(Dataset):
    def __init__(self, data: Sequence[dict], tokenizer):
        self.data = data
        self.encoded_texts: List[List[int]] = []
        self.instruction_lengths: List[int] = []
        for entry in data:
            prompt = format_input(entry)
            full = prompt + f"\n\n### Response:\n{entry['output']}"
            self.encoded_texts.append(tokenizer.encode(full))
            self.instruction_lengths.append(len(tokenizer.encode(prompt)))

    def __getitem__(self, index):
        return self.instruction_lengths[index], self.encoded_texts[index]

    def __len__(self):
        return len(self.data)


def format_input_phi(entry: dict) -> str:
    """Phi-style prompt (reference datautils/dataset_instruction_finetune.py:28-42):
    ``<|user|>\n{instruction}`` plus ``\n{input}`` when there is one."""
    return f"<|user|>\n{entry['instruction']}" + (f"\n{entry['input']}" if entry.get("input") else "")


class InstructionDatasetPhi(Dataset):
    """Phi-format instruction data (reference dataset_instruction_finetune.py:79-99): prompt +
    ``\n<|assistant|>:\n{output}``.  The reference's items are bare token lists, which its own
    collate cannot take (it unpacks (prompt length, ids) pairs); here an item is
    ``(prompt length, ids)`` like ``InstructionDataset``, so ``custom_collate_fn`` masks the prompt."""

    def __init__(self, data: Sequence[dict], tokenizer):
        self.data = data
        self.encoded_texts: List[List[int]] = []
        self.instruction_lengths: List[int] = []
        for entry in data:
            prompt = format_input_phi(entry)
            self.encoded_texts.append(tokenizer.encode(prompt + f"\n<|assistant|>:\n{entry['output']}"))
            self.instruction_lengths.append(len(tokenizer.encode(prompt)))

    def __getitem__(self, index):
        return self.instruction_lengths[index], self.encoded_texts[index]

    def __len__(self):
        return len(self.data)


def custom_collate_fn(batch, pad_token_id: int = 50256, ignore_index: int = -100,
                      allowed_max_length: Optional[int] = None):
    batch_max_length = max(len(item) + 1 for _, item in batch)
    inputs_list, targets_list = [], []
    for instruction_length, item in batch:
        item = list(item) + [pad_token_id]
        padded = item + [pad_token_id] * (batch_max_length - len(item))
        inputs = torch.tensor(padded[:-1], dtype=torch.long)
        targets = torch.tensor(padded[1:], dtype=torch.long)
        pad_pos = torch.nonzero(targets == pad_token_id).flatten()
        if pad_pos.numel() > 1:
            targets[pad_pos[1:]] = ignore_index
        targets[:max(instruction_length - 1, 0)] = ignore_index
        if allowed_max_length is not None:
            inputs = inputs[:allowed_max_length]
            targets = targets[:allowed_max_length]
        inputs_list.append(inputs)
        targets_list.append(targets)
    return torch.stack(inputs_list), torch.stack(targets_list)
