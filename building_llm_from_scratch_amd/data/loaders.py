"""Dataloader factories (reference datautils/dataloader.py:9-103 and
dataloader_instruction_finetune.py:53-134).

Semantics kept: raw text split by characters ``train_ratio`` / rest; train loader shuffled
with ``drop_last=True``, val loader in order; multi-GPU uses a ``DistributedSampler`` (which
shuffles, seed 0, pads by repetition) with ``set_epoch`` called by the trainer.
Differences: the instruction pad id defaults to the model's eos id (SURVEY §2.8 defect 7),
and ``get_total_steps_epoch`` reuses cached tokenisation.
"""
from __future__ import annotations

from functools import partial

import torch
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler

from ..utils.misc import read_json_file, read_text_file
from .datasets import DatasetPT, InstructionDataset, custom_collate_fn


def _is_dist() -> bool:
    return torch.distributed.is_available() and torch.distributed.is_initialized()


class DataloaderPT:
    def __init__(self, tokenizer, batch_size, max_length, stride, eos_text="<|endoftext|>",
                 dataset_name="gutenberg", run_type="single_gpu", train_ratio=0.90,
                 collate_func=None, pin_memory=None):
        self.tokenizer = tokenizer
        self.batch_size = batch_size
        self.max_length = max_length
        self.stride = stride
        self.train_ratio = train_ratio
        self.run_type = run_type
        self.collate_func = collate_func
        self.dataset_name = dataset_name
        self.eos_text = eos_text
        self.pin_memory = torch.cuda.is_available() if pin_memory is None else pin_memory
        # allow the model's eos text as a special token (fixes SURVEY §2.8 defect 13)
        self.allowed_special = frozenset({"<|endoftext|>", eos_text})

    def create_dataloader(self, txt, shuffle=True, drop_last=True, num_workers=0):
        if self.dataset_name != "gutenberg":
            raise NotImplementedError(f"Dataset '{self.dataset_name}' not supported.")
        ds = DatasetPT(txt, self.tokenizer, self.max_length, self.stride, self.allowed_special)
        if self.run_type == "multi_gpu" and _is_dist():
            return DataLoader(ds, batch_size=self.batch_size, pin_memory=self.pin_memory,
                              shuffle=False, drop_last=drop_last, sampler=DistributedSampler(ds),
                              collate_fn=self.collate_func)
        return DataLoader(ds, batch_size=self.batch_size, pin_memory=self.pin_memory, shuffle=shuffle,
                          drop_last=drop_last, num_workers=num_workers, collate_fn=self.collate_func,
                          persistent_workers=False)

    def create_dataloaders(self, text_data, num_workers=0):
        split = int(self.train_ratio * len(text_data))
        train = self.create_dataloader(text_data[:split], drop_last=True, shuffle=True, num_workers=num_workers)
        val = self.create_dataloader(text_data[split:], drop_last=False, shuffle=False, num_workers=num_workers)
        return train, val

    def get_total_steps_epoch(self, data_files):
        n = 0
        for fp in data_files:
            text = read_text_file(fp) + " " + self.eos_text + " "
            train, _ = self.create_dataloaders(text, num_workers=0)
            n += len(train)
        return n


class DataloaderIF:
    def __init__(self, tokenizer, batch_size, max_length, dataset_name="alpaca",
                 run_type="single_gpu", train_ratio=0.90, collate_func=None, pad_token_id=50256,
                 pin_memory=None):
        self.tokenizer = tokenizer
        self.batch_size = batch_size
        self.max_length = max_length
        self.train_ratio = train_ratio
        self.run_type = run_type
        self.collate_func = collate_func or partial(custom_collate_fn, pad_token_id=pad_token_id,
                                                    allowed_max_length=max_length)
        self.dataset_name = dataset_name.lower()
        self.pin_memory = torch.cuda.is_available() if pin_memory is None else pin_memory
        if self.dataset_name not in ("alpaca",):
            raise ValueError(f"Dataset '{self.dataset_name}' is not supported.")

    def create_dataloader(self, data, shuffle=True, drop_last=True, num_workers=0):
        ds = InstructionDataset(data, self.tokenizer)
        if self.run_type == "multi_gpu" and _is_dist():
            return DataLoader(ds, batch_size=self.batch_size, pin_memory=self.pin_memory, shuffle=False,
                              drop_last=drop_last, sampler=DistributedSampler(ds), collate_fn=self.collate_func)
        return DataLoader(ds, batch_size=self.batch_size, pin_memory=self.pin_memory, shuffle=shuffle,
                          drop_last=drop_last, num_workers=num_workers, collate_fn=self.collate_func)

    def create_dataloaders(self, data, num_workers=0):
        if not isinstance(data, list):
            raise TypeError("Data must be a list of instruction-format samples.")
        split = int(self.train_ratio * len(data))
        train = self.create_dataloader(data[:split], shuffle=True, drop_last=True, num_workers=num_workers)
        val = self.create_dataloader(data[split:], shuffle=False, drop_last=False, num_workers=num_workers)
        return train, val

    def get_total_steps_epoch(self, data_files):
        n = 0
        for fp in data_files:
            train, _ = self.create_dataloaders(read_json_file(fp), num_workers=0)
            n += len(train)
        return n
