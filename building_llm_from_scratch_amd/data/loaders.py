"""Dataloader factories (reference datautils/dataloader.py:9-103 and
dataloader_instruction_finetune.py:53-134).

Semantics kept: raw text split by characters ``train_ratio`` / rest; train loader shuffled
with ``drop_last=True``, val loader in order on one process; multi-GPU uses a
``DistributedSampler`` for both (which shuffles, seed 0, pads by repetition) with ``set_epoch``
called by the trainer.
Differences: the instruction pad id defaults to the model's eos id (SURVEY §2.8 defect 7),
``get_total_steps_epoch`` reuses cached tokenisation (``cache_dir``: a memory-mapped uint32
token stream per text, written once), worker processes are used under DistributedSampler too,
and the single-process shuffle takes an explicit ``generator`` so a resumed run replays the
same batch order (trainer seeds it per (epoch, file)).
"""
from __future__ import annotations

from functools import partial

import torch
from torch.utils.data import DataLoader, RandomSampler
from torch.utils.data.distributed import DistributedSampler

from ..utils.misc import read_json_file, read_text_file
from .datasets import DatasetPT, InstructionDataset, custom_collate_fn


def _is_dist() -> bool:
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def _make_loader(owner, ds, shuffle, drop_last, num_workers, generator):
    # persistent workers: the trainer re-uses a file's loaders across epochs (reseeding the shuffle
    # generator / set_epoch), so their worker processes are forked once instead of per epoch
    workers = dict(num_workers=num_workers, persistent_workers=num_workers > 0)
    if num_workers > 0:
        workers["prefetch_factor"] = 4
    if owner.run_type == "multi_gpu" and _is_dist():
        # DistributedSampler(shuffle=True, seed=0) + set_epoch: identical order on resume.  The
        # validation loader shuffles too, as the reference's DistributedSampler(dataset) default
        # does (datautils/dataloader.py:50, dataloader_instruction_finetune.py:94): eval_iter
        # batches then come from a seeded random subset, not the leading one
        return DataLoader(ds, batch_size=owner.batch_size, pin_memory=owner.pin_memory, shuffle=False,
                          drop_last=drop_last, sampler=DistributedSampler(ds, shuffle=True),
                          collate_fn=owner.collate_func, **workers)
    # the shuffle draws only from ``generator`` (its own sampler): the DataLoader's worker base
    # seed comes from a separate fixed generator, so a loader re-used with ``generator`` reseeded
    # (persistent workers skip that draw) yields the order a fresh loader with that seed yields
    sampler = RandomSampler(ds, generator=generator) if shuffle else None
    return DataLoader(ds, batch_size=owner.batch_size, pin_memory=owner.pin_memory, sampler=sampler,
                      drop_last=drop_last, collate_fn=owner.collate_func,
                      generator=torch.Generator().manual_seed(0), **workers)


def first_batches(loader, n):
    """The first ``n`` batches ``iter(loader)`` yields, read in this process.

    Evaluation reads ``eval_iter`` (5) batches of each loader every ``eval_freq`` steps.  For a
    loader with worker processes, ``iter(loader)`` forks its workers each time: ~2 s of GPU idle
    per loader per evaluation on an MI355X box under a 240 GiB Llama-3-8B run (rocprofv3 gaps,
    profiles/r5/cli2/gaps.txt).  The batch sampler gives the same batch indices, and five batches
    of memory-mapped windows collate in milliseconds in the main process.
    """
    if n <= 0:
        return
    if getattr(loader, "num_workers", 0) == 0 or getattr(loader, "batch_sampler", None) is None:
        for i, batch in enumerate(loader):
            if i >= n:
                break
            yield batch
        return
    for i, idx in enumerate(loader.batch_sampler):
        if i >= n:
            break
        yield loader.collate_fn([loader.dataset[j] for j in idx])


class DataloaderPT:
    def __init__(self, tokenizer, batch_size, max_length, stride, eos_text="<|endoftext|>",
                 dataset_name="gutenberg", run_type="single_gpu", train_ratio=0.90,
                 collate_func=None, pin_memory=None, cache_dir=None):
        self.tokenizer = tokenizer
        self.batch_size = batch_size
        self.max_length = max_length
        self.stride = stride
        self.cache_dir = cache_dir
        self.train_ratio = train_ratio
        self.run_type = run_type
        self.collate_func = collate_func
        self.dataset_name = dataset_name
        self.eos_text = eos_text
        self.pin_memory = torch.cuda.is_available() if pin_memory is None else pin_memory
        # allow the model's eos text as a special token (fixes SURVEY §2.8 defect 13)
        self.allowed_special = frozenset({"<|endoftext|>", eos_text})

    def create_dataloader(self, txt, shuffle=True, drop_last=True, num_workers=0, generator=None):
        if self.dataset_name != "gutenberg":
            raise NotImplementedError(f"Dataset '{self.dataset_name}' not supported.")
        ds = DatasetPT(txt, self.tokenizer, self.max_length, self.stride, self.allowed_special,
                       cache_dir=self.cache_dir)
        return _make_loader(self, ds, shuffle, drop_last, num_workers, generator)

    def create_dataloaders(self, text_data, num_workers=0, generator=None):
        split = int(self.train_ratio * len(text_data))
        train = self.create_dataloader(text_data[:split], drop_last=True, shuffle=True, num_workers=num_workers,
                                       generator=generator)
        val = self.create_dataloader(text_data[split:], drop_last=False, shuffle=False, num_workers=num_workers)
        return train, val

    def pretokenize(self, data_files):
        """Tokenise every file's train/val split into the memmap cache (call on one rank,
        then barrier: the other ranks map the files instead of re-tokenising)."""
        for fp in data_files:
            text = read_text_file(fp) + " " + self.eos_text + " "
            self.create_dataloaders(text, num_workers=0)

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

    def create_dataloader(self, data, shuffle=True, drop_last=True, num_workers=0, generator=None):
        ds = InstructionDataset(data, self.tokenizer)
        return _make_loader(self, ds, shuffle, drop_last, num_workers, generator)

    def create_dataloaders(self, data, num_workers=0, generator=None):
        if not isinstance(data, list):
            raise TypeError("Data must be a list of instruction-format samples.")
        split = int(self.train_ratio * len(data))
        train = self.create_dataloader(data[:split], shuffle=True, drop_last=True, num_workers=num_workers,
                                       generator=generator)
        val = self.create_dataloader(data[split:], shuffle=False, drop_last=False, num_workers=num_workers)
        return train, val

    def pretokenize(self, data_files):
        pass

    def get_total_steps_epoch(self, data_files):
        n = 0
        for fp in data_files:
            train, _ = self.create_dataloaders(read_json_file(fp), num_workers=0)
            n += len(train)
        return n
