"""Exact token accounting at N > 1 (reference train.py:123 counts
``input_batch.numel()`` per rank).  Instruction batches are padded per rank to that rank's longest
example, so each rank's count differs: the trainer sums every rank's own count (real,
non-ignored targets for instruction data; every position for pretraining) with one all-reduce at
each eval / checkpoint point instead of multiplying this rank's count by the world size."""
import os
from types import SimpleNamespace

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from building_llm_from_scratch_amd.config import get_config
from building_llm_from_scratch_amd.data.datasets import custom_collate_fn
from building_llm_from_scratch_amd.models import build_model
from building_llm_from_scratch_amd.train.optim import FusedAdamW
from building_llm_from_scratch_amd.train.trainer import Trainer


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batches(rank):
    """Alpaca-shaped batches through the reference collate: rank 0's examples are short, rank 1's
    long, so the two ranks' padded lengths and real-target counts differ."""
    g = torch.Generator().manual_seed(11 + rank)
    out = []
    for step in range(3):
        lens = [3 + 2 * rank + step, 5 + 9 * rank, 4 + rank * step]
        batch = [(2, torch.randint(1, 90, (n,), generator=g).tolist()) for n in lens]
        out.append(custom_collate_fn(batch, pad_token_id=96, ignore_index=-100))
    return out


def _worker(rank, world, port, mode, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        cfg = get_config("llama3_2", "1B").replace(context_length=32, emb_dim=32, n_heads=2, n_kv_groups=1,
                                                    hidden_dim=48, n_layers=1, vocab_size=97,
                                                    dtype=torch.float32)
        m = build_model(cfg)
        opt = FusedAdamW(m, lr=1e-3, weight_decay=0.0)
        loader = SimpleNamespace(batch_size=3, tokenizer=None)
        tr = Trainer(m, opt, cfg, [], loader, "/tmp", device="cpu", rank=rank, world_size=world)
        tr.count_target_tokens = mode == "instruction"
        mine = 0
        for inp, tgt in _batches(rank):
            tr.train_batch(inp, tgt)
            mine += int((tgt != -100).sum()) if mode == "instruction" else inp.numel()
        tr._flush_tokens()
        out[rank] = (mine, tr.tokens_seen, int(_batches(rank)[0][0].shape[1]))
    finally:
        dist.destroy_process_group()


def _run(mode):
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.start_processes(_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True, start_method="spawn")
    return dict(out)


def test_world2_instruction_tokens_exact():
    res = _run("instruction")
    (m0, t0, len0), (m1, t1, len1) = res[0], res[1]
    assert len0 != len1, "ranks must pad to different lengths for this test to mean anything"
    assert m0 != m1
    assert t0 == t1 == m0 + m1, res


def test_world2_pretrain_tokens_exact():
    res = _run("pretrain")
    (m0, t0, _), (m1, t1, _) = res[0], res[1]
    assert t0 == t1 == m0 + m1, res


def test_shutdown_loader_stops_persistent_workers():
    """a multi-file run rebuilds each file's loaders per epoch; the finished file's
    persistent workers are shut down at once instead of at garbage collection."""
    from torch.utils.data import DataLoader
    from building_llm_from_scratch_amd.train.trainer import _shutdown_loader
    dl = DataLoader(list(range(32)), batch_size=4, num_workers=2, persistent_workers=True)
    assert sum(1 for _ in dl) == 8
    workers = list(dl._iterator._workers)
    assert workers and all(w.is_alive() for w in workers)
    _shutdown_loader(dl)
    for w in workers:
        w.join(timeout=10)
    assert not any(w.is_alive() for w in workers)
    assert dl._iterator is None


def test_resume_state_records_data_order_version(caplog):
    """the resume state carries the data-order version; a state written by an older
    build (no version) still loads, with a warning that the batch order after it differs."""
    import logging
    from building_llm_from_scratch_amd.train.trainer import Trainer
    cfg = get_config("llama3_2", "1B").replace(context_length=16, emb_dim=32, n_heads=2, n_kv_groups=1,
                                                hidden_dim=48, n_layers=1, vocab_size=97, dtype=torch.float32)
    m = build_model(cfg)
    opt = FusedAdamW(m, lr=1e-3, weight_decay=0.0)
    tr = Trainer(m, opt, cfg, [], SimpleNamespace(batch_size=2, tokenizer=None), "/tmp")
    st = tr.trainer_state()
    assert st["data_order_version"] == Trainer.DATA_ORDER_VERSION
    old = dict(st)
    old.pop("data_order_version")
    tr2 = Trainer(m, opt, cfg, [], SimpleNamespace(batch_size=2, tokenizer=None), "/tmp")
    logging.getLogger("train").propagate = True
    with caplog.at_level(logging.WARNING):
        tr2.load_trainer_state(old)
    assert tr2.pos == tuple(st["pos"])
    assert any("data-order version" in r.getMessage() for r in caplog.records)
