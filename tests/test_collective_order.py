"""Run-time collective-order check (parallel/seqcheck.py): at gloo world 8 the
ranks' warm-up collectives are compared over the rendezvous store, and a rank that issues one
extra collective makes EVERY rank fail within seconds with an error naming that collective --
instead of an RCCL timeout tens of minutes later.  Also: identical orders pass through the
trainer's warm-up steps and bench.py's, and the comparison helper finds the first divergence."""
import os
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from building_llm_from_scratch_amd.parallel.seqcheck import (CollectiveOrderError, CollectiveSequence,
                                                               first_divergence)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, inject_rank, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from building_llm_from_scratch_amd.config import get_config
    from building_llm_from_scratch_amd.models import build_model
    from building_llm_from_scratch_amd.parallel import setup_engine
    from building_llm_from_scratch_amd.train.optim import FusedAdamW
    from building_llm_from_scratch_amd.train.trainer import Trainer
    from types import SimpleNamespace
    torch.manual_seed(0)
    cfg = get_config("llama3_2", "1B").replace(context_length=16, emb_dim=32, n_heads=2, n_kv_groups=1,
                                                hidden_dim=48, n_layers=2, vocab_size=97, dtype=torch.float32)
    m = build_model(cfg)
    eng = setup_engine(m, "fsdp", device="cpu")
    opt = FusedAdamW(m, lr=1e-3, weight_decay=0.0, engine=eng)
    if rank == inject_rank:   # a rank-dependent extra collective inside the optimizer step
        step = opt.step

        def step_plus(*a, **k):
            dist.all_reduce(torch.ones(3), async_op=True)
            return step(*a, **k)
        opt.step = step_plus
    tr = Trainer(m, opt, cfg, [], SimpleNamespace(batch_size=2, tokenizer=None), "/tmp", device="cpu", rank=rank,
                 world_size=world, engine=eng, comm_adapt_steps=1)
    tr._seq_timeout_s = 60.0
    g = torch.Generator().manual_seed(rank)
    t0 = time.time()
    try:
        for _ in range(3):
            x = torch.randint(0, 97, (2, 17), generator=g)
            tr.train_batch(x[:, :-1], x[:, 1:])
        out[rank] = ("ok", time.time() - t0, tr._seq.checks if tr._seq else 0)
    except CollectiveOrderError as e:
        out[rank] = ("error", time.time() - t0, str(e))
    # a pending unmatched gloo collective can block teardown: leave without it
    os._exit(0)


def _run(world, inject_rank):
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.start_processes(_worker, args=(world, _free_port(), inject_rank, out), nprocs=world, join=True,
                       start_method="spawn")
    return dict(out)


def test_world8_extra_collective_named_within_seconds():
    res = _run(8, inject_rank=5)
    assert sorted(res) == list(range(8)), res
    for r, (status, dt, msg) in res.items():
        assert status == "error", (r, status, msg)
        assert dt < 30, (r, dt)                      # seconds, not the PG timeout
        assert "all_reduce(12 B, float32)" in msg, msg   # the injected call, named
        assert "rank 5" in msg and "step0" in msg, msg


def test_world4_identical_orders_pass_warmup():
    res = _run(4, inject_rank=-1)
    for r, (status, dt, checks) in res.items():
        assert status == "ok", (r, checks)
        assert checks == 2, checks                   # steps 0 and 1 (comm_adapt_steps=1) checked


def test_first_divergence_helper():
    a = [{"op": "all_gather", "bytes": 8, "dtype": "bfloat16"}, {"op": "all_reduce", "bytes": 4, "dtype": "float32"}]
    assert first_divergence([a, list(a)]) is None
    assert first_divergence([a, a[:1]]) == 1
    b = [dict(a[0], bytes=16), a[1]]
    assert first_divergence([a, b, a]) == 0


def test_disabled_without_process_group():
    seq = CollectiveSequence()
    assert not seq.enabled
    with seq.recording("x"):
        pass
    assert seq.verify("x") == 0


def test_rccl_topology_parser(tmp_path):
    """bench.py's ``rccl_topology``: RCCL's INIT/GRAPH log lines -> ranks, channel counts, ring /
    tree examples and the algorithm-related lines."""
    from building_llm_from_scratch_amd.utils.telemetry import rccl_topology
    log = tmp_path / "r0.log"
    log.write_text("h:1:1 [0] NCCL INFO comm 0x1 rank 0 nRanks 8 nNodes 1 localRanks 8 localRank 0 MNNVL 0\n"
                   "h [0] NCCL INFO Channel 00/16 : 0 1 2 3 4 5 6 7\n"
                   "h [0] NCCL INFO Channel 01/16 : 0 2 4 6 1 3 5 7\n"
                   "h [0] NCCL INFO Tree 0 : -1 -> 0 -> 1/-1/-1\n"
                   "h [0] NCCL INFO 16 coll channels, 16 collnet channels, 0 nvls channels, 16 p2p channels, "
                   "2 p2p channels per peer\n"
                   "h [0] NCCL INFO Connected all rings\n"
                   "unrelated line\n")
    t = rccl_topology(str(log))
    assert t["n_ranks"] == 8 and t["local_ranks"] == 8 and t["channels"] == 16
    assert t["coll_channels"] == 16 and t["p2p_channels"] == 16 and t["trees"] == 1
    assert len(t["rings"]) == 2 and t["decisions"] == ["Connected all rings"]
    assert rccl_topology(str(tmp_path / "missing.log")) is None
