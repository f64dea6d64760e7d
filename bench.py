#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): whole-node training tokens/s, Llama-3-8B bf16 FSDP
full-shard + activation checkpointing, at 1/2/4/8 MI355X.

    python bench.py --gpus N --steps K --warmup W          # N > 1: bench.py spawns N ranks itself
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Launch: under torchrun (RANK / WORLD_SIZE in the environment) each process is one rank.  Without
it, ``--gpus N > 1`` starts N worker processes itself with torch.multiprocessing spawn, as the
reference's ``mp.spawn(main, nprocs=torch.cuda.device_count())`` (main.py:185-191) — before
anything in the parent touches the GPU (only ``torch.cuda.device_count()``, which does not
initialise HIP, and no exec); rank 0 prints the one JSON line.

Every run — N=1 included — initialises a process group (RCCL; gloo with ``--device cpu``) and
trains through the SAME ``FSDPEngine`` (parallel/fsdp.py).  At N=1 that engine behaves like
torch FSDP at world size 1, which clamps FULL_SHARD to NO_SHARD (torch/distributed/fsdp/
_init_utils.py:426-437): the single rank's shard is the whole flat, so no collective runs.

One step = forward, fused CE, backward (with activation checkpointing), global-norm clip 1.0
(one scalar all-reduce) and AdamW(wd 0.1) with fp32 master weights on this rank's shard, on
random-init weights of the full architecture and synthetic token ids.  W untimed warm-up
steps, then exactly K timed steps bracketed by barrier + device sync; the slowest rank's time
is reported (every rank's time and peak memory are in the JSON).  Weak scaling: the per-GPU
micro-batch is fixed, total tokens grow with N.

Activation checkpointing (headline default ``--actv_ckpt auto``): the granularity is chosen per
N from the 288 GB budget by train/memplan.py — every block ``selective`` (norm outputs and the
SwiGLU activation recomputed inside passes the backward runs anyway), plus the fewest fully
recomputed blocks that keep the predicted per-rank peak under ``--ckpt_budget_gib`` (250); the
first warm-up step measures the real peak and re-plans if it is over.  FSDP sharding at N > 1
frees the fp32 master / moments, so the plan can only get lighter with N.  ``--actv_ckpt
full`` is the reference's ``--use_actv_ckpt`` exactly (``checkpoint_sequential(segments=
n_layers)``, Llama3.py:198-199: 31 of 32 blocks re-run in backward); the JSON states which.

Micro-batch: the reference's ``--batch_size`` default 4 (args.py:53) was sized for a 16 GB T4;
one MI355X holds 288 GB, so each rank runs 40 x 1024 tokens (``--batch_size 4`` reproduces the
reference default).

``mfu`` counts model FLOPs only (6·N_nonemb + 12·L·d·T per token, no recompute); ``hfu`` adds
what the hardware also executes under full checkpointing: each block's forward re-run minus its
last projection, which the recompute skips (config.recompute_flops_per_token).  Peak is 2.5 PF
dense bf16.

Other BASELINE configs (``--preset``; each prints one JSON line of its own):
  gpt2_774m_ddp          #2  GPT2-774M pretrain, DDP, bf16, dropout 0.1
  llama32_1b_lora_alpaca #4  Llama-3.2-1B Alpaca instruction finetune, LoRA r=16 a=32: variable
                             length batches through the reference collate (pad to batch max,
                             -100 masking) from synthetic Alpaca-shaped records, DataLoader in
                             the timed loop; tokens counted like the reference's tokens_seen
                             (padded B x T)
  llama2_7b_fsdp_mp      #5  Llama-2-7B pretrain, FSDP full shard (params, grads AND optimizer
                             state sharded = ZeRO-3, a superset of the ZeRO optimizer) +
                             ``--mixed_precision bf16`` policy
``--device cpu`` runs a tiny config of the same model family on gloo (multi-process plumbing
check only; never a headline number).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import timedelta

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TOKENS_PER_S = None  # the reference publishes no number
METRIC = "tokens/sec (whole node) Llama-3-8B bf16 FSDP at 1/2/4/8 MI355X"
PEAK_BF16 = 2.5e15

# Micro-batches per GPU chosen by same-box sweeps against the 288 GB budget (profiles/r3/):
# LoRA 24 -> 96 tokens/s +26 % at 56.7 GiB (variable-length Alpaca rows: the low-rank kernels and
# the frozen GEMMs need the larger M); Llama-3-8B's 40 is the planner-checked headline batch.
PRESETS = {
    "llama3_8b_fsdp": dict(model="llama3", num_params="8B", parallel="fsdp", actv_ckpt="auto", batch_size=40,
                           data="pretrain", mixed_precision=None, lora_rank=0,
                           tunableop="configs/tunableop_llama3_8b_b40_mi355x.csv"),
    "gpt2_774m_ddp": dict(model="GPT2", num_params="774M", parallel="ddp", actv_ckpt="none", batch_size=64,
                          data="pretrain", mixed_precision=None, lora_rank=0,
                          tunableop="configs/tunableop_gpt2_774m_b64_mi355x.csv"),
    "llama32_1b_lora_alpaca": dict(model="llama3_2", num_params="1B", parallel="ddp", actv_ckpt="none",
                                   batch_size=96, data="alpaca", mixed_precision=None, lora_rank=16),
    "llama2_7b_fsdp_mp": dict(model="llama2", num_params="7B", parallel="fsdp", actv_ckpt="none", batch_size=24,
                              data="pretrain", mixed_precision="bf16", lora_rank=0),
}
NICE = {"llama3": "Llama-3-8B", "GPT2": "GPT2-774M", "llama3_2": "Llama-3.2-1B", "llama2": "Llama-2-7B"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--preset", default="llama3_8b_fsdp", choices=sorted(PRESETS))
    ap.add_argument("--model", default=None)
    ap.add_argument("--num_params", default=None)
    ap.add_argument("--batch_size", type=int, default=None, help="micro-batch per GPU (reference CLI default: 4)")
    ap.add_argument("--seq_len", type=int, default=1024)
    ap.add_argument("--actv_ckpt", default=None, choices=["none", "selective", "full", "auto"],
                    help="auto = granularity from the HBM budget (headline); full = reference "
                         "checkpoint_sequential semantics; selective recomputes norms + SwiGLU/GELU act")
    ap.add_argument("--ckpt_segments", type=int, default=None,
                    help="full mode: checkpoint_sequential segments (default n_layers = the reference's "
                         "--use_actv_ckpt; fewer segments recompute fewer blocks)")
    ap.add_argument("--ckpt_budget_gib", type=float, default=None,
                    help="auto mode: per-rank peak-memory ceiling (default 250 GiB, capped at device - 18 GiB)")
    ap.add_argument("--parallel", default=None, choices=["fsdp", "ddp", "zero1"])
    ap.add_argument("--mixed_precision", default=None, choices=["bf16", "fp16", "bf16_hybrid", "fp32"])
    ap.add_argument("--lora_rank", type=int, default=None)
    ap.add_argument("--lora_alpha", type=int, default=32)
    ap.add_argument("--reshard_after_forward", type=int, default=1)
    ap.add_argument("--bucket_mb", type=float, default=256.0,
                    help="DDP / ZeRO-1 gradient bucket size (MiB); DDP grows it in warm-up while its "
                         "all-reduce wait shows in the step")
    ap.add_argument("--fsdp_prefetch", type=int, default=0,
                    help="FSDP units all-gathered ahead (0 = auto: gather time over xGMI vs unit compute)")
    ap.add_argument("--layers", type=int, default=None, help="(debug only) override n_layers; invalidates the metric")
    ap.add_argument("--profile", action="store_true", help="print a per-phase timing breakdown to stderr")
    ap.add_argument("--gemm_epilogues", nargs="?", const="swiglu,rope,gelu", default="",
                    help="gate/up + SwiGLU, QKV + RoPE, c_fc + bias + GELU on csrc/gemm_nt.hip's fused-epilogue "
                         "kernel instead of the library GEMM + a separate pass (measured slower, A/B); "
                         "bare flag = all three, or a comma list of swiglu,rope,gelu")
    ap.add_argument("--overlap_optimizer", action="store_true",
                    help="run AdamW on a side HIP stream under the next forward")
    ap.add_argument("--data", default=None, choices=["pretrain", "random_ids", "fixed_ids", "alpaca"],
                    help="pretrain (default for pretraining presets): synthetic Gutenberg text -> offline "
                         "tokenizer -> memmap cache -> DataloaderPT windows (DistributedSampler at N>1), the "
                         "reference's data path; random_ids: device-resident random token ids (A/B only); "
                         "fixed_ids: one seeded GLOBAL batch per step, rank r trains rows [rB, (r+1)B), and "
                         "the JSON gets the per-step loss trace, so a world-N run can be compared with world 1 "
                         "at N x B (rehearsal check, not a measurement)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: tiny config on gloo (distributed plumbing check, not a measurement)")
    ap.add_argument("--pg_timeout_min", type=float, default=20.0)
    ap.add_argument("--one_device", action="store_true",
                    help="(rehearsal only) every rank on cuda:0 over gloo (RCCL refuses two ranks on one "
                         "GPU): the world-N sharded path on a one-GPU box; invalidates the metric")
    ap.add_argument("--force_comm", action="store_true",
                    help="world 1: run the engines' N>1 collective path (RCCL copies) instead of the "
                         "world-1 shortcut (BLLM_FORCE_COMM=1) — a one-GPU rehearsal of the multi-GPU path")
    ap.add_argument("--tunableop_tune", default=None,
                    help="tune every hipBLASLt/rocBLAS GEMM shape this run meets with PyTorch TunableOp and write "
                         "the results CSV here (a tuning run, not a measurement)")
    ap.add_argument("--tunableop", default=None,
                    help="PyTorch TunableOp results CSV (every hipBLASLt + rocBLAS solution timed per GEMM "
                         "shape); the headline and GPT-2 presets use configs/tunableop_*_mi355x.csv (+0.35 %% / "
                         "+1.25 %% same box, profiles/r4/tunableop_default/, profiles/r4/tunableop_gpt2/); "
                         "read-only: shapes not in the file, "
                         "or a file whose library versions do not match, keep hipBLASLt's heuristic; 'none' = off")
    a = ap.parse_args(argv)
    for k, v in PRESETS[a.preset].items():
        if getattr(a, k, None) is None:
            setattr(a, k, v)
    return a


def init_dist(a):
    """Process group for every N (world 1 included) with a collective timeout, so a wedged
    collective raises instead of hanging the node."""
    import torch
    import torch.distributed as dist
    launched = "WORLD_SIZE" in os.environ and "RANK" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    if a.device == "cuda":
        local = 0 if a.one_device else local
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    kw = dict(timeout=timedelta(minutes=a.pg_timeout_min))
    rccl = dev.type == "cuda" and not a.one_device
    # per-collective start / end events on RCCL's stream (Work._get_duration: the bandwidth
    # account of parallel/commstats.py); read by ProcessGroupNCCL at construction
    os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")
    a.rccl_log = None
    if rccl:
        from building_llm_from_scratch_amd.parallel import nccl_pg_options
        if world > 1 or a.force_comm:   # RCCL's channel / algorithm choices -> "rccl_topology"
            from building_llm_from_scratch_amd.utils.telemetry import rccl_debug_env
            a.rccl_log = rccl_debug_env(rank)
        kw["device_id"] = dev
        kw["pg_options"] = nccl_pg_options(kw["timeout"])
    backend = "nccl" if rccl else "gloo"
    if launched:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend, **kw)
    else:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, **kw)
    return dist, dev, world, rank


def build_config(a, dev):
    import torch
    from building_llm_from_scratch_amd.config import get_config
    from building_llm_from_scratch_amd.parallel.mixed_precision import get_policy
    cfg = get_config(a.model, a.num_params, context_length=a.seq_len)
    dtype = get_policy(a.mixed_precision).param_dtype if a.mixed_precision else torch.bfloat16
    if dev.type == "cpu":  # plumbing-size model, fp32 (the CPU path has no bf16 kernels)
        a.seq_len = min(a.seq_len, 32)
        a.batch_size = min(a.batch_size, 2)
        cfg = cfg.replace(n_layers=2, emb_dim=64, n_heads=4, n_kv_groups=2 if cfg.is_llama else 4, hidden_dim=128,
                          vocab_size=512, context_length=a.seq_len)
        dtype = torch.float32
    cfg = cfg.replace(dtype=dtype)
    if a.layers:
        cfg = cfg.replace(n_layers=a.layers)
    return cfg


def alpaca_loader(a, cfg, rank, world):
    """Synthetic Alpaca records -> InstructionDataset -> reference collate (variable T)."""
    from functools import partial

    import torch
    from torch.utils.data import DataLoader

    from building_llm_from_scratch_amd.data.datasets import InstructionDataset, custom_collate_fn
    from building_llm_from_scratch_amd.data.synthetic import alpaca_records
    from building_llm_from_scratch_amd.data.tokenizer import build_tokenizer
    tok = build_tokenizer(a.model, cfg, None)
    recs = alpaca_records(4096, seed=123)[rank::world]
    ds = InstructionDataset(recs, tok)
    collate = partial(custom_collate_fn, pad_token_id=cfg.eos_id, allowed_max_length=cfg.context_length)
    g = torch.Generator().manual_seed(1000 + rank)
    dl = DataLoader(ds, batch_size=a.batch_size, shuffle=True, drop_last=True, collate_fn=collate,
                    num_workers=2, pin_memory=torch.cuda.is_available(), generator=g, persistent_workers=True)

    def forever():
        while True:
            yield from dl
    return forever()


def pretrain_loader(a, cfg, dist, rank, world):
    """The reference's pretraining data path (train.py:162-172, datautils/dataloader.py:42-62):
    synthetic Gutenberg-shaped text (data/synthetic.py, ``combined_1.txt`` format) + " <eos> ",
    tokenised ONCE into the uint32 memmap cache by rank 0 before the timer (the other ranks map
    it), split 90/10 by characters, DatasetPT windows with stride = context, and a
    DistributedSampler over the N ranks (set_epoch per pass).  Returns (batch iterator,
    description, sampler-order function for the disjointness check)."""
    import tempfile

    from building_llm_from_scratch_amd.data.loaders import DataloaderPT
    from building_llm_from_scratch_amd.data.synthetic import make_gutenberg_corpus
    from building_llm_from_scratch_amd.data.tokenizer import build_tokenizer
    from building_llm_from_scratch_amd.utils.misc import read_text_file
    B, T = a.batch_size, a.seq_len
    # enough text for every timed + warm-up window of every rank (byte tokenizer: ~1 token per
    # character; BPE would give fewer tokens and the sampler simply starts another epoch)
    need = (a.warmup + a.steps + 4) * B * (T + 1) * world / 0.9
    mb = round(min(256.0, max(0.5, need / 2 ** 20 * 1.05)), 2)
    root = os.path.join(tempfile.gettempdir(), f"bllm_bench_gutenberg_{os.getuid()}_{mb}mb")
    path = os.path.join(root, "combined_1.txt")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if local == 0 and not os.path.exists(path):
        tmp = f"{root}.{os.getpid()}.tmp"
        make_gutenberg_corpus(tmp, n_files=1, mb_per_file=mb, seed=123)
        os.makedirs(root, exist_ok=True)
        os.replace(os.path.join(tmp, "combined_1.txt"), path)
        os.rmdir(tmp)
    dist.barrier()
    tok = build_tokenizer(a.model, cfg, None)
    ldr = DataloaderPT(tok, batch_size=B, max_length=T, stride=T, eos_text=cfg.eos_text,
                       run_type="multi_gpu" if world > 1 else "single_gpu", cache_dir=os.path.join(root, "tokens"))
    text = read_text_file(path) + " " + cfg.eos_text + " "
    if rank == 0:
        ldr.create_dataloaders(text, num_workers=0)      # fills the memmap cache
    dist.barrier()
    train, _ = ldr.create_dataloaders(text, num_workers=0, generator=torch_gen(1000 + rank))
    n_tok = train.dataset.tokens.numel()

    def forever():
        ep = 0
        while True:
            if hasattr(train.sampler, "set_epoch"):
                train.sampler.set_epoch(ep)
            yield from train
            ep += 1

    def order(epoch=0):   # window indices this rank consumes in ``epoch``, in order
        if hasattr(train.sampler, "set_epoch"):
            train.sampler.set_epoch(epoch)
        return list(iter(train.sampler))
    desc = (f"synthetic Gutenberg-shaped text ({mb} MB, data/synthetic.py) -> {type(tok).__name__} "
            f"({n_tok} train tokens, memmap cache) -> DataloaderPT windows (stride {T}) -> "
            + ("DistributedSampler over %d ranks" % world if world > 1 else "shuffled sampler (1 rank)"))
    return forever(), desc, order, len(train.dataset)


def torch_gen(seed):
    import torch
    g = torch.Generator()
    g.manual_seed(seed)
    return g


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn_worker(local_rank: int, argv, world: int, port: int):
    """One rank of a self-launched run (the parent did not touch the GPU)."""
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      BLLM_BENCH_LAUNCHER="spawn")
    main(argv)


def launch(argv=None):
    """Entry point: run in-process (N = 1, or one rank under torchrun) or spawn N ranks."""
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import torch
        import torch.multiprocessing as mp
        if a.device == "cuda" and not a.one_device:
            n = torch.cuda.device_count()   # counts devices without initialising HIP in this process
            if n < a.gpus:
                raise SystemExit(f"bench.py: --gpus {a.gpus} but only {n} GPU(s) visible")
        mp.start_processes(_spawn_worker, args=(argv, a.gpus, _free_port()), nprocs=a.gpus, join=True,
                           start_method="spawn")
        return
    main(argv)


def main(argv=None):
    a = parse(argv)
    if a.tunableop_tune:
        # a tuning run writes its own file; a preset's read-only table would switch tuning off
        a.tunableop = None
        os.environ.update(PYTORCH_TUNABLEOP_ENABLED="1", PYTORCH_TUNABLEOP_TUNING="1",
                          PYTORCH_TUNABLEOP_FILENAME=os.path.abspath(a.tunableop_tune).replace(".csv", "%d.csv"))
    from building_llm_from_scratch_amd.utils.gemm_tuning import install_table, resolve_table
    a.tunableop = resolve_table(a.tunableop) if a.device == "cuda" else None
    # must be set before the first GEMM
    install_table(a.tunableop, int(os.environ.get("LOCAL_RANK", "0")))
    import torch
    from building_llm_from_scratch_amd import ops
    from building_llm_from_scratch_amd.models import build_model, replace_linear_with_lora
    from building_llm_from_scratch_amd.parallel import setup_engine
    from building_llm_from_scratch_amd.parallel.mixed_precision import get_policy
    from building_llm_from_scratch_amd.train.optim import FusedAdamW

    if a.force_comm:
        os.environ["BLLM_FORCE_COMM"] = "1"
    dist, dev, world, rank = init_dist(a)
    cuda = dev.type == "cuda"
    rccl_on = cuda and not a.one_device and (world > 1 or a.force_comm)
    if cuda:
        ops.load_ext(required=True)
    sync = torch.cuda.synchronize if cuda else (lambda: None)

    cfg = build_config(a, dev)
    if a.gemm_epilogues:
        from building_llm_from_scratch_amd.models.linear import use_gemm_epilogues
        use_gemm_epilogues([e for e in a.gemm_epilogues.split(",") if e])
    torch.manual_seed(123)
    plan = None
    ckpt_mode = "selective" if a.actv_ckpt == "auto" else a.actv_ckpt
    # built on the meta device: every engine initialises the weights unit by unit on this rank's
    # device under per-unit seeds (models/base.py:init_unit_), so no rank materialises the whole
    # model and nothing is broadcast (FSDP keeps only its shard of each unit)
    model = build_model(cfg, use_actv_ckpt=ckpt_mode, device="meta")
    if a.ckpt_segments:
        model.set_actv_ckpt(a.actv_ckpt, a.ckpt_segments)
    B, T = a.batch_size, a.seq_len
    if a.actv_ckpt == "auto":
        from building_llm_from_scratch_amd.train import memplan
        total = torch.cuda.get_device_properties(dev).total_memory if cuda else None
        budget = a.ckpt_budget_gib * memplan.GIB if a.ckpt_budget_gib else None
        plan = memplan.plan_ckpt(cfg, B, T, world=world, engine=a.parallel, budget=budget, device_total=total,
                                 elt=torch.empty((), dtype=cfg.dtype).element_size(), prefetch=max(1, a.fsdp_prefetch or 2))
        model.set_block_modes(plan.modes)
    if a.lora_rank:
        for p in model.parameters():
            p.requires_grad = False
        replace_linear_with_lora(model, rank=a.lora_rank, alpha=a.lora_alpha)
    reduce = get_policy(a.mixed_precision).reduce_dtype if a.mixed_precision else None
    engine = setup_engine(model, a.parallel, device=dev, reduce_dtype=reduce, bucket_mb=a.bucket_mb,
                          reshard_after_forward=bool(a.reshard_after_forward), prefetch=a.fsdp_prefetch)
    opt = FusedAdamW(model, lr=3e-4, weight_decay=0.1, engine=engine, overlap=a.overlap_optimizer)

    data_desc, sampler_order, n_windows = None, None, None
    if a.data == "alpaca":
        batches = alpaca_loader(a, cfg, rank, world)

        def next_batch(i):
            x, y = next(batches)
            return x.to(dev, non_blocking=True), y.to(dev, non_blocking=True)
    elif a.data == "pretrain":
        batches, data_desc, sampler_order, n_windows = pretrain_loader(a, cfg, dist, rank, world)

        def next_batch(i):
            x, y = next(batches)
            return x.to(dev, non_blocking=True), y.to(dev, non_blocking=True)
    elif a.data == "fixed_ids":
        g = torch.Generator(device=dev)
        g.manual_seed(1000)
        data = [torch.randint(0, cfg.vocab_size, (world * B, T + 1), device=dev, generator=g)[rank * B:(rank + 1) * B]
                for _ in range(4)]

        def next_batch(i):
            b = data[i % len(data)]
            return b[:, :-1], b[:, 1:]
    else:
        g = torch.Generator(device=dev)
        g.manual_seed(1000 + rank)
        data = [torch.randint(0, cfg.vocab_size, (B, T + 1), device=dev, generator=g) for _ in range(4)]

        def next_batch(i):
            b = data[i % len(data)]
            return b[:, :-1], b[:, 1:]

    tokens = 0
    loss_trace = [] if a.data == "fixed_ids" else None

    def step(i):
        nonlocal tokens
        x, y = next_batch(i)
        opt.zero_grad()
        loss = model(x, y)
        loss.backward()
        opt.clip_grad_norm_(1.0)
        opt.step()
        tokens += x.numel()
        if loss_trace is not None:   # mean over ranks == the world-1 loss of the whole global batch
            lt = loss.detach().float().reshape(1)
            dist.all_reduce(lt)
            loss_trace.append(lt.item() / world)
        return loss

    probe_peak = None
    comm = getattr(engine, "comm", None)
    adapt_hist = []
    reprobe = False

    def reprobe_plan(prev):
        """The last step's measured peak (max over ranks) against the checkpoint plan; adds fully
        recomputed blocks if it was over budget.  Returns the peak."""
        nonlocal plan
        sync()
        pk = torch.tensor([float(torch.cuda.max_memory_allocated(dev))], device=dev)
        dist.all_reduce(pk, op=dist.ReduceOp.MAX)
        new = memplan.replan_after_probe(plan, cfg, B, T, pk.item(),
                                         elt=torch.empty((), dtype=cfg.dtype).element_size())
        if new is not plan:
            plan = new
            model.set_block_modes(plan.modes)
            torch.cuda.reset_peak_memory_stats(dev)
        return pk.item() if prev is None else max(prev, pk.item())
    # every warm-up step's collectives (op, bytes, dtype) compared across ranks over the
    # rendezvous store right after the step is issued, before anything waits on them: a divergent
    # order raises naming the first differing call instead of hanging until the PG timeout
    from building_llm_from_scratch_amd.parallel.seqcheck import CollectiveSequence
    seq = CollectiveSequence(enabled=world > 1 or a.force_comm)
    seq_checked = 0
    for i in range(a.warmup):
        if comm is not None:
            comm.reset(enabled=True)      # this warm-up step's exposed waits (adaptation input)
        sync()
        tw = time.perf_counter()
        with seq.recording(f"warmup{i}"):
            loss = step(i)
        seq_checked += seq.verify(f"warmup{i}")
        if i == 0 and plan is not None and cuda:
            # memory probe: the first step's measured peak (max over ranks) checks the plan
            probe_peak = reprobe_plan(probe_peak)
        # warm-up adaptation (after the cold first step): FSDP prefetch depth / DDP bucket
        # size grown while a collective wait shows in the step (MAX over ranks, parallel/)
        if i >= 1 and hasattr(engine, "adapt"):
            sync()
            if reprobe:   # the step after a prefetch change: its peak checks the plan again
                probe_peak = reprobe_plan(probe_peak)
                reprobe = False
            rec = engine.adapt(1e3 * (time.perf_counter() - tw))
            if rec is not None:
                adapt_hist.append(rec)
                if plan is not None and cuda and any(k.endswith("_new") for k in rec):
                    torch.cuda.reset_peak_memory_stats(dev)
                    reprobe = True
    sync()
    dist.barrier()
    sync()
    if comm is not None:
        comm.reset(enabled=True)     # exposed collective waits of the timed steps only
    tokens = 0
    from building_llm_from_scratch_amd.utils.telemetry import GpuTelemetry, library_versions, tunableop_status
    telem = GpuTelemetry(int(os.environ.get("LOCAL_RANK", "0"))) if cuda else None
    if telem is not None:
        telem.start()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(a.warmup + i)
    sync()
    dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    telemetry = telem.stop() if telem is not None else {"source": None, "samples": 0}
    comm_by_kind = comm.summary() if comm is not None else {}
    comm_bw = comm.bandwidth() if comm is not None else {}
    if comm is not None:
        comm.enabled = False
    comm_ms = sum(v["ms"] for v in comm_by_kind.values()) / a.steps
    peak = float(torch.cuda.max_memory_allocated(dev)) if cuda else 0.0
    # every rank's (time, tokens, peak, exposed comm ms/step): rank 0 reports the max time, the
    # token sum and the spread
    mine = torch.tensor([elapsed, float(tokens), peak, comm_ms], device=dev, dtype=torch.float64)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    per_rank = torch.stack(allr).cpu().tolist()
    elapsed = max(r[0] for r in per_rank)
    total_tokens = sum(r[1] for r in per_rank)
    tps = total_tokens / elapsed
    ms = 1000 * elapsed / a.steps
    n_ckpt = sum(model.rctx.block_mode(i) == "full" for i in range(cfg.n_layers))
    T_eff = total_tokens / (world * a.steps * B)           # mean padded length (alpaca); == T otherwise
    flops_tok = cfg.train_flops_per_token(int(round(T_eff)))
    if a.lora_rank:  # frozen base: no weight-gradient GEMMs (2 of the 6 N FLOPs per param)
        flops_tok -= 2.0 * (cfg.num_params() - cfg.vocab_size * cfg.emb_dim)
    mfu = tps / world * flops_tok / PEAK_BF16
    # recomputed blocks only (checkpoint_sequential leaves the last segment un-checkpointed)
    extra = cfg.recompute_flops_per_token(int(round(T_eff))) * n_ckpt / cfg.n_layers
    recompute = (flops_tok + extra) / flops_tok
    # data sharding check: the windows each rank consumed in the first pass of the sampler
    data_check = None
    if sampler_order is not None:
        per = a.batch_size * (a.warmup + a.steps)
        mine_w = sampler_order(0)[:per]
        allw = [None] * world
        dist.all_gather_object(allw, mine_w)
        sets = [set(w) for w in allw]
        union = set().union(*sets)
        data_check = {"sampler": "DistributedSampler" if world > 1 else "RandomSampler",
                      "windows": n_windows, "windows_per_rank_used": len(mine_w),
                      "disjoint_across_ranks": len(union) == sum(len(x) for x in sets)
                      or per * world > n_windows}
    comm_kinds = [None] * world
    dist.all_gather_object(comm_kinds, comm_by_kind)
    telem_all = [None] * world
    dist.all_gather_object(telem_all, telemetry)
    # the adapted comm parameters of every rank (must agree: they fix the collective order)
    knobs_all = [None] * world
    dist.all_gather_object(knobs_all, (getattr(engine, "prefetch", None), getattr(engine, "bucket_mb", None)))
    prof = profile_phases(model, opt, next_batch, dev) if (a.profile and rank == 0 and cuda) else None
    if rank == 0:
        headline = a.preset == "llama3_8b_fsdp" and cuda and not a.layers and not a.one_device
        name = NICE.get(a.model, f"{cfg.name}-{cfg.size}")
        if cuda:
            dtype = "bf16" if cfg.dtype == torch.bfloat16 else str(cfg.dtype).replace("torch.", "")
        else:
            dtype = "fp32"
        metric = METRIC if headline else (
            f"tokens/sec (whole node) {name} {dtype} {a.parallel.upper()}"
            + (f" LoRA r={a.lora_rank} Alpaca finetune" if a.lora_rank else "")
            + (f" mixed_precision={a.mixed_precision}" if a.mixed_precision else "")
            + (" [cpu plumbing, tiny config]" if not cuda else ""))
        summ = model.ckpt_summary()
        if a.actv_ckpt == "auto":
            ckpt_desc = (f"{summ['full']}/{cfg.n_layers} fully recomputed, {summ['selective']} selective "
                         "(auto: memory planner)")
        elif a.actv_ckpt == "full":
            ckpt_desc = f"{n_ckpt}/{cfg.n_layers} recomputed" + (
                f" (checkpoint_sequential segments={a.ckpt_segments})" if a.ckpt_segments
                else " (checkpoint_sequential segments=n_layers, as the reference)")
        else:
            ckpt_desc = f"{n_ckpt}/{cfg.n_layers} recomputed ({a.actv_ckpt})"
        gib = lambda v: round(v / 2 ** 30, 1)  # noqa: E731
        out = {
            "metric": metric,
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (tps / BASELINE_TOKENS_PER_S) if BASELINE_TOKENS_PER_S else None,
            "dtype": dtype,
            "data": ("synthetic Alpaca-shaped records, offline byte tokenizer, reference collate (variable T)"
                     if a.data == "alpaca" else (data_desc if a.data == "pretrain"
                                                 else "synthetic random token ids (Gutenberg-pretraining shape)"))
                    + ", random-init weights (seeded per unit, meta-built)",
            "config": {
                "model": name + (f" ({cfg.n_layers} layers, INVALID)" if a.layers else "")
                + (" (all ranks on one GPU over gloo, INVALID)" if a.one_device else "")
                + ("" if cuda else " (tiny cpu config, INVALID as a measurement)"),
                "global_batch": world * B,
                "micro_batch_per_gpu": B,
                "seq_len": T if a.data != "alpaca" else f"variable (mean {T_eff:.0f}, max {cfg.context_length})",
                "parallelism": f"{a.parallel}{world}",
                "engine": type(engine).__name__ + (" (world 1: no-shard)" if getattr(engine, "no_shard", False)
                                                   else (" (world 1: forced collective path)"
                                                         if world == 1 and a.force_comm else "")),
                "actv_ckpt": a.actv_ckpt,
                "ckpt_blocks": ckpt_desc,
                "mixed_precision": a.mixed_precision,
                "lora": {"rank": a.lora_rank, "alpha": a.lora_alpha} if a.lora_rank else None,
                "optimizer": "AdamW fp32 master, wd 0.1, clip 1.0",
                "gemm_tuning": (os.path.relpath(a.tunableop, os.path.dirname(os.path.abspath(__file__)))
                                if a.tunableop else None),
                "gemm_epilogues": a.gemm_epilogues or None,
            },
            "mfu": round(mfu, 4),
            "hfu": round(mfu * recompute, 4),
            "peak_mem_gib": gib(max(r[2] for r in per_rank)) if cuda else None,
            "final_loss": round(float(loss.item()), 4),
            "rccl_world": dist.get_world_size(),
            "backend": dist.get_backend(),
            "launcher": os.environ.get("BLLM_BENCH_LAUNCHER", "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ
                                       else ("env" if world > 1 else "single")),
            "per_rank": {"ms_per_step_min": round(1000 * min(r[0] for r in per_rank) / a.steps, 2),
                         "ms_per_step_max": round(ms, 2),
                         "ms_per_step": [round(1000 * r[0] / a.steps, 2) for r in per_rank],
                         "peak_mem_gib": [gib(r[2]) for r in per_rank] if cuda else None,
                         "comm_exposed_ms": [round(r[3], 3) for r in per_rank]},
            # per-step time each rank's compute stream sat waiting on a collective (parallel/
            # commstats.py); max over ranks.  0 at world 1 (no-shard engines issue none)
            "comm_exposed_ms": round(max(r[3] for r in per_rank), 3),
            "comm": {"by_kind_rank0": comm_kinds[0],
                     # achieved bandwidth of every collective of the timed steps (rank 0):
                     # RCCL's own issue-to-complete time per collective; busbw is per link
                     "gbps_by_kind": comm_bw,
                     "fsdp_prefetch": getattr(engine, "prefetch", None) if a.parallel == "fsdp" else None,
                     "bucket_mib": getattr(engine, "bucket_mb", None),
                     "adapted": adapt_hist,
                     "per_rank_fsdp_prefetch": [k[0] for k in knobs_all] if a.parallel == "fsdp" else None,
                     "per_rank_bucket_mib": [k[1] for k in knobs_all],
                     "deferred_init": bool(getattr(engine, "deferred_init", False)),
                     # warm-up steps' collectives compared across ranks (parallel/seqcheck.py)
                     "order_check": {"enabled": seq.enabled, "calls_checked_rank0": seq_checked,
                                     "steps": a.warmup}},
        }
        if rccl_on:
            from building_llm_from_scratch_amd.utils.telemetry import rccl_topology
            out["rccl_topology"] = rccl_topology(a.rccl_log) or {"log": a.rccl_log, "lines": 0}
        # what the box did during the timed steps (clocks, power, temperature, throttle residency)
        # and whether the GEMM tuning table was taken: box-to-box differences become readable
        out["telemetry"] = {"rank0": telem_all[0],
                            "sclk_mhz_avg_per_rank": [t.get("sclk_mhz_avg") for t in telem_all]}
        out["versions"] = library_versions() if cuda else {"torch": torch.__version__, "hip": torch.version.hip}
        out["tunableop"] = tunableop_status(a.tunableop) if cuda else None
        if data_check is not None:
            out["data_check"] = data_check
        if loss_trace is not None:
            out["loss_trace"] = [round(v, 6) for v in loss_trace]
        if getattr(engine, "prefetch", None) is not None and not getattr(engine, "no_shard", True):
            out["config"]["fsdp_prefetch"] = engine.prefetch
        if plan is not None:
            out["ckpt_plan"] = dict(plan.summary(), probe_peak_gib=gib(probe_peak) if probe_peak else None)
        if prof is not None:
            out["profile_ms"] = prof
        print(json.dumps(out), flush=True)
    if a.tunableop_tune and cuda and hasattr(torch.cuda.tunable, "write_file"):
        torch.cuda.tunable.write_file()     # (newer PyTorch writes the results file at exit itself)
    # leave together: a rank tearing its gloo pairs down while rank 0 still assembles the line
    # aborted one rank of eight (SIGABRT at exit) under a loaded CPU test run
    dist.barrier()
    dist.destroy_process_group()


def profile_phases(model, opt, next_batch, dev, n=3):
    import torch
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    res = {"fwd": 0.0, "bwd": 0.0, "clip+opt": 0.0}
    for i in range(n):
        x, y = next_batch(i)
        e = [ev() for _ in range(4)]
        e[0].record()
        loss = model(x, y)
        e[1].record()
        loss.backward()
        e[2].record()
        opt.clip_grad_norm_(1.0)
        opt.step()
        e[3].record()
        torch.cuda.synchronize()
        res["fwd"] += e[0].elapsed_time(e[1]) / n
        res["bwd"] += e[1].elapsed_time(e[2]) / n
        res["clip+opt"] += e[2].elapsed_time(e[3]) / n
    return {k: round(v, 2) for k, v in res.items()}


if __name__ == "__main__":
    launch(sys.argv[1:])
