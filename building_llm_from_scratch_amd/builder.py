"""Component builder (reference build_components.py:50-323).

build_config -> build_model (weights, LoRA, engine: local / DDP / ZeRO-1 / FSDP) ->
build_optimizer (fused AdamW, wd 0.1; sharded slots under ZeRO-1 / FSDP) -> build_tokenizer.

Differences: errors propagate instead of ``return None``; GPT-2 honours
``--data_type``; Llama-2 builds (theta 10000, eos ``</s>``/2, activation checkpointing);
``--mixed_precision`` maps to the FSDP compute/reduce dtype with fp32 master weights
(the reference's import of non-existent ``fpSixteen``/``bfSixteen`` is defect 2).
"""
from __future__ import annotations

import torch

from .config import datatype_mapping, debug_config, get_config
from .data.tokenizer import build_tokenizer as _build_tokenizer
from .logger import setup_logger
from .models import build_model as _build_model
from .models.lora import replace_linear_with_lora
from .models.weights import load_pretrained
from .parallel import setup_engine
from .parallel.mixed_precision import get_policy
from .train.optim import FusedAdamW
from .utils import misc

logger = setup_logger("build_components")


def precision_policy(args):
    """``--mixed_precision`` policy (parallel/mixed_precision.py) or None."""
    mp = getattr(args, "mixed_precision", None)
    return get_policy(mp) if mp else None


def compute_dtype(args) -> torch.dtype:
    pol = precision_policy(args)
    if pol is not None:
        return pol.param_dtype
    return datatype_mapping[args.data_type]


def build_config(args):
    cfg = get_config(args.model, args.num_params, context_length=getattr(args, "context_length", 1024) or 1024)
    cfg = cfg.replace(dtype=compute_dtype(args))
    if args.debug:
        cfg = debug_config(cfg)
    # after --debug (the reference applies its debug qkv_bias=False last, build_components.py:
    # 69-80, which makes --debug --load_weights unloadable: HF GPT-2 always has qkv biases)
    if args.load_weights and args.model == "GPT2":
        cfg = cfg.replace(qkv_bias=True)
    return cfg


def engine_kind(args) -> str:
    if args.run_type != "multi_gpu":
        return "local"
    if args.use_fsdp:
        return "fsdp"
    if args.use_zero_opt:
        return "zero1"
    return "ddp"


def plan_checkpointing(config, args, device, world: int = 1):
    """``--actv_ckpt_mode auto``: the per-block plan of train/memplan.py for this rank's engine,
    batch and device capacity (bench.py's headline policy)."""
    from .train import memplan
    total = None
    if device is not None and torch.device(device).type == "cuda":
        total = torch.cuda.get_device_properties(torch.device(device)).total_memory
    budget = args.ckpt_budget_gib * memplan.GIB if getattr(args, "ckpt_budget_gib", None) else None
    trainable = 1.0
    if args.use_lora:   # frozen base: no fp32 master / moments / grads for it (LoRA params are tiny)
        trainable = 0.0
    elt = torch.empty((), dtype=config.dtype).element_size()
    return memplan.plan_ckpt(config, args.batch_size, config.context_length, world=world, engine=engine_kind(args),
                             budget=budget, device_total=total, elt=elt,
                             prefetch=max(1, getattr(args, "fsdp_prefetch", 0) or 2), trainable_frac=trainable)


def build_model(config, rank, device, args):
    misc.start_memory_tracking()
    if getattr(args, "gemm_epilogues", ""):
        from .models.linear import use_gemm_epilogues
        use_gemm_epilogues([e for e in args.gemm_epilogues.split(",") if e])
    ckpt = getattr(args, "actv_ckpt_mode", None) or ("full" if args.use_actv_ckpt else "none")
    plan = None
    if ckpt == "auto":
        plan = plan_checkpointing(config, args, device, getattr(args, "world_size", 1))
        ckpt = "selective"
    model = _build_model(config, use_actv_ckpt=ckpt, device=device)
    if plan is not None:
        model.set_block_modes(plan.modes)
        model.ckpt_plan = plan    # the trainer re-plans after the first step's measured peak
        if rank == 0:
            s = plan.summary()
            logger.info(f"Activation checkpointing (auto): {s['full']} blocks fully recomputed, "
                        f"{s['selective']} selective; estimated peak {s['est_peak_gib']} GiB of "
                        f"{s['budget_gib']} GiB budget")
    if getattr(args, "actv_ckpt_segments", None):
        model.set_actv_ckpt(ckpt, args.actv_ckpt_segments)
    if rank == 0:
        logger.info(f"Total parameters: {misc.get_num_params(model):,}")
        misc.model_memory_size(model, config.dtype)
    if args.load_weights:
        path = load_pretrained(model, args.model, args.num_params, getattr(args, "weights_path", None))
        if rank == 0:
            logger.info(f"Loaded pretrained weights from {path}")
    if args.use_lora:
        for p in model.parameters():
            p.requires_grad = False
        replace_linear_with_lora(model, rank=args.lora_rank, alpha=args.lora_alpha, dtype=config.dtype)
        if rank == 0:
            n = sum(p.numel() for p in model.parameters() if p.requires_grad)
            logger.info(f"Total trainable LoRA parameters: {n:,}")
    if getattr(args, "resume", None):
        # weights go in BEFORE the engine shards / buckets them and before the optimizer
        # copies its fp32 master from them (loading later would be reverted by the next step)
        from .train.checkpoint import load_model
        load_model(model, args.resume)
        if rank == 0:
            logger.info(f"Resumed weights from {args.resume}")
    pol = precision_policy(args)
    reduce = pol.reduce_dtype if pol is not None else None
    if pol is not None and rank == 0:
        logger.info(f"Mixed precision: {pol}")
    engine = setup_engine(model, engine_kind(args), device=device, reduce_dtype=reduce,
                          reshard_after_forward=not getattr(args, "no_reshard_after_forward", False),
                          prefetch=getattr(args, "fsdp_prefetch", 0),
                          bucket_mb=getattr(args, "bucket_mb", 256.0))
    if rank == 0:
        misc.print_memory_usage()
    return model, engine


def build_optimizer(args, model, engine):
    return FusedAdamW(model, lr=args.lr, weight_decay=0.1, engine=engine)


def build_tokenizer(rank, args, config):
    return _build_tokenizer(args.model, config, getattr(args, "tokenizer_path", None))


def build_components(rank: int, device, args):
    """Returns (config, model, optimizer, tokenizer, engine)."""
    config = build_config(args)
    model, engine = build_model(config, rank, device, args)
    optimizer = build_optimizer(args, model, engine)
    tokenizer = build_tokenizer(rank, args, config)
    return config, model, optimizer, tokenizer, engine
