"""Command line (reference args.py:8-99 and main.py:22-193).

The 27 reference flags keep their names, types, choices, defaults and validation rules;
extensions are additive and default to reference behaviour.  Launch modes:
  * ``--run_type single_gpu``: one process (GPU if present, else CPU);
  * ``--run_type multi_gpu``: under ``torchrun`` (RANK/WORLD_SIZE/LOCAL_RANK from the env)
    or, like the reference, self-spawned with ``mp.spawn`` over every visible GPU.
Collectives: backend ``nccl`` (= RCCL on ROCm, over xGMI) on GPUs, ``gloo`` on CPU.
"""
from __future__ import annotations

import argparse
import os
import warnings
from datetime import timedelta
from functools import partial
from pathlib import Path

import torch

from .config import model_params_mapping
from .logger import setup_logger

logger = setup_logger("main")


def perform_checks(args):
    if not args.warnings:
        warnings.filterwarnings("ignore")
    if not os.path.exists(args.data_dir):
        if args.synthetic_data:
            os.makedirs(args.data_dir, exist_ok=True)
        else:
            raise FileNotFoundError(f"Data directory '{args.data_dir}' does not exist.")
    if args.num_params not in model_params_mapping.get(args.model, []):
        raise ValueError(f"Unsupported model configuration: {args.model} with {args.num_params}. "
                         f"Supported sizes: {model_params_mapping.get(args.model, [])}")
    if args.run_type == "single_gpu" and args.use_fsdp:
        raise ValueError("FSDP requires multi-GPU. It's not supported for single GPU training.")
    if args.use_zero_opt and args.use_fsdp:
        raise ValueError("Zero Redundancy Optimizer cannot be used with FSDP.")
    if args.use_fsdp and not torch.cuda.is_available() and args.backend != "gloo":
        raise EnvironmentError("FSDP requires GPU devices (or --backend gloo for CPU testing).")
    if not args.use_fsdp and args.mixed_precision:
        raise ValueError("Mixed precision can only be enabled with FSDP.")
    if getattr(args, "actv_ckpt_mode", None) == "auto" and getattr(args, "actv_ckpt_segments", None):
        # the planner's per-block modes ARE the segmentation; a segment count would replace them
        # with plain selective checkpointing while the log and the first-step probe still
        # reasoned about the plan
        raise ValueError("--actv_ckpt_mode auto chooses the recomputed blocks itself; "
                         "it cannot be combined with --actv_ckpt_segments.")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Large Language Model Training Configuration (MI355X-native)")
    # ---- reference flags (args.py:46-93)
    p.add_argument("--data_dir", type=str,
                   default="/home/ec2-user/train-llm-from-scratch/Datasets/Gutenberg/data_dir_small")
    p.add_argument("--output_dir", type=str, default="model_checkpoints")
    p.add_argument("--n_epochs", type=int, default=2)
    p.add_argument("--batch_size", type=int, default=4)
    p.add_argument("--lr", type=float, default=5e-4)
    p.add_argument("--warmup_steps", type=int, default=10)
    p.add_argument("--initial_lr", type=float, default=1e-5)
    p.add_argument("--min_lr", type=float, default=1e-6)
    p.add_argument("--print_sample_iter", type=int, default=10)
    p.add_argument("--eval_freq", type=int, default=10)
    p.add_argument("--save_ckpt_freq", type=int, default=100)
    p.add_argument("--model", type=str, default="GPT2", choices=["GPT2", "llama2", "llama3", "llama3_1", "llama3_2"])
    p.add_argument("--num_params", type=str, default="124M")
    p.add_argument("--load_weights", action="store_true")
    p.add_argument("--debug", action="store_true")
    p.add_argument("--run_type", type=str, default="single_gpu", choices=["single_gpu", "multi_gpu"])
    p.add_argument("--use_fsdp", action="store_true")
    p.add_argument("--use_zero_opt", action="store_true")
    p.add_argument("--use_actv_ckpt", action="store_true")
    p.add_argument("--data_type", type=str, default="fp32", choices=["fp32", "fp16", "bf16"])
    p.add_argument("--mixed_precision", type=str, choices=["fp16", "bf16", "bf16_hybrid", "fp32"])
    p.add_argument("--finetune", action="store_true")
    p.add_argument("--dataset", type=str, default="gutenberg", choices=["gutenberg", "alpaca"])
    p.add_argument("--use_lora", action="store_true")
    p.add_argument("--lora_rank", type=int, default=64)
    p.add_argument("--lora_alpha", type=int, default=32)
    p.add_argument("--warnings", action="store_true")
    # ---- extensions (defaults = reference behaviour)
    x = p.add_argument_group("extensions")
    x.add_argument("--context_length", type=int, default=1024, help="Llama ctx clamp (reference: fixed 1024)")
    x.add_argument("--actv_ckpt_mode", choices=["none", "selective", "full", "auto"], default=None,
                   help="granularity; --use_actv_ckpt alone = full (reference semantics); auto = the HBM "
                        "memory planner (train/memplan.py: every block selective plus the fewest fully "
                        "recomputed blocks under --ckpt_budget_gib, re-planned after the first step's "
                        "measured peak) -- the headline bench's policy")
    x.add_argument("--ckpt_budget_gib", type=float, default=None,
                   help="auto mode: per-rank peak-memory ceiling (default 250 GiB, capped at device - 18 GiB)")
    x.add_argument("--gemm_epilogues", nargs="?", const="swiglu,rope,gelu", default="",
                   help="gate/up + SwiGLU, QKV + RoPE and c_fc + bias + GELU on the fused-epilogue GEMM kernel "
                        "(csrc/gemm_nt.hip) instead of the library GEMM + a separate pass; measured slower on "
                        "MI355X; bare flag = all three, or a comma list of swiglu,rope,gelu")
    x.add_argument("--actv_ckpt_segments", type=int, default=None,
                   help="full mode: checkpoint_sequential segments (default n_layers = reference); "
                        "fewer segments recompute fewer blocks for more memory")
    x.add_argument("--tokenizer_path", type=str, default=None)
    x.add_argument("--weights_path", type=str, default=None)
    x.add_argument("--max_steps", type=int, default=None)
    x.add_argument("--metrics_file", type=str, default=None, help="JSONL metrics (rank 0)")
    x.add_argument("--seed", type=int, default=123)
    x.add_argument("--backend", choices=["nccl", "gloo"], default=None, help="default: nccl on GPU, gloo on CPU")
    x.add_argument("--nprocs", type=int, default=None, help="processes for self-spawned multi_gpu (default: #GPUs)")
    x.add_argument("--device", choices=["auto", "cpu", "cuda"], default="auto")
    x.add_argument("--synthetic_data", action="store_true",
                   help="generate Gutenberg-/Alpaca-shaped data into --data_dir if it is empty")
    x.add_argument("--synthetic_mb", type=float, default=0.5,
                   help="size of the generated Gutenberg-shaped corpus (MB of text)")
    x.add_argument("--sample_tokens", type=int, default=200)
    x.add_argument("--resume", type=str, default=None,
                   help="model_pg_*.pth to resume from (+ its .state.pt written by --save_resume_state)")
    x.add_argument("--save_resume_state", action="store_true",
                   help="write optimizer / step / RNG / data-position state next to every checkpoint")
    x.add_argument("--num_workers", type=int, default=2, help="DataLoader workers (reference train.py:167,195)")
    x.add_argument("--token_cache", type=str, default=None,
                   help="memmapped token cache dir (default <output_dir>/token_cache; 'none' disables)")
    x.add_argument("--pg_timeout_min", type=float, default=30.0,
                   help="collective timeout (minutes): a wedged RCCL/gloo collective raises instead of hanging")
    x.add_argument("--bucket_mb", type=float, default=256.0, help="DDP all-reduce bucket size")
    x.add_argument("--fsdp_prefetch", type=int, default=0,
                   help="FSDP: units all-gathered ahead of the computing one (0 = auto from gather vs compute time)")
    x.add_argument("--comm_adapt_steps", type=int, default=3,
                   help="first N steps: grow the FSDP prefetch depth / DDP bucket size while an exposed "
                        "collective wait exceeds 2%% of the step (MAX over ranks)")
    x.add_argument("--no_reshard_after_forward", action="store_true",
                   help="FSDP: keep gathered params from forward to backward (ZeRO-2 style)")
    x.add_argument("--tunableop", type=str, default="auto",
                   help="TunableOp GEMM table (read-only): a CSV path, 'auto' = the shipped MI355X table of "
                        "--model/--num_params if there is one (configs/tunableop_*), or 'none'")
    x.add_argument("--no_plot", action="store_true")
    x.add_argument("--skip_final_save", action="store_true",
                   help="do not write model_pg_final.pth (throughput runs of multi-GB models)")
    x.add_argument("--profile_steps", type=str, default=None,
                   help="torch.profiler window 'first:last' (global steps) -> chrome trace in --output_dir")
    return p


def get_args(argv=None):
    args = build_parser().parse_args(argv)
    perform_checks(args)
    return args


# ---------------------------------------------------------------------------
def _device_for(args, local_rank: int):
    use_cuda = torch.cuda.is_available() and args.device != "cpu"
    if use_cuda:
        torch.cuda.set_device(local_rank)
        return torch.device("cuda", local_rank)
    return torch.device("cpu")


def ddp_setup(rank: int, world_size: int, args):
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "12355")
    device = _device_for(args, int(os.environ.get("LOCAL_RANK", rank)))
    backend = args.backend or ("nccl" if device.type == "cuda" else "gloo")
    timeout = timedelta(minutes=getattr(args, "pg_timeout_min", 30.0))
    if backend == "nccl":
        from .parallel import nccl_pg_options
        dist.init_process_group("nccl", rank=rank, world_size=world_size, device_id=device, timeout=timeout,
                                pg_options=nccl_pg_options(timeout))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world_size, timeout=timeout)
    return device


def _prepare_data(args, cfg, rank):
    from .data.synthetic import make_alpaca_json, make_gutenberg_corpus
    files = [os.path.join(path, n) for path, _, fs in os.walk(args.data_dir) for n in fs
             if n.endswith((".txt", ".json"))]
    if not files and args.synthetic_data and rank == 0:
        if args.finetune:
            make_alpaca_json(os.path.join(args.data_dir, "instruction-data-alpaca.json"), 1000)
        else:
            make_gutenberg_corpus(args.data_dir, n_files=1, mb_per_file=getattr(args, "synthetic_mb", 0.5))
    return files


def main(rank: int, args):
    import torch.distributed as dist

    from . import utils
    from .builder import build_components
    from .data.datasets import custom_collate_fn
    from .data.loaders import DataloaderIF, DataloaderPT
    from .train.checkpoint import load_resume_state, rank_state_path, resume_state_path
    from .train.trainer import DynamicLossScaler, Trainer

    from .utils.gemm_tuning import install_table, resolve_table
    world = getattr(args, "world_size", 1)
    if torch.cuda.is_available() and args.device != "cpu":   # before the first GEMM
        table = resolve_table(args.tunableop, args.model, args.num_params)
        install_table(table, int(os.environ.get("LOCAL_RANK", rank)))
        if rank == 0 and table:
            logger.info(f"GEMM selection table (TunableOp, read-only): {os.path.relpath(table)}")
    if args.run_type == "multi_gpu":
        device = ddp_setup(rank, world, args)
    else:
        device = _device_for(args, 0)

    utils.set_seed(args.seed)
    config, model, optimizer, tokenizer, engine = build_components(rank, device, args)

    _prepare_data(args, config, rank)
    if args.run_type == "multi_gpu":
        dist.barrier()
    all_files = sorted(os.path.join(path, n) for path, _, fs in os.walk(args.data_dir) for n in fs
                       if n.endswith((".txt", ".json")))
    if not all_files:
        raise FileNotFoundError("No training files found in specified directory.")
    if rank == 0:
        logger.info(f"Total training files detected: {len(all_files)}")

    kw = dict(tokenizer=tokenizer, batch_size=args.batch_size, max_length=config["context_length"],
              dataset_name=args.dataset, run_type=args.run_type, train_ratio=0.9)
    if args.finetune:
        collate = partial(custom_collate_fn, pad_token_id=config["eos_id"], allowed_max_length=config["context_length"])
        loader = DataloaderIF(collate_func=collate, **kw)
    else:
        cache = None if args.token_cache == "none" else (args.token_cache or os.path.join(args.output_dir, "token_cache"))
        loader = DataloaderPT(stride=config["context_length"], eos_text=config["eos_text"], collate_func=None,
                              cache_dir=cache, **kw)
        # rank 0 tokenises every file once into the memmapped cache; the others map it
        if cache and rank == 0:
            loader.pretokenize(all_files)
        if cache and args.run_type == "multi_gpu":
            dist.barrier()

    out_dir = Path(args.output_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    trainer = Trainer(model=model, optimizer=optimizer, config=config, data_files=all_files, loaderObj=loader,
                      save_dir=out_dir, warmup_steps=args.warmup_steps, initial_lr=args.initial_lr,
                      min_lr=args.min_lr, device=device, rank=rank, eval_freq=args.eval_freq,
                      save_ckpt_freq=args.save_ckpt_freq, print_sample_iter=args.print_sample_iter, eval_iter=5,
                      engine=engine, metrics_file=args.metrics_file,
                      loss_scaler=DynamicLossScaler() if config.dtype == torch.float16 else None,
                      max_steps=args.max_steps, sample_tokens=args.sample_tokens,
                      save_resume=args.save_resume_state, world_size=world, profile_steps=args.profile_steps,
                      num_workers=args.num_workers, seed=args.seed, comm_adapt_steps=args.comm_adapt_steps)
    trainer.generate_and_print_sample("Every effort moves you", temperature=1.0, top_k=5, memory_check=True)
    if args.resume:
        # after the start-up sample: the restored host RNG state is the one saved at the checkpoint
        st_path = resume_state_path(args.resume)
        if rank_state_path(st_path, rank, world).exists():
            trainer.load_trainer_state(load_resume_state(st_path, optimizer, rank, world))
            if rank == 0:
                logger.info(f"Resumed optimizer / step / data position from {st_path} (step {trainer.global_step})")
        elif rank == 0:
            logger.warning(f"--resume: no optimizer state next to {args.resume} ({st_path.name}); "
                           "continuing from the weights only with fresh AdamW moments and step 0")
    if args.finetune:
        train_losses, val_losses, tokens_seen, lrs = trainer.finetune_model(n_epochs=args.n_epochs)
    else:
        train_losses, val_losses, tokens_seen, lrs = trainer.train_model(n_epochs=args.n_epochs)
    if rank == 0:
        if train_losses and not args.no_plot:
            epochs = torch.linspace(0, args.n_epochs, len(train_losses))
            utils.plot_losses(epochs, tokens_seen, train_losses, val_losses, out_dir)
        logger.info("Training complete. Final model saved.")
        if device.type == "cuda":
            logger.info(f"Maximum GPU memory used: {torch.cuda.max_memory_allocated() / 1e9:.2f} GB")
    if not args.skip_final_save:
        trainer.save_checkpoint("model_pg_final.pth")
    if args.run_type == "multi_gpu":
        dist.barrier()
        dist.destroy_process_group()
    return trainer


def _spawn_entry(rank, args):
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(args.world_size)
    main(rank, args)


def cli(argv=None):
    args = get_args(argv)
    if args.run_type == "multi_gpu":
        if "RANK" in os.environ and "WORLD_SIZE" in os.environ:  # torchrun
            args.world_size = int(os.environ["WORLD_SIZE"])
            return main(int(os.environ["RANK"]), args)
        import torch.multiprocessing as mp
        n = args.nprocs or (torch.cuda.device_count() if torch.cuda.is_available() else 2)
        args.world_size = n
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "12355")
        mp.spawn(_spawn_entry, args=(args,), nprocs=n, join=True)
        return None
    args.world_size = 1
    return main(0, args)
