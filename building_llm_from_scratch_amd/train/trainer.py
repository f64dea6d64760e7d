"""Training runtime (reference train.py:43-276).

Kept from the reference: constructor signature, ``train_model`` / ``finetune_model`` /
``train_epoch`` / ``train_batch`` / ``evaluate_model`` / ``calc_loss_loader`` /
``generate_and_print_sample`` / ``save_checkpoint``; linear warm-up ``initial_lr -> lr`` over
``warmup_steps`` then cosine to ``min_lr`` over the whole run (train.py:99-107); eval every
``eval_freq`` steps on ``eval_iter`` batches; a sample every ``print_sample_iter`` steps
("Every effort moves you", top-k 5, temperature 1, 200 tokens); ``model_pg_{step}.pth`` every
``save_ckpt_freq`` steps incl. step 0; ``model_pg_{step}_interrupted.pth`` on Ctrl-C; the same
log line format; returned (train_losses, val_losses, tokens_seen, lrs).

Changed on purpose: exceptions propagate (no log-and-continue), ``calc_loss_loader``
stops after ``num_batches`` (defect 8), logged losses / tokens are all-reduced across ranks
(defect 12), plus a tokens/s metric, JSONL metrics, fp16 dynamic loss scaling, a non-finite
loss guard, optional ``max_steps`` and resume state.
"""
from __future__ import annotations

import contextlib
import itertools
import math
import time
from pathlib import Path
from typing import Optional

import torch
import torch.distributed as dist

from ..logger import MetricsWriter, setup_logger
from ..utils.misc import read_json_file, read_text_file, text_to_token_ids, token_ids_to_text
from ..data.loaders import first_batches
from .checkpoint import resume_state_path, save_model, save_resume_state
from .generate import generate_cached

IGNORE_INDEX = -100   # the instruction collate's masked-target id (data/datasets.py)

logger = setup_logger("train")

# loaders are kept across epochs (read / tokenised / workers forked once) only for a one-file run:
# with several files, every file's dataset, persistent workers and prefetched batches would stay
# resident for the whole run; those runs rebuild a file's loaders per epoch and shut the previous
# file's workers down as soon as it is done
MAX_CACHED_FILES = 1


def _shutdown_loader(loader):
    """Stop a DataLoader's persistent worker processes now instead of at garbage collection."""
    it = getattr(loader, "_iterator", None)
    if it is not None and hasattr(it, "_shutdown_workers"):
        it._shutdown_workers()
    loader._iterator = None

ALPACA_CONTEXT = ("Below is an instruction that describes a task. Write a response that appropriately "
                  "completes the request.\n\n### Instruction:\nWhat is an antonym of 'complicated'?")


class DynamicLossScaler:
    """fp16 loss scaling: grow x2 every ``interval`` clean steps, halve and skip on overflow."""

    def __init__(self, init_scale=2.0 ** 16, interval=1000):
        self.scale = float(init_scale)
        self.interval = interval
        self.clean = 0

    def update(self, overflow: bool) -> bool:
        if overflow:
            self.scale = max(self.scale / 2.0, 1.0)
            self.clean = 0
            return False
        self.clean += 1
        if self.clean % self.interval == 0:
            self.scale *= 2.0
        return True


class Trainer:
    def __init__(self, model, optimizer, config, data_files, loaderObj, save_dir, warmup_steps=10,
                 initial_lr=1e-5, min_lr=1e-6, device="cpu", rank=0, eval_freq=1, save_ckpt_freq=1,
                 print_sample_iter=1, eval_iter=1, engine=None, max_grad_norm=1.0, metrics_file=None,
                 loss_scaler: Optional[DynamicLossScaler] = None, max_steps: Optional[int] = None,
                 sample_tokens: int = 200, save_resume: bool = False, world_size: int = 1,
                 profile_steps: Optional[str] = None, num_workers: int = 0, seed: int = 123,
                 comm_adapt_steps: int = 3):
        self.config = config
        self.model = model
        self.optimizer = optimizer
        self.data_files = data_files
        self.loaderObj = loaderObj
        self.save_dir = Path(save_dir)
        self.device = device
        self.rank = rank
        self.world_size = world_size
        self.engine = engine
        self.warmup_steps = warmup_steps
        self.initial_lr = initial_lr
        self.min_lr = min_lr
        self.eval_freq = eval_freq
        self.save_ckpt_freq = save_ckpt_freq
        self.print_sample_iter = print_sample_iter
        self.eval_iter = eval_iter
        self.max_grad_norm = max_grad_norm
        self.loss_scaler = loss_scaler
        self.max_steps = max_steps
        self.sample_tokens = sample_tokens
        self.save_resume = save_resume
        self.global_step = -1
        self.tokens_seen = 0
        # this rank's tokens since the last exact all-rank sum (_flush_tokens); instruction data
        # counts its real (non-ignored) targets, pretraining every input position
        self._tokens_pending = 0
        self.count_target_tokens = False
        self.train_losses, self.val_losses, self.track_lrs, self.track_tokens_seen = [], [], [], []
        self.metrics = MetricsWriter(metrics_file if rank == 0 else None)
        self._t_last = None
        self._tok_last = 0
        self.peak_lr = optimizer.param_groups[0]["lr"]
        self.total_training_steps = 1
        self.lr_increment = 0.0
        self.stop = False
        self.num_workers = num_workers
        self.seed = seed
        # data position: (epoch, file index, train batches of that file consumed); saved with
        # the resume state so a resumed run continues with the very next batch
        self.pos = (0, 0, 0)
        self._resume_pos = None
        # torch.profiler window "first:last" (global steps, inclusive) -> chrome trace per rank
        self.profile_steps = None
        if profile_steps:
            a, b = (int(v) for v in str(profile_steps).split(":"))
            self.profile_steps = (a, b)
        self._prof = None
        self._probed = False
        self._data_wait = 0.0
        # steps 1..comm_adapt_steps feed the engine's warm-up adaptation (parallel/ fsdp, ddp)
        self.comm_adapt_steps = comm_adapt_steps
        # file index -> (train loader, val loader, shuffle generator), kept across epochs when there
        # are few files: the data is read and tokenised once and the persistent workers forked once
        self._loaders = {}
        self._seq = None              # parallel/seqcheck.CollectiveSequence (warm-up steps)
        self._seq_timeout_s = 120.0

    # ------------------------------------------------------------------ helpers
    def _sync(self):
        if torch.cuda.is_available() and torch.device(self.device).type == "cuda":
            torch.cuda.synchronize()

    def _dist(self) -> bool:
        return self.world_size > 1 and dist.is_available() and dist.is_initialized()

    def _allreduce_mean(self, x: float) -> float:
        if not self._dist():
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        dist.all_reduce(t)
        return t.item() / self.world_size

    def _flush_tokens(self):
        """Add every rank's tokens since the last flush to ``tokens_seen`` (one int64 SUM
        all-reduce; called at the same steps on all ranks: eval points and checkpoint saves)."""
        n = self._tokens_pending
        self._tokens_pending = 0
        if self._dist():
            t = torch.tensor([n], dtype=torch.int64, device=self.device)
            dist.all_reduce(t)
            n = int(t.item())
        self.tokens_seen += n

    def lr_at(self, step: int) -> float:
        if step < self.warmup_steps:
            return self.initial_lr + step * self.lr_increment
        denom = max(1, self.total_training_steps - self.warmup_steps)
        progress = min(1.0, (step - self.warmup_steps) / denom)
        return self.min_lr + (self.peak_lr - self.min_lr) * 0.5 * (1 + math.cos(math.pi * progress))

    # ------------------------------------------------------------------ steps
    def calc_loss_batch(self, input_batch, target_batch):
        input_batch = input_batch.to(self.device, non_blocking=True)
        target_batch = target_batch.to(self.device, non_blocking=True)
        return self.model(input_batch, target_batch)

    def _profiler_tick(self):
        """Start / stop torch.profiler around the requested step window (HIP kernels appear as
        device events; rocprofv3 gives the kernel-level view, see profiles/)."""
        if self.profile_steps is None:
            return
        a, b = self.profile_steps
        if self.global_step == a and self._prof is None:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self._prof.__enter__()
        elif self.global_step == b + 1 and self._prof is not None:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self._prof.__exit__(None, None, None)
            path = self.save_dir / f"trace_steps{a}-{b}_rank{self.rank}.json"
            self._prof.export_chrome_trace(str(path))
            if self.rank == 0:
                logger.info(f"profiler trace written: {path}")
            self._prof = None

    def _order_check(self):
        """The collective-order checker for this step (None when not distributed or past warm-up)."""
        if not self._dist() or self.global_step > self.comm_adapt_steps:
            return None
        if self._seq is None:
            from ..parallel.seqcheck import CollectiveSequence
            self._seq = CollectiveSequence(timeout_s=self._seq_timeout_s)
        return self._seq

    def _step_body(self, input_batch, target_batch):
        loss = self.calc_loss_batch(input_batch, target_batch)
        if self.loss_scaler is not None:
            (loss * self.loss_scaler.scale).backward()
            inv = torch.tensor([1.0 / self.loss_scaler.scale], device=self.device)
            norm = self.optimizer.clip_grad_norm_(self.max_grad_norm, extra_scale=inv)
            overflow = not bool(torch.isfinite(norm).item())
            if self.loss_scaler.update(overflow):
                self.optimizer.step()
            elif self.rank == 0:
                logger.warning(f"fp16 overflow at step {self.global_step}; loss scale -> {self.loss_scaler.scale}")
        else:
            loss.backward()
            self.optimizer.clip_grad_norm_(self.max_grad_norm)
            self.optimizer.step()
        return loss

    def train_batch(self, input_batch, target_batch):
        self.optimizer.zero_grad()
        self.global_step += 1
        adapting = (self.engine is not None and hasattr(self.engine, "adapt")
                    and 1 <= self.global_step <= self.comm_adapt_steps)
        if adapting:   # the engine grows its prefetch / bucket size while a collective wait shows
            self._sync()
            self.engine.comm.reset(enabled=True)
            t_step = time.perf_counter()
        self._profiler_tick()
        lr = self.lr_at(self.global_step)
        for g in self.optimizer.param_groups:
            g["lr"] = lr
        self.track_lrs.append(lr)
        rc = getattr(self.model, "rctx", None)
        if rc is not None and self.loss_scaler is not None:
            # the fused head takes the logit gradient inside its forward: tell it the dloss that
            # backward will bring, so fp16 softmax tails are scaled before they are rounded
            rc.loss_scale = float(self.loss_scaler.scale)
        # warm-up steps 0..comm_adapt_steps: the step's collectives are recorded and compared
        # across ranks right after they are issued (parallel/seqcheck.py) -- a divergent order
        # raises naming the first differing call instead of hanging until the PG timeout
        seq = self._order_check()
        with seq.recording(f"step{self.global_step}") if seq is not None else contextlib.nullcontext():
            loss = self._step_body(input_batch, target_batch)
        if seq is not None:
            seq.verify(f"step{self.global_step}")
        # this rank's own count (reference train.py:123 counts per rank); padded instruction
        # batches differ in length across ranks, so the node total is an exact sum
        # (_flush_tokens) at every eval / checkpoint point, never numel x world_size
        if self.count_target_tokens:
            self._tokens_pending += int((target_batch != IGNORE_INDEX).sum())
        else:
            self._tokens_pending += input_batch.numel()
        if adapting:
            self._sync()
            rec = self.engine.adapt(1e3 * (time.perf_counter() - t_step))
            self.engine.comm.enabled = False
            if rec is not None and any(k.endswith("_new") for k in rec):
                if self.rank == 0:
                    logger.info(f"comm adaptation at step {self.global_step}: {rec}")
                # a deeper FSDP prefetch holds more gathered units than the checkpoint plan was
                # sized for (prefetch 2): measure the next step's peak and re-plan against it
                if getattr(self.model, "ckpt_plan", None) is not None and torch.device(self.device).type == "cuda":
                    torch.cuda.reset_peak_memory_stats(self.device)
                    self._probed = False
        if not self._probed and not adapting:
            self._probed = True
            self._probe_ckpt_plan()
        return loss

    def _probe_ckpt_plan(self):
        """``--actv_ckpt_mode auto``: check the planner's estimate against the first step's measured
        peak (max over ranks) and add fully recomputed blocks if it was over budget, exactly as
        bench.py does for the headline."""
        plan = getattr(self.model, "ckpt_plan", None)
        if plan is None or torch.device(self.device).type != "cuda":
            return
        from . import memplan
        torch.cuda.synchronize()
        pk = torch.tensor([float(torch.cuda.max_memory_allocated(self.device))], device=self.device)
        if self._dist():
            dist.all_reduce(pk, op=dist.ReduceOp.MAX)
        elt = torch.empty((), dtype=self.config.dtype).element_size()
        new = memplan.replan_after_probe(plan, self.config, self.loaderObj.batch_size,
                                         self.config.context_length, pk.item(), elt=elt)
        if new is not plan:
            self.model.set_block_modes(new.modes)
            self.model.ckpt_plan = new
            torch.cuda.reset_peak_memory_stats(self.device)
        if self.rank == 0:
            logger.info(f"Activation checkpointing (auto): first-step peak {pk.item() / memplan.GIB:.1f} GiB; "
                        + ("plan kept" if new is plan else f"re-planned: {new.summary()}"))

    def train_epoch(self, epoch_no, train_loader, val_loader, start_context="Every effort moves you",
                    file_index: int = 0, skip_batches: int = 0):
        self.model.train()
        it = iter(train_loader)
        if skip_batches:
            it = itertools.islice(it, skip_batches, None)
        bi = skip_batches - 1
        while True:
            t_wait = time.perf_counter()
            try:
                input_batch, target_batch = next(it)
            except StopIteration:
                break
            self._data_wait += time.perf_counter() - t_wait   # host time blocked on the loader
            bi += 1
            self.pos = (epoch_no, file_index, bi + 1)
            loss = self.train_batch(input_batch, target_batch)
            if self.global_step % self.eval_freq == 0:
                lv = float(loss.item())
                # training throughput since the last eval point, measured up to this loss read
                # (a device sync) and restarted after eval / sample / checkpoint: those phases
                # never count against tok/s
                now = time.perf_counter()
                if not math.isfinite(lv):
                    raise FloatingPointError(f"non-finite training loss at step {self.global_step}")
                self._flush_tokens()
                train_loss, val_loss = self.evaluate_model(train_loader, val_loader, self.eval_iter)
                self.train_losses.append(train_loss)
                self.val_losses.append(val_loss)
                self.track_tokens_seen.append(self.tokens_seen)
                tps = None
                if self._t_last is not None:
                    tps = (self.tokens_seen - self._tok_last) / max(now - self._t_last, 1e-9)
                self._tok_last = self.tokens_seen
                self._t_last = None
                if self.rank == 0:
                    logger.info(f"Epoch {epoch_no + 1} | Step {self.global_step} "
                                f"| Train Loss: {train_loss:.3f} | Val Loss: {val_loss:.3f}"
                                + (f" | {tps:,.0f} tok/s" if tps else ""))
                    cuda = torch.cuda.is_available()
                    self.metrics.write(step=self.global_step, epoch=epoch_no, train_loss=train_loss,
                                       val_loss=val_loss, lr=self.track_lrs[-1], tokens_seen=self.tokens_seen,
                                       tokens_per_s=tps, batch_loss=lv,
                                       # host seconds blocked on the data loader since the last
                                       # eval point, and the caching allocator's cumulative
                                       # free-and-retry count (each one a device sync)
                                       data_wait_s=round(self._data_wait, 4),
                                       alloc_retries=(torch.cuda.memory_stats().get("num_alloc_retries", 0)
                                                      if cuda else None),
                                       max_mem_gb=(torch.cuda.max_memory_allocated() / 1e9 if cuda else None))
                self._data_wait = 0.0
            if self.print_sample_iter and self.global_step % self.print_sample_iter == 0:
                self.generate_and_print_sample(start_context)
            if self.save_ckpt_freq and self.global_step % self.save_ckpt_freq == 0:
                self.save_checkpoint(f"model_pg_{self.global_step}.pth")
            if self._t_last is None:   # (re)start the throughput clock after the eval-step phases
                if torch.cuda.is_available() and torch.device(self.device).type == "cuda":
                    torch.cuda.synchronize()
                self._t_last = time.perf_counter()
                self._tok_last = self.tokens_seen
            if self.max_steps is not None and self.global_step + 1 >= self.max_steps:
                self.stop = True
                return

    def _setup_schedule(self, n_epochs):
        self.peak_lr = self.optimizer.param_groups[0]["lr"]
        self.total_training_steps = max(1, self.loaderObj.get_total_steps_epoch(self.data_files) * n_epochs)
        if self.max_steps is not None:
            self.total_training_steps = min(self.total_training_steps, self.max_steps)
        self.lr_increment = (self.peak_lr - self.initial_lr) / max(1, self.warmup_steps)

    def _progress(self, total):
        if self.rank != 0:
            return None
        try:
            from tqdm import tqdm
            return tqdm(total=total)
        except Exception:  # pragma: no cover
            return None

    def _loop(self, n_epochs, read, start_context):
        self._setup_schedule(n_epochs)
        pbar = self._progress(n_epochs * len(self.data_files))
        start = self._resume_pos or (0, 0, 0)
        try:
            for epoch in range(n_epochs):
                for fi, fp in enumerate(self.data_files):
                    if (epoch, fi) < start[:2]:
                        if pbar is not None:
                            pbar.update(1)
                        continue
                    skip = start[2] if (epoch, fi) == start[:2] else 0
                    # per-(epoch, file) shuffle seed: the order does not depend on how many
                    # random numbers were drawn before (sampling, dropout), so resume replays it
                    shuffle_seed = self.seed * 1_000_003 + epoch * 1009 + fi
                    cached = self._loaders.get(fi)
                    if cached is not None:
                        # the same loaders with the generator reseeded: the order a fresh
                        # generator with this seed gives (the sampler draws at iter())
                        train_loader, val_loader, g = cached
                        g.manual_seed(shuffle_seed)
                    else:
                        g = torch.Generator().manual_seed(shuffle_seed)
                        train_loader, val_loader = self.loaderObj.create_dataloaders(
                            read(fp), num_workers=self.num_workers, generator=g)
                        if len(self.data_files) <= MAX_CACHED_FILES:
                            self._loaders[fi] = (train_loader, val_loader, g)
                    if hasattr(train_loader.sampler, "set_epoch"):
                        train_loader.sampler.set_epoch(epoch)
                    self.train_epoch(epoch, train_loader, val_loader, start_context=start_context,
                                     file_index=fi, skip_batches=skip)
                    if fi not in self._loaders:
                        _shutdown_loader(train_loader)
                        _shutdown_loader(val_loader)
                        del train_loader, val_loader
                    if pbar is not None:
                        pbar.update(1)
                    if self.stop:
                        return self._results()
        except KeyboardInterrupt:
            self.save_checkpoint(f"model_pg_{self.global_step}_interrupted.pth")
        return self._results()

    def train_model(self, n_epochs):
        eos = self.config["eos_text"]
        return self._loop(n_epochs, lambda fp: read_text_file(fp) + " " + eos + " ", "Every effort moves you")

    def finetune_model(self, n_epochs):
        self.count_target_tokens = True   # padded instruction batches: count real targets
        return self._loop(n_epochs, read_json_file, ALPACA_CONTEXT)

    def _results(self):
        self._flush_tokens()
        return self.train_losses, self.val_losses, self.track_tokens_seen, self.track_lrs

    # ------------------------------------------------------------------ eval / sample / ckpt
    def generate_and_print_sample(self, start_context, temperature=1.0, top_k=5, memory_check=True,
                                  max_new_tokens=None):
        self.model.eval()
        encoded = text_to_token_ids(start_context, self.loaderObj.tokenizer, self.config).to(self.device)
        token_ids = generate_cached(self.model, encoded, max_new_tokens or self.sample_tokens,
                             self.config["context_length"], temperature=temperature, top_k=top_k,
                             eos_id=self.config["eos_id"])
        decoded = token_ids_to_text(token_ids.cpu(), self.loaderObj.tokenizer)
        self.model.train()
        if self.rank == 0 and memory_check:
            logger.info(f"Generated Sample: {decoded.replace(chr(10), ' ')}")
        return decoded

    def save_checkpoint(self, file_name):
        self._flush_tokens()   # the resume state carries the exact all-rank count
        if self._dist():
            dist.barrier()
        path = self.save_dir / file_name
        save_model(self.model, path, self.engine, self.rank)
        if self.save_resume:
            save_resume_state(resume_state_path(path), self.optimizer, self.trainer_state(),
                              self.rank, self.world_size)
        if self.rank == 0:
            logger.info(f"Checkpoint saved: {path}")
        if self._dist():
            dist.barrier()

    _STATE_KEYS = ("global_step", "tokens_seen", "train_losses", "val_losses", "track_lrs", "track_tokens_seen")
    # batch order for a given (seed, epoch, file): 2 = the shuffle drawn straight from the
    # per-(epoch, file) generator by RandomSampler, worker seeds from a fixed generator
    # (data/loaders.py); states without it were written by builds that drew the worker base seed
    # from that generator first, so their skip-ahead replays a different order
    DATA_ORDER_VERSION = 2

    def trainer_state(self) -> dict:
        st = {k: getattr(self, k) for k in self._STATE_KEYS}
        rc = self.model.rctx
        st.update(pos=list(self.pos), rng_seed=int(rc.seed), rng_offset=int(rc._offset),
                  data_order_version=self.DATA_ORDER_VERSION,
                  loss_scale=(self.loss_scaler.scale if self.loss_scaler else None),
                  loss_scale_clean=(self.loss_scaler.clean if self.loss_scaler else None))
        return st

    def load_trainer_state(self, st: dict):
        for k in self._STATE_KEYS:
            setattr(self, k, st[k])
        if "pos" in st:
            if st.get("data_order_version") != self.DATA_ORDER_VERSION and self.rank == 0:
                logger.warning(f"resume state has data-order version {st.get('data_order_version')} "
                               f"(this build: {self.DATA_ORDER_VERSION}): the batches after the resume "
                               "point follow this build's shuffle, not the interrupted run's")
            self.pos = tuple(st["pos"])
            self._resume_pos = self.pos
            rc = self.model.rctx
            rc.seed, rc._offset = st["rng_seed"], st["rng_offset"]
            if self.loss_scaler is not None and st.get("loss_scale") is not None:
                self.loss_scaler.scale, self.loss_scaler.clean = st["loss_scale"], st["loss_scale_clean"]

    @torch.no_grad()
    def calc_loss_loader(self, data_loader, num_batches=None):
        if len(data_loader) == 0:
            return float("nan")
        num_batches = min(num_batches or len(data_loader), len(data_loader))
        total = 0.0
        for inp, tgt in first_batches(data_loader, num_batches):
            total += float(self.calc_loss_batch(inp, tgt).item())
        return self._allreduce_mean(total / num_batches)

    def evaluate_model(self, train_loader, val_loader, eval_iter=5):
        self.model.eval()
        with torch.no_grad():
            train_loss = self.calc_loss_loader(train_loader, eval_iter)
            val_loss = self.calc_loss_loader(val_loader, eval_iter)
        self.model.train()
        return train_loss, val_loss
