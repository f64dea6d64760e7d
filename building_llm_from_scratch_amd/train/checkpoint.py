"""Checkpoints with the reference's layout + optional resume state.

* ``model_pg_{step}.pth`` / ``model_pg_{step}_interrupted.pth`` / ``model_pg_final.pth``:
  ``torch.save`` of a plain, prefix-free ``state_dict`` (reference train.py:231-257) —
  identical key names (incl. the ``att.mask|cos|sin`` buffers and fp32 RMSNorm weights).
  Rank 0 writes; under FSDP the full state dict is gathered unit by unit to rank 0.
* Extension (off unless ``--save_resume_state``): next to every ``<name>.pth`` a
  ``<name>.state.pt`` (``.rank{r}`` per rank when world > 1) with the optimizer state (fp32
  master, exp_avg, exp_avg_sq per flat slot — rank-local shards under ZeRO / FSDP), global
  step, LR, host RNGs, the model's dropout RNG counter, the data position (epoch, file, batch)
  and loss history.  ``--resume <name>.pth`` loads the weights BEFORE the engine shards them
  and the optimizer is built, then this state.  The reference has no resume path at all.
"""
from __future__ import annotations

import os
import random
from pathlib import Path
from typing import Optional

import numpy as np
import torch


def model_state_dict(model, engine=None) -> Optional[dict]:
    """Full, unwrapped state dict on CPU (rank 0 only gets a dict under FSDP)."""
    if engine is not None and hasattr(engine, "full_state_dict"):
        return engine.full_state_dict()
    return {k: v.detach().to("cpu") for k, v in model.state_dict().items()}


def save_model(model, path, engine=None, rank: int = 0):
    sd = model_state_dict(model, engine)
    if rank == 0 and sd is not None:
        tmp = str(path) + ".tmp"
        torch.save(sd, tmp)
        os.replace(tmp, path)


def resume_state_path(ckpt_path) -> Path:
    p = Path(ckpt_path)
    return p.with_name(p.stem + ".state.pt")


def load_state(path) -> dict:
    return torch.load(path, map_location="cpu", weights_only=True)


def load_model(model, path, strict: bool = True):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    return model.load_state_dict(sd, strict=strict)


def save_resume_state(path, optimizer, trainer_state: dict, rank: int = 0, world: int = 1):
    """Per-rank file (optimizer slots are rank-local under ZeRO / FSDP)."""
    st = {
        "trainer": trainer_state,
        "optim": [{k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in optimizer.state[s.param].items()}
                  for s in optimizer.slots],
        "lr": optimizer.param_groups[0]["lr"],
        "rng": _rng_state(),
        "world": world,
    }
    p = rank_state_path(path, rank, world)
    tmp = str(p) + ".tmp"
    torch.save(st, tmp)
    os.replace(tmp, p)


def rank_state_path(path, rank: int = 0, world: int = 1) -> Path:
    p = Path(path)
    return p.with_name(p.stem + f".rank{rank}" + p.suffix) if world > 1 else p


def load_resume_state(path, optimizer, rank: int = 0, world: int = 1) -> dict:
    p = rank_state_path(path, rank, world)
    st = torch.load(p, map_location="cpu", weights_only=True)
    assert st["world"] == world, "resume requires the same world size"
    for s, saved in zip(optimizer.slots, st["optim"]):
        cur = optimizer.state[s.param]
        for k, v in saved.items():
            if torch.is_tensor(v):
                cur[k].copy_(v.to(cur[k].device))
            else:
                cur[k] = v
        if "master" in cur:
            s.param.reshape(-1).copy_(cur["master"].to(s.param.dtype))
    _set_rng_state(st["rng"])
    return st["trainer"]


# RNG states as tensors / ints only, so resume files load with ``weights_only=True``
def _rng_state() -> dict:
    name, keys, pos, has_gauss, gauss = np.random.get_state()
    version, pstate, pgauss = random.getstate()
    return {"torch": torch.get_rng_state(), "np_name": name, "np_keys": torch.from_numpy(keys.astype(np.int64)),
            "np_pos": int(pos), "np_has_gauss": int(has_gauss), "np_gauss": float(gauss),
            "py_version": version, "py_state": torch.tensor(pstate, dtype=torch.int64),
            "py_gauss": pgauss}


def _set_rng_state(r: dict):
    torch.set_rng_state(r["torch"])
    np.random.set_state((r["np_name"], r["np_keys"].numpy().astype(np.uint32), r["np_pos"], r["np_has_gauss"],
                         r["np_gauss"]))
    random.setstate((r["py_version"], tuple(int(x) for x in r["py_state"].tolist()), r["py_gauss"]))
