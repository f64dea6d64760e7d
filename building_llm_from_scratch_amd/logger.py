"""Logging (reference logger.py:4-42) with a rank prefix and an optional JSONL metrics sink.

The reference's ``setup_logger(name, level)`` contract is kept (per-module StreamHandler,
``'%(asctime)s - %(name)s - %(levelname)s - %(message)s'``, ``propagate=False``); the
format additionally carries ``[rank N]`` when running distributed.
"""
from __future__ import annotations

import json
import logging
import os
import time
from typing import Optional


class _RankFilter(logging.Filter):
    def filter(self, record):
        r = os.environ.get("RANK")
        record.rank = f"[rank {r}] " if r is not None and os.environ.get("WORLD_SIZE", "1") != "1" else ""
        return True


def setup_logger(name: str, level: int = logging.INFO) -> logging.Logger:
    logger = logging.getLogger(name)
    logger.setLevel(level)
    if not logger.handlers:
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter(
            fmt="%(asctime)s - %(name)s - %(levelname)s - %(rank)s%(message)s",
            datefmt="%Y-%m-%d %H:%M:%S"))
        h.addFilter(_RankFilter())
        logger.addHandler(h)
        logger.propagate = False
    return logger


class MetricsWriter:
    """Append-only JSONL metrics (step, loss, lr, tokens/s, memory). Rank-0 only by caller."""

    def __init__(self, path: Optional[str]):
        self.path = path
        self._fh = open(path, "a", encoding="utf-8") if path else None

    def write(self, **record):
        if self._fh is None:
            return
        record.setdefault("time", time.time())
        self._fh.write(json.dumps(record) + "\n")
        self._fh.flush()

    def close(self):
        if self._fh:
            self._fh.close()
            self._fh = None
