"""Rank-gated printing and JSONL progress logging (reference: rank-0 prints every 10 steps,
part3_mpi_gpu_train.py:118-119)."""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Any, Optional


class RankLogger:
    def __init__(self, rank: int = 0, jsonl_path: Optional[str] = None, quiet: bool = False):
        self.rank = rank
        self.quiet = quiet
        self.jsonl_path = jsonl_path
        if jsonl_path and rank == 0:
            os.makedirs(os.path.dirname(jsonl_path) or ".", exist_ok=True)

    def info(self, msg: str, all_ranks: bool = False) -> None:
        if self.quiet or (self.rank != 0 and not all_ranks):
            return
        prefix = f"[rank {self.rank}] " if all_ranks else ""
        print(prefix + msg, flush=True, file=sys.stdout)

    def event(self, kind: str, **fields: Any) -> None:
        if self.rank != 0 or not self.jsonl_path:
            return
        rec = {"ts": time.time(), "event": kind, **fields}
        with open(self.jsonl_path, "a") as f:
            f.write(json.dumps(rec) + "\n")
