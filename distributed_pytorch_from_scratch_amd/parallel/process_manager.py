"""Process-group manager: one process per MI355X, laid out on a (dp, tp) grid.

Reference parity: ``process_manager.py:8-25`` (``ProcessGroupManager``, ``init_pgm``, module
global ``pgm``).  The reference only supports ``tp_size == world_size``; here the grid is
``world = dp_size x tp_size`` with TP innermost, so the ranks of one TP group are adjacent
GPUs (``LOCAL_RANK`` ``k*tp .. k*tp+tp-1``), which on an 8-GPU xGMI node are all directly
linked (fully connected mesh), and DP replicas sit across TP groups.  ``dp_size == 1`` gives
the reference behaviour exactly (``tp_rank == global_rank``, ``grid == arange(world)``).

Layers read ``pm.pgm`` at construction and forward time, so the model must be built after
``init_pgm`` (same contract as the reference, ``SURVEY.md`` §2.1 row 11).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

pgm: Optional["ProcessGroupManager"] = None


class ProcessGroupManager:
    """Holds the rank coordinates and the torch.distributed groups of one process."""

    def __init__(self, tp_size: int, dp_size: Optional[int] = None):
        assert dist.is_initialized(), "call torch.distributed.init_process_group first"
        self.global_rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        if dp_size is None:
            assert self.world_size % tp_size == 0, (
                f"world_size {self.world_size} not divisible by tp_size {tp_size}")
            dp_size = self.world_size // tp_size
        assert tp_size * dp_size == self.world_size, (
            f"tp_size({tp_size}) x dp_size({dp_size}) != world_size({self.world_size})")
        self.tp_size = tp_size
        self.dp_size = dp_size
        # grid[dp_rank, tp_rank] = global rank; TP innermost (adjacent GPUs).
        self.grid = torch.arange(self.world_size).view(dp_size, tp_size)
        self.dp_rank, self.tp_rank = [int(v) for v in (self.grid == self.global_rank).nonzero()[0]]
        self.backend = dist.get_backend()

        # Every rank must take part in every new_group call, in the same order.  RCCL groups get
        # high-priority HIP streams (their collectives sit on the overlapped critical path).
        kw = {}
        if self.backend == "nccl":
            kw["pg_options"] = dist.ProcessGroupNCCL.Options()
            kw["pg_options"].is_high_priority_stream = True
        self.tp_group = None
        self.dp_group = None
        for d in range(dp_size):
            ranks = self.grid[d].tolist()
            g = dist.new_group(ranks, **kw) if tp_size < self.world_size else dist.group.WORLD
            if d == self.dp_rank:
                self.tp_group = g
        for t in range(tp_size):
            ranks = self.grid[:, t].tolist()
            g = dist.new_group(ranks, **kw) if dp_size < self.world_size else dist.group.WORLD
            if t == self.tp_rank:
                self.dp_group = g
        self.tp_ranks = self.grid[self.dp_rank].tolist()
        self.dp_ranks = self.grid[:, self.tp_rank].tolist()
        self.tp_src_rank = self.tp_ranks[0]

    @property
    def is_tp_first(self) -> bool:
        return self.tp_rank == 0

    def __repr__(self) -> str:
        if self.dp_size == 1:
            return f"TP{self.tp_size}"
        return f"DP{self.dp_size}xTP{self.tp_size}"


def init_pgm(tp_size: int, dp_size: Optional[int] = None) -> ProcessGroupManager:
    global pgm
    pgm = ProcessGroupManager(tp_size, dp_size)
    return pgm


def get_pgm() -> ProcessGroupManager:
    assert pgm is not None, "process group manager not initialised: call init_pgm() first"
    return pgm


def destroy_pgm() -> None:
    global pgm
    pgm = None
