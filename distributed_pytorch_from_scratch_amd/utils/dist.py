"""Distributed bootstrap, seeding and launch helpers.

Reference parity: ``utils.py:12-24`` (``set_seed``, ``init_dist_env``) and the ``mp.spawn``
launch model of ``train.py:151`` / ``test.py:172``.  Two launch styles are supported:

* ``spawn(fn, nprocs, args)`` — the reference's one-command launch (rank = spawn index =
  ``LOCAL_RANK`` = HIP device index);
* ``torchrun`` / ``python -m torch.distributed.run`` — ranks come from the environment.

The backend is RCCL (``"nccl"``) when a GPU is present and ``gloo`` otherwise (CPU plumbing).
``HSA_ENABLE_IPC_MODE_LEGACY=0`` is kept in the environment: the host driver only supports
dmabuf IPC, and RCCL's peer transport over xGMI needs it.
"""
from __future__ import annotations

import datetime
import os
import random
import socket
from argparse import Namespace
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..parallel import process_manager as pm


def set_seed(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def default_backend() -> str:
    return "nccl" if torch.cuda.is_available() else "gloo"


def init_dist_env(args: Optional[Namespace] = None, rank: Optional[int] = None, *,
                  tp_size: Optional[int] = None, dp_size: Optional[int] = None,
                  world_size: Optional[int] = None, backend: Optional[str] = None,
                  timeout_s: float = 600.0) -> pm.ProcessGroupManager:
    """Initialise ``torch.distributed`` + the process-group manager.

    ``init_dist_env(args, rank)`` mirrors the reference (``args.master_addr``,
    ``args.master_port``, ``args.tp_size``); with ``rank=None`` RANK/WORLD_SIZE/LOCAL_RANK are
    read from the environment (torchrun).
    """
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if args is not None:
        if getattr(args, "master_addr", None):
            os.environ["MASTER_ADDR"] = str(args.master_addr)
        if getattr(args, "master_port", None):
            os.environ["MASTER_PORT"] = str(args.master_port)
        tp_size = tp_size or getattr(args, "tp_size", None)
        dp_size = dp_size or getattr(args, "dp_size", None)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
        world_size = int(os.environ.get("WORLD_SIZE", "1"))
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    else:
        if world_size is None:
            world_size = (tp_size or 1) * (dp_size or 1)
        local_rank = rank
        os.environ["RANK"] = str(rank)
        os.environ["LOCAL_RANK"] = str(rank)
        os.environ["WORLD_SIZE"] = str(world_size)
    # DPFS_BACKEND=gloo: several ranks on one GPU (rehearsal of a multi-GPU launch on a
    # single device; the TP collectives can still run on the xGMI kernels, DPFS_TP_COMM=xgmi).
    backend = backend or os.environ.get("DPFS_BACKEND") or default_backend()
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        kw["device_id"] = torch.device("cuda", local_rank)
        # RCCL collectives on a high-priority HIP stream: they overlap the other ping-pong
        # chunk's compute and are on its critical path.
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        # the timeout is the init_process_group kwarg; the options object carries the same value
        # (torch warns whenever the two differ, and Options() defaults to its own)
        opts._timeout = datetime.timedelta(seconds=timeout_s)
        kw["pg_options"] = opts
    elif os.environ.get("DPFS_BACKEND") == "gloo" and torch.cuda.is_available():
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
    if not dist.is_initialized():
        dist.init_process_group(backend=backend, init_method="env://", world_size=world_size,
                                rank=rank, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    tp_size = tp_size or world_size
    return pm.init_pgm(tp_size, dp_size)


def destroy_dist_env() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
    pm.destroy_pgm()


def spawn(fn: Callable, nprocs: int, args=()):
    """``mp.spawn`` with a fresh rendezvous port (reference launch model)."""
    import torch.multiprocessing as mp
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(free_port()))
    mp.spawn(fn, args=args, nprocs=nprocs, join=True)


def device_for_rank() -> torch.device:
    if torch.cuda.is_available() and dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")
