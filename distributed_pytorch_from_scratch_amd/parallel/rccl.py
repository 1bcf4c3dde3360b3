"""Native RCCL communicator (``csrc/comm/rccl_comm.hip``): the RCCL C API on explicit streams.

SURVEY.md §5.1 item 2 ("an RcclComm wrapper issuing ncclAllReduce / ncclAllGather /
ncclReduceScatter / ncclBroadcast on explicit side HIP streams, with HIP events for
producer/consumer ordering").  Bootstrap: rank 0 of the group draws an ``ncclUniqueId``, the
c10d store carries it (``broadcast_object_list``), every rank calls ``ncclCommInitRank`` on its
own device.  Calls are enqueued on a high-priority side stream after an event hand-off from
the caller's stream and return a handle whose ``wait()`` makes the caller's stream wait —
the same contract as ``torch.distributed``'s ``async_op=True`` and :class:`~.xgmi.XgmiComm`,
without ProcessGroupNCCL's work objects or watchdog, and capturable in a HIP graph.

Reference parity: the reference's TP collectives (``models/comm_ops.py:26,39,59,74``) are
synchronous ProcessGroupNCCL calls on the default stream; :mod:`.tp_comm` can route the TP
group's collectives here (``DPFS_TP_COMM=native``, or ``auto`` when it measures faster).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..ops import _ext
from .xgmi import _Work

_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}


class RcclComm:
    """One RCCL communicator over the ranks of ``group`` (all on this process's device)."""

    def __init__(self, group=None, high_priority: bool = True):
        C = _ext.require()
        self.C = C
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        obj = [C.rccl_unique_id() if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=src, group=group)
        self.h = C.rccl_init(obj[0], self.world, self.rank)
        self.stream = torch.cuda.Stream(priority=-1 if high_priority else 0)

    def _run(self, fn, tensors, async_op: bool):
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            fn()
            ev = torch.cuda.Event()
            ev.record(self.stream)
        for t in tensors:
            t.record_stream(self.stream)
        work = _Work(ev)
        if not async_op:
            work.wait()
            return None
        return work

    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = True):
        """In place over the group."""
        assert t.is_contiguous()
        return self._run(lambda: self.C.rccl_all_reduce(self.h, t, t, _OPS[op]), (t,), async_op)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum", async_op: bool = True):
        """out = rank-th of ``world`` equal slices of the reduction of inp (``reduce_scatter_tensor``)."""
        inp = inp.contiguous()
        return self._run(lambda: self.C.rccl_reduce_scatter(self.h, out, inp, self.world, _OPS[op]), (out, inp),
                         async_op)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = True):
        """out = concatenation of inp over the group in rank order (``all_gather_into_tensor``)."""
        inp = inp.contiguous()
        return self._run(lambda: self.C.rccl_all_gather(self.h, out, inp, self.world), (out, inp), async_op)

    def broadcast(self, t: torch.Tensor, src: int = 0, async_op: bool = True):
        """``src`` is a rank of the group."""
        assert t.is_contiguous()
        return self._run(lambda: self.C.rccl_broadcast(self.h, t, src), (t,), async_op)

    def error(self) -> Optional[str]:
        """RCCL's asynchronous error of this communicator, if any."""
        e = self.C.rccl_async_error(self.h)
        return e or None

    def check(self):
        e = self.error()
        if e:
            raise RuntimeError(f"RCCL communicator (TP rank {self.rank}): {e}")

    def close(self):
        if self.h:
            torch.cuda.synchronize()
            self.C.rccl_destroy(self.h)
            self.h = 0
