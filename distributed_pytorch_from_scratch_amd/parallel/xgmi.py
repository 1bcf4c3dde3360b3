"""Tensor-parallel collectives over xGMI peer memory (``csrc/comm/xgmi.hip``).

On an 8 x MI355X node every GPU has a direct xGMI link to each of its 7 peers.  RCCL (the
``nccl`` backend of ``torch.distributed``) is used for bootstrap, DP gradients and as the
fallback; the TP activation/gradient collectives of the training engine can instead run on
:class:`XgmiComm`, whose kernels read from all peers at once (two-shot all-reduce,
reduce-scatter, all-gather; see the kernel file for the protocol and its memory ordering).

Bootstrap: every rank allocates one IPC data buffer
``[in | tmp]`` and one signal buffer, the IPC handles are all-gathered over the TP group (the
c10d store / RCCL carries the bytes), and every rank maps its peers' buffers.  Calls are
issued on a dedicated HIP side stream with event hand-off to and from the caller's stream, so
they overlap compute exactly like an ``async_op=True`` RCCL call.

Reference parity: the reference's TP collectives are synchronous NCCL calls on the default
stream (``models/comm_ops.py:26,39,59,74``); this is the MI355X-native replacement of the
in-node transport, with identical semantics (sum / concatenate over the TP group).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import _ext

_ALL_REDUCE, _REDUCE_SCATTER, _ALL_GATHER, _ALL_REDUCE_1 = 0, 1, 2, 3
_NAMES = ("all_reduce", "reduce_scatter", "all_gather", "all_reduce")


class _Work:
    """``async_op`` handle: ``wait()`` makes the caller's current stream wait for the call."""

    __slots__ = ("event",)

    def __init__(self, event: torch.cuda.Event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)
        return True

    def is_completed(self) -> bool:
        return self.event.query()


class XgmiComm:
    """Peer-memory collectives for one TP group (every rank of the group on this node)."""

    def __init__(self, group=None, cap_bytes: Optional[int] = None, timeout_s: float = 120.0,
                 blocks: Optional[int] = None, nslots: Optional[int] = None):
        C = _ext.require()
        self.C = C
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        assert 1 < self.world <= 8, "xGMI collectives: 2..8 ranks of one node"
        cap = cap_bytes or int(os.environ.get("DPFS_XGMI_CAP_MB", "256")) * (1 << 20)
        self.cap = cap
        self.timeout_s = timeout_s
        self.nslots = 4 if nslots is None else nslots
        # Every step below is agreed on by the whole group, so a rank whose allocation or peer
        # mapping fails makes every rank raise together (tp_comm._build then drops xGMI on all
        # of them) instead of leaving the others blocked in the next collective.
        self.h, err = 0, ""
        try:
            self.h, handle = C.xgmi_create(self.rank, self.world, cap, self.nslots)
        except Exception as e:   # noqa: BLE001
            handle, err = b"", f"{type(e).__name__}: {e}"
        handles: List[Optional[bytes]] = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        if not all(handles):
            self._abort(f"xGMI buffers could not be allocated on every rank ({err or 'a peer failed'})")
        try:
            C.xgmi_open(self.h, b"".join(handles))
        except Exception as e:   # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        ok = torch.tensor([0.0 if err else 1.0], device="cuda" if dist.get_backend(group) == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        if ok.item() == 0:
            self._abort(f"xGMI peer buffers could not be mapped on every rank ({err or 'a peer failed'})")
        blocks = blocks or int(os.environ.get("DPFS_XGMI_BLOCKS", "32"))
        C.xgmi_set_blocks(self.h, blocks)
        self._blocks = blocks
        # per-op grid width (tp_comm picks one per op); None = the communicator default
        self.op_blocks = {"all_reduce": None, "reduce_scatter": None, "all_gather": None}
        # High-priority side stream: a collective that overlaps compute is the critical path
        # of the other chunk, so its (narrow) kernel should win the CU arbitration.
        self.stream = torch.cuda.Stream(priority=-1)
        dev = torch.device("cuda", torch.cuda.current_device())
        # Staging slots: producer GEMMs write their output straight into one (``staging``), so
        # the reduce-scatter / all-reduce of it skips the copy-in.
        self._slots = [C.xgmi_slot_tensor(self.h, i, cap, dev) for i in range(self.nslots)]
        self.one_shot_cap = int(C.xgmi_one_shot_capacity(self.h))
        dist.barrier(group=group)

    def _abort(self, why: str):
        if self.h:
            self.C.xgmi_destroy(self.h)
            self.h = 0
        raise RuntimeError(why)

    # ------------------------------------------------------------------------ core ----
    def staging(self, slot: int, shape, dtype: torch.dtype) -> Optional[torch.Tensor]:
        """A tensor of ``shape`` / ``dtype`` living in staging slot ``slot`` (None if it does
        not fit).  The caller owns the slot until the collective it feeds has been waited,
        and keeps one slot per in-flight chunk."""
        if not 0 <= slot < self.nslots:
            return None
        numel = 1
        for d in shape:
            numel *= d
        nbytes = numel * torch.empty((), dtype=dtype).element_size()
        if nbytes > self.cap or nbytes % 16:
            return None
        return self._slots[slot][:nbytes].view(dtype).view(*shape)

    def _slot_of(self, t: torch.Tensor) -> int:
        p = t.data_ptr()
        for i, sl in enumerate(self._slots):
            if sl.data_ptr() == p:
                return i
        return -1

    def _launch(self, op: int, x: torch.Tensor, out: torch.Tensor, timeout_s: Optional[float] = None,
                slot: int = -1):
        nb = self.op_blocks[_NAMES[op]]
        if nb is not None and nb != self._blocks:   # same call sequence on every rank
            self.set_blocks(nb)
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self.C.xgmi_run(self.h, op, x, out, self.world, timeout_s or self.timeout_s, slot)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        for t in (x, out):   # caching-allocator memory only (slots are the communicator's)
            if self._slot_of(t) < 0 and (t is x or t.data_ptr() != x.data_ptr()):
                t.record_stream(self.stream)
        return _Work(ev)

    def _max_elems(self, t: torch.Tensor) -> int:
        vec = 16 // t.element_size()
        per = self.cap // t.element_size()
        return (per // (self.world * vec)) * (self.world * vec)

    def one_shot_ok(self, t: torch.Tensor) -> bool:
        """Whether ``t`` can take the one-shot all-reduce (unstaged, within its capacity)."""
        nb = t.numel() * t.element_size()
        return 0 < nb <= self.one_shot_cap and nb % 16 == 0 and self._slot_of(t) < 0

    def all_reduce(self, t: torch.Tensor, async_op: bool = True, timeout_s: Optional[float] = None,
                   one_shot: bool = False):
        """In-place SUM over the group (bf16/fp32, fp32 accumulation in rank order, so every
        rank receives bitwise-identical values).  ``one_shot``: every rank reads every peer's
        whole message after ONE barrier (small messages; the same values as the two-shot form);
        falls back to two-shot where it does not apply."""
        assert t.is_contiguous()
        if one_shot and self.one_shot_ok(t):
            flat = t.view(-1)
            work = self._launch(_ALL_REDUCE_1, flat, flat, timeout_s)
            if not async_op:
                work.wait()
                return None
            return work
        slot = self._slot_of(t)
        if slot >= 0:                      # produced in a staging slot: no copy-in
            work = self._launch(_ALL_REDUCE, t.view(-1), t.view(-1), timeout_s, slot)
            if not async_op:
                work.wait()
                return None
            return work
        flat = t.view(-1)
        step = self._max_elems(t)
        work = None
        for o in range(0, flat.numel(), step):
            piece = flat[o: o + step]
            work = self._launch(_ALL_REDUCE, piece, piece, timeout_s)
        if not async_op:
            work.wait()
            return None
        return work

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = True,
                       timeout_s: Optional[float] = None):
        """out = (sum over ranks of inp)[rank-th of W equal slices] (same contract as
        ``dist.reduce_scatter_tensor``)."""
        assert inp.numel() == out.numel() * self.world and inp.numel() * inp.element_size() <= self.cap
        inp = inp.contiguous()
        work = self._launch(_REDUCE_SCATTER, inp, out, timeout_s, slot=self._slot_of(inp))
        if not async_op:
            work.wait()
            return None
        return work

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = True,
                   timeout_s: Optional[float] = None):
        """out = concat over ranks of inp (same contract as ``dist.all_gather_into_tensor``)."""
        assert out.numel() == inp.numel() * self.world and inp.numel() * inp.element_size() <= self.cap
        work = self._launch(_ALL_GATHER, inp.contiguous(), out, timeout_s)
        if not async_op:
            work.wait()
            return None
        return work

    def set_blocks(self, blocks: int):
        """Workgroups per collective launch (must be equal on every rank of the group)."""
        self.C.xgmi_set_blocks(self.h, int(blocks))
        self._blocks = int(blocks)

    # --------------------------------------------------------------------- health ----
    def error(self) -> int:
        """Non-zero once any barrier of any call timed out (host-mapped word, no sync)."""
        return int(self.C.xgmi_error(self.h))

    def clear_error(self):
        self.C.xgmi_clear_error(self.h)

    def check(self):
        if self.error():
            raise RuntimeError(f"xGMI collective timed out on TP rank {self.rank} (a peer never arrived)")

    def close(self):
        if self.h:
            torch.cuda.synchronize()
            dist.barrier(group=self.group)
            self.C.xgmi_destroy(self.h)
            self.h = 0
