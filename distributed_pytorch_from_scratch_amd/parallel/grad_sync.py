"""Gradient synchronisation outside the TP autograd collectives.

* ``allreduce_sequence_parallel_grads``: under sequence parallelism every rank computes the
  grads of replicated parameters (norm scales, row-parallel biases) from its *own token
  shard*, so they must be summed over the TP group.  Without SP the grads are identical on
  every TP rank by construction (deterministic kernels on identical inputs, SURVEY.md §7.5
  item 4) and no communication is needed.
* ``DataParallelGradSync``: bucketed gradient all-reduce over the DP group (extension — the
  reference has no DP).  Gradients are packed into flat fp32 buckets of ``bucket_mb`` and
  reduced with ``async_op=True`` as soon as a bucket is complete during backward (hooked on
  ``post_accumulate_grad``), so RCCL traffic overlaps the remaining backward GEMMs.  On an
  8-GPU xGMI node a ring all-reduce is bound by one link per GPU; ~25-64 MB buckets keep
  every ring step in the bandwidth regime while leaving enough buckets to overlap.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

from . import process_manager as pm

# ---------------------------------------------------------------- bucket size for DP all-reduce
# A ring all-reduce over the 8-GPU xGMI mesh moves 2 (W-1)/W of the message per GPU in W-1
# steps over one link per direction; below some size each step is latency-bound and the bus
# rate collapses.  ``dp_bucket_bytes`` picks the bucket as the smallest message that reaches
# ``DP_BUCKET_FRACTION`` of the best measured bus rate on the live DP group (the knee of the
# curve on this node, RCCL protocol and channel count included), so the fused engines merge
# small per-layer gradient groups (e.g. at TP 8, ~3.5 MB per GPT-2-small layer and rank) into
# buckets that run at link speed, while large groups still start as soon as they are complete.
DP_BUCKET_SIZES_MB = (1, 2, 4, 8, 16, 32, 64)
DP_BUCKET_FRACTION = 0.85
_BUCKET_CACHE: Dict[int, int] = {}


def measure_bucket_knee(group, device, sizes_mb=DP_BUCKET_SIZES_MB, frac: float = DP_BUCKET_FRACTION,
                        reps: int = 3) -> int:
    """Bytes of the smallest all-reduce message whose bus rate (max time over the group's ranks)
    is within ``frac`` of the best of ``sizes_mb``.  Every rank returns the same value (the
    times are MAX-reduced before the choice)."""
    cuda = device.type == "cuda"
    times = []
    for mb in sizes_mb:
        buf = torch.zeros(int(mb * 2 ** 20) // 4, dtype=torch.float32, device=device)
        dist.all_reduce(buf, group=group)                 # warm the protocol / channels
        if cuda:
            torch.cuda.synchronize(device)
        dist.barrier(group=group)
        if cuda:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                dist.all_reduce(buf, group=group)
            e.record()
            e.synchronize()
            ms = s.elapsed_time(e) / reps
        else:
            import time
            t0 = time.perf_counter()
            for _ in range(reps):
                dist.all_reduce(buf, group=group)
            ms = (time.perf_counter() - t0) * 1e3 / reps
        times.append(ms)
    t = torch.tensor(times, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    rates = [mb / max(ms, 1e-9) for mb, ms in zip(sizes_mb, t.tolist())]
    best = max(rates)
    for mb, r in zip(sizes_mb, rates):
        if r >= frac * best:
            return int(mb * 2 ** 20)
    return int(sizes_mb[-1] * 2 ** 20)


def _bucket_env() -> Optional[float]:
    """``DPFS_DP_BUCKET_MB``: None = auto, else MB (validated here, outside any autograd pass)."""
    env = os.environ.get("DPFS_DP_BUCKET_MB", "auto").strip().lower()
    if env == "auto":
        return None
    try:
        mb = float(env)
    except ValueError:
        raise ValueError(f"DPFS_DP_BUCKET_MB must be 'auto' or a number of MB, got {env!r}") from None
    if mb < 0:
        raise ValueError(f"DPFS_DP_BUCKET_MB must be >= 0, got {mb}")
    return mb


def dp_bucket_bytes(group, device, world_max: bool = False) -> int:
    """DP bucket size of the fused engines: ``DPFS_DP_BUCKET_MB`` = a number of MB (0: every
    gradient group is its own all-reduce, the pre-bucketing behaviour), or ``auto`` (default on
    RCCL: ``measure_bucket_knee`` once per group; on gloo 0).  ``world_max``: the value is
    MAX-reduced over the default (WORLD) group, so every DP group of a TP x DP grid uses one
    size -- every rank must call it then (``setup_dp_buckets``, at step construction)."""
    key = id(group)
    if key in _BUCKET_CACHE:
        return _BUCKET_CACHE[key]
    mb = _bucket_env()
    if mb is None:
        nb = measure_bucket_knee(group, device) if dist.get_backend(group) == "nccl" else 0
    else:
        nb = int(mb * 2 ** 20)
    if world_max and dist.get_world_size() > 1:
        t = torch.tensor([float(nb)], dtype=torch.float64,
                         device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        nb = int(t.item())
    _BUCKET_CACHE[key] = nb
    return nb


def setup_dp_buckets(device) -> None:
    """Measure (or read) the DP bucket size once at step construction, outside the backward,
    on every rank (MAX over the WORLD group)."""
    p = pm.pgm
    if p is not None and p.dp_size > 1:
        dp_bucket_bytes(p.dp_group, device, world_max=True)


def reset() -> None:
    """Forget the cached bucket sizes (a new process-group layout)."""
    _BUCKET_CACHE.clear()


class GradArena:
    """One flat fp32 buffer holding every gradient of the fused engines' step, laid out in the
    order the backward completes them (``groups``: a list of (group name, [(key, param), ...])).

    The engines write each gradient straight into its view (the weight-gradient GEMMs, the bias /
    norm / embedding reductions take it as their output; later ping-pong chunks accumulate into
    it), the parameters' ``.grad`` become those views, and a DP bucket is a contiguous range of
    the buffer: the data-parallel all-reduce runs on it in place -- no pack, no copy back.  The
    buffer lives with the model (allocated once), so the previous step's gradients and this
    step's share the same 4 bytes per parameter (utils/memory.py)."""

    def __init__(self, groups, device):
        self.order = [name for name, _ in groups]
        self.ranges: Dict[str, tuple] = {}
        self.slots: Dict[tuple, tuple] = {}       # (group, key) -> (offset, shape)
        off = 0
        for name, items in groups:
            start = off
            for key, p in items:
                if p is None:
                    continue
                # a tuple key names the slot explicitly: (group, key) of another group whose
                # gradient is stored in this group's range (the SP replicated gradients)
                self.slots[key if isinstance(key, tuple) else (name, key)] = (off, tuple(p.shape))
                off += p.numel()
            self.ranges[name] = (start, off)
        self.numel = off
        self.buf = torch.empty(off, dtype=torch.float32, device=device)
        self.signature = None

    def view(self, name, key) -> Optional[torch.Tensor]:
        s = self.slots.get((name, key))
        if s is None:
            return None
        off, shape = s
        n = 1
        for d in shape:
            n *= d
        return self.buf[off:off + n].view(shape)


def arena_for(model, groups, tag: str) -> GradArena:
    """The model's gradient arena for this engine layout (``tag``), rebuilt when a parameter is
    replaced, moved or resized."""
    sig = (tag,) + tuple((name, key, id(p), tuple(p.shape), str(p.device)) for name, items in groups
                         for key, p in items if p is not None)
    a = getattr(model, "_dpfs_grad_arena", None)
    if a is None or a.signature != sig:
        dev = next(p for _, items in groups for _, p in items if p is not None).device
        a = GradArena(groups, dev)
        a.signature = sig
        model._dpfs_grad_arena = a
    return a


class DPBucketer:
    """The fused engines' DP gradient averaging over a :class:`GradArena`: gradient groups are
    marked complete (``add(name)``) in arena order as the backward finishes them, and a bucket
    -- the contiguous range of completed groups -- goes out as ONE async all-reduce of that slice
    of the arena, in place, once it holds ``bucket_bytes`` (0: every group at once).  ``finish``
    launches the rest, waits and averages in place.  ``before_launch`` runs before a bucket is
    launched (the engines flush their deferred gradient sums there)."""

    def __init__(self, arena: Optional[GradArena], group, dp: int, bucket_bytes: int,
                 before_launch: Optional[Callable[[], None]] = None):
        self.arena, self.group, self.dp, self.bucket_bytes = arena, group, dp, bucket_bytes
        self.before_launch = before_launch
        self._lo = self._hi = None
        self._pending: List[tuple] = []
        self.launches = 0

    def add(self, name: str) -> None:
        if self.dp <= 1 or self.arena is None:
            return
        a, b = self.arena.ranges[name]
        if b == a:
            return
        if self._hi is not None and a != self._hi:    # not adjacent to the open bucket: close it
            self._launch()
        if self._lo is None:
            self._lo = a
        self._hi = b
        if 4 * (self._hi - self._lo) >= self.bucket_bytes:
            self._launch()

    def _launch(self) -> None:
        if self._lo is None or self._hi == self._lo:
            self._lo = self._hi = None
            return
        if self.before_launch is not None:
            self.before_launch()
        sl = self.arena.buf[self._lo:self._hi]
        # RCCL averages in the collective (ncclAvg): no separate pass over the gradients;
        # gloo has no AVG, so it sums and the bucket is divided after the wait
        avg = _has_avg(self.group)
        h = dist.all_reduce(sl, op=dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM, group=self.group,
                            async_op=True)
        self._pending.append((h, sl, avg))
        self._lo = self._hi = None
        self.launches += 1

    def finish(self) -> bool:
        """Launch what is open, wait for every bucket, average in place; True if anything was
        reduced."""
        self._launch()
        done = bool(self._pending)
        for h, sl, avg in self._pending:
            h.wait()
            if not avg:
                sl.div_(self.dp)
        self._pending = []
        return done


def _flat_allreduce(tensors: List[torch.Tensor], group, average_by: int = 1) -> None:
    if not tensors:
        return
    flat = torch.cat([t.reshape(-1).float() for t in tensors])
    dist.all_reduce(flat, group=group)
    if average_by > 1:
        flat /= average_by
    # one multi-tensor copy back (per-tensor copy_ calls cost a launch + stream hand-off each)
    parts = flat.split([t.numel() for t in tensors])
    torch._foreach_copy_(tensors, [q.view_as(t) for q, t in zip(parts, tensors)])


def _has_avg(group) -> bool:
    """``ReduceOp.AVG`` exists on the NCCL (= RCCL) backend only."""
    try:
        return dist.get_backend(group) == "nccl"
    except Exception:
        return False


def allreduce_sequence_parallel_grads(model: torch.nn.Module) -> None:
    p = pm.pgm
    if p is None or p.tp_size == 1:
        return
    a = getattr(model, "_dpfs_grad_arena", None)
    if a is not None and "sprep" in a.ranges:
        # the SP fused engine keeps every replicated gradient in one contiguous arena range
        # ("sprep", fused_engine.arena_groups): one in-place all-reduce, no pack / copy back
        lo, hi = a.ranges["sprep"]
        rep = [q for q in model.parameters() if getattr(q, "sequence_parallel_grad", False) and q.grad is not None]
        base, end = a.buf.data_ptr(), a.buf.data_ptr() + 4 * a.numel
        if rep and all(base + 4 * lo <= q.grad.data_ptr() < base + 4 * hi for q in rep):
            if hi > lo:
                dist.all_reduce(a.buf[lo:hi], group=p.tp_group)
            return
    grads = [q.grad for q in model.parameters()
             if getattr(q, "sequence_parallel_grad", False) and q.grad is not None]
    _flat_allreduce(grads, p.tp_group)


class DataParallelGradSync:
    """Overlapped, bucketed DP gradient averaging (no-op when ``dp_size == 1``)."""

    def __init__(self, model: torch.nn.Module, bucket_mb: float = 32.0):
        self.model = model
        self.p = pm.get_pgm()
        self.params = [q for q in model.parameters() if q.requires_grad]
        self.enabled = self.p.dp_size > 1
        self.bucket_bytes = int(bucket_mb * 2 ** 20)
        self._buckets: List[List[torch.nn.Parameter]] = []
        self._index: Dict[int, int] = {}
        self._pending: Dict[int, int] = {}
        self._handles = []
        if not self.enabled:
            return
        # Reverse order ~ order in which grads become ready in backward.
        cur, size = [], 0
        for q in reversed(self.params):
            cur.append(q)
            size += q.numel() * 4
            if size >= self.bucket_bytes:
                self._buckets.append(cur)
                cur, size = [], 0
        if cur:
            self._buckets.append(cur)
        for bi, b in enumerate(self._buckets):
            for q in b:
                self._index[id(q)] = bi
                q.register_post_accumulate_grad_hook(self._hook)
        self._reset()

    def _reset(self):
        self._pending = {i: len(b) for i, b in enumerate(self._buckets)}
        self._flat = {}

    def _hook(self, param):
        if getattr(self.model, "_dpfs_dp_reduced", False):
            return   # the fused engine already averaged this step's grads (overlapped)
        bi = self._index[id(param)]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            b = self._buckets[bi]
            flat = torch.cat([q.grad.reshape(-1).float() for q in b])
            h = dist.all_reduce(flat, group=self.p.dp_group, async_op=True)
            self._handles.append((h, bi, flat))

    def finish(self) -> None:
        """Wait for all buckets (call after backward, before the optimizer step)."""
        if not self.enabled:
            return
        if getattr(self.model, "_dpfs_dp_reduced", False):
            self.model._dpfs_dp_reduced = False
            self._handles = []
            self._reset()
            return
        # Buckets whose params got no grad this step are reduced here synchronously.
        for bi, n in self._pending.items():
            if 0 < n:
                b = [q for q in self._buckets[bi] if q.grad is not None]
                _flat_allreduce(b and [q.grad for q in b], self.p.dp_group)
                for q in b:
                    q.grad /= self.p.dp_size
        for h, bi, flat in self._handles:
            h.wait()
            flat /= self.p.dp_size
            off = 0
            for q in self._buckets[bi]:
                n = q.numel()
                q.grad.copy_(flat[off:off + n].view_as(q.grad))
                off += n
        self._handles = []
        self._reset()
