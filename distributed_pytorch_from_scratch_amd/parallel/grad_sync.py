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


def dp_bucket_bytes(group, device) -> int:
    """DP bucket size of the fused engines: ``DPFS_DP_BUCKET_MB`` = a number of MB (0: every
    gradient group is its own all-reduce, the pre-bucketing behaviour), or ``auto`` (default on
    RCCL: ``measure_bucket_knee`` once per group; on gloo 0)."""
    key = id(group)
    if key in _BUCKET_CACHE:
        return _BUCKET_CACHE[key]
    env = os.environ.get("DPFS_DP_BUCKET_MB", "auto").strip().lower()
    if env == "auto":
        nb = measure_bucket_knee(group, device) if dist.get_backend(group) == "nccl" else 0
    else:
        nb = int(float(env) * 2 ** 20)
    _BUCKET_CACHE[key] = nb
    return nb


class DPBucketer:
    """The fused engines' DP gradient averaging: gradient groups (a dict of fp32 tensors and the
    keys to reduce) are queued as the backward completes them and launched as ONE async
    all-reduce of a flat buffer once the queued bytes reach ``bucket_bytes`` (0: every group at
    once); ``finish`` launches the rest, waits, averages and writes the values back into the
    dicts (the flat buffer's views replace the tensors).  ``before_pack`` runs before a bucket
    is packed (the engines flush their deferred gradient sums there)."""

    def __init__(self, group, dp: int, bucket_bytes: int, before_pack: Optional[Callable[[], None]] = None):
        self.group, self.dp, self.bucket_bytes, self.before_pack = group, dp, bucket_bytes, before_pack
        self._queued: List[tuple] = []
        self._bytes = 0
        self._pending: List[tuple] = []
        self.launches = 0

    def add(self, d: dict, keys=None) -> None:
        if self.dp <= 1:
            return
        keys = [k for k in (keys or sorted(d)) if d.get(k) is not None]
        if not keys:
            return
        self._queued.append((d, keys))
        self._bytes += sum(d[k].numel() * 4 for k in keys)
        if self._bytes >= self.bucket_bytes:
            self._launch()

    def _launch(self) -> None:
        if not self._queued:
            return
        if self.before_pack is not None:
            self.before_pack()
        flat = torch.cat([d[k].reshape(-1).float() for d, keys in self._queued for k in keys])
        h = dist.all_reduce(flat, group=self.group, async_op=True)
        self._pending.append((h, flat, self._queued))
        self._queued, self._bytes = [], 0
        self.launches += 1

    def finish(self) -> bool:
        """Launch what is queued, wait for every bucket, average; True if anything was reduced."""
        self._launch()
        done = bool(self._pending)
        for h, flat, groups in self._pending:
            h.wait()
            flat /= self.dp
            off = 0
            for d, keys in groups:
                for k in keys:
                    n = d[k].numel()
                    d[k] = flat[off:off + n].view_as(d[k])
                    off += n
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


def allreduce_sequence_parallel_grads(model: torch.nn.Module) -> None:
    p = pm.pgm
    if p is None or p.tp_size == 1:
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
