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

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import process_manager as pm


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
