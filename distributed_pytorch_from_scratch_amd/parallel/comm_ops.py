"""Autograd collectives over the tensor-parallel group.

Reference parity: ``models/comm_ops.py:7-83`` — the four Megatron conjugate pairs

=========  ===========================================  ==========================================
op         forward                                      backward
=========  ===========================================  ==========================================
Split      keep this rank's slice of the last dim       all-gather along the last dim
Reduce     all-reduce(SUM)                              identity
Copy       identity                                     all-reduce(SUM)
Gather     all-gather along the last dim                keep this rank's slice
=========  ===========================================  ==========================================

plus the sequence-parallel pair (not in the reference; Megatron-SP): ``ScatterSeq`` /
``GatherSeq`` (reduce-scatter / all-gather along dim 0 of a ``(tokens, hidden)`` tensor).

Design differences from the reference (MI355X-first):

* Collectives run on RCCL (``torch.distributed`` backend ``nccl`` on ROCm) on the
  process group's own HIP stream; ``Gather`` writes straight into one contiguous output
  with ``all_gather_into_tensor`` instead of ``tp_size`` temporary tensors + ``torch.cat``
  (``comm_ops.py:72-75`` allocates n zero tensors per call).
* ``Reduce.forward`` reduces a *fresh* GEMM output, so it is done in place (as the
  reference); ``Copy.backward`` clones-free too because autograd hands it a gradient
  buffer it owns.
* Uneven shards are supported (``sizes=``) for the head-partitioned layers (GPT-2 small has
  12 heads; TP=8 gives 2 heads to ranks 0-3 and 1 head to ranks 4-7).
* Every entry is a no-op at ``tp_size == 1`` (``comm_ops.py:13,23,37,57,70,79``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from . import process_manager as pm
from . import tp_comm


def _tp():
    p = pm.get_pgm()
    return p.tp_size, p.tp_rank, p.tp_group


def _even_sizes(total: int, n: int) -> List[int]:
    assert total % n == 0, f"dim {total} not divisible by tp_size {n}"
    return [total // n] * n


def all_gather_last_dim(x: torch.Tensor, sizes: Optional[Sequence[int]] = None) -> torch.Tensor:
    """All-gather ``x`` (this rank's ``(..., sizes[r])`` slice) into ``(..., sum(sizes))``."""
    n, r, group = _tp()
    if n == 1:
        return x
    x = x.contiguous()
    if sizes is None or len(set(sizes)) == 1:
        # Gather rank-major into one buffer (one RCCL call), then move the rank axis next to
        # the last dim: (n, ..., d) -> (..., n, d) -> (..., n*d).
        out = x.new_empty((n * x.size(0),) + tuple(x.shape[1:]))
        dist.all_gather_into_tensor(out, x, group=group)
        return out.view((n,) + tuple(x.shape)).movedim(0, -2).reshape(*x.shape[:-1], n * x.shape[-1])
    # Uneven shards: pad every shard to the largest size, one all_gather_into_tensor (RCCL and
    # gloo both require equal sizes), then drop the padding.
    mx = max(sizes)
    if x.size(-1) < mx:
        x = torch.nn.functional.pad(x, (0, mx - x.size(-1)))
    x2 = x.reshape(-1, mx).contiguous()
    out = x2.new_empty((n * x2.size(0), mx))
    dist.all_gather_into_tensor(out, x2, group=group)
    out = out.view(n, -1, mx)
    parts = [out[i, :, :sizes[i]] for i in range(n)]
    return torch.cat(parts, dim=-1).view(*x.shape[:-1], sum(sizes))


def slice_last_dim(x: torch.Tensor, sizes: Optional[Sequence[int]] = None) -> torch.Tensor:
    n, r, _ = _tp()
    if n == 1:
        return x
    if sizes is None:
        sizes = _even_sizes(x.size(-1), n)
    st = sum(sizes[:r])
    return x[..., st:st + sizes[r]].contiguous()


def all_reduce_(x: torch.Tensor, async_op: bool = False):
    n, _, group = _tp()
    if n == 1:
        return None
    return tp_comm.all_reduce(x, async_op=async_op)


class Split(torch.autograd.Function):
    """fwd: this rank's slice of the last dim; bwd: all-gather (``comm_ops.py:7-28``)."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, sizes: Optional[Sequence[int]] = None) -> torch.Tensor:
        ctx.sizes = sizes
        return slice_last_dim(x, sizes)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        return all_gather_last_dim(g, ctx.sizes), None


class Reduce(torch.autograd.Function):
    """fwd: all-reduce(SUM) in place; bwd: identity (``comm_ops.py:31-44``)."""

    @staticmethod
    def forward(ctx, x: torch.Tensor) -> torch.Tensor:
        all_reduce_(x)
        return x

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        return g


class Copy(torch.autograd.Function):
    """fwd: identity; bwd: all-reduce(SUM) (``comm_ops.py:47-60``)."""

    @staticmethod
    def forward(ctx, x: torch.Tensor) -> torch.Tensor:
        return x

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        g = g.contiguous()
        all_reduce_(g)
        return g


class Gather(torch.autograd.Function):
    """fwd: all-gather along the last dim; bwd: keep this rank's slice (``comm_ops.py:63-83``)."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, sizes: Optional[Sequence[int]] = None) -> torch.Tensor:
        ctx.sizes = sizes
        return all_gather_last_dim(x, sizes)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        return slice_last_dim(g, ctx.sizes), None


# ----------------------------------------------------------------------------------------
# Sequence-parallel pair (extension): rows = tokens, sharded over the TP group.
# ----------------------------------------------------------------------------------------

def reduce_scatter_rows(x: torch.Tensor) -> torch.Tensor:
    n, _, group = _tp()
    if n == 1:
        return x
    x = x.contiguous()
    assert x.size(0) % n == 0, f"rows {x.size(0)} not divisible by tp_size {n}"
    out = x.new_empty((x.size(0) // n,) + tuple(x.shape[1:]))
    tp_comm.reduce_scatter(out, x, async_op=False)
    return out


def all_gather_rows(x: torch.Tensor, async_op: bool = False):
    n, _, group = _tp()
    if n == 1:
        return (x, None) if async_op else x
    x = x.contiguous()
    out = x.new_empty((x.size(0) * n,) + tuple(x.shape[1:]))
    h = tp_comm.all_gather(out, x, async_op=async_op)
    return (out, h) if async_op else out


class ScatterSeq(torch.autograd.Function):
    """fwd: reduce-scatter rows (sum partials, keep my token slice); bwd: all-gather rows."""

    @staticmethod
    def forward(ctx, x: torch.Tensor) -> torch.Tensor:
        return reduce_scatter_rows(x)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        return all_gather_rows(g)


class GatherSeq(torch.autograd.Function):
    """fwd: all-gather rows; bwd: reduce-scatter rows."""

    @staticmethod
    def forward(ctx, x: torch.Tensor) -> torch.Tensor:
        return all_gather_rows(x)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        return reduce_scatter_rows(g)
