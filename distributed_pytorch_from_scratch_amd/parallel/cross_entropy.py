"""Vocab-parallel cross-entropy (extension; north-star item).

The reference all-gathers the full ``(B, T, V)`` logits on every rank (``models/model.py:137``,
``comm_ops.py:68-75``) and runs a dense fp32 ``F.cross_entropy(ignore_index=-1)``
(``train.py:101-104``).  Here each rank keeps its ``(M, V/n)`` logit shard:

forward
    1. ``ce_fwd_stats`` kernel: one pass over the shard -> per-row ``[max, sum exp(x-max),
       target logit or 0]`` (M, 3) fp32.
    2. ONE ``all_gather_into_tensor`` of the (M, 3) stats over the TP group (12 B/token on the
       wire instead of ``V/n * 4`` B/token for the logits all-gather).
    3. each rank merges the n partial log-sum-exps locally -> ``lse``, ``loss = lse - tgt``.
backward
    ``ce_bwd`` kernel writes ``(softmax - onehot) * dloss`` *in place over the logits shard*
    (no extra ``(M, V/n)`` buffer), which then feeds the lm_head dgrad/wgrad GEMMs.

Padded vocab columns (e.g. GPT-2's 50257 padded to 50304) are excluded from the softmax.
Semantics match ``F.cross_entropy(reduction='mean', ignore_index=IGNORE_INDEX)``.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops.dispatch import K
from . import process_manager as pm

IGNORE_INDEX = -1


class VocabParallelCrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, vocab_start: int, vocab_valid: int, ignore_index: int,
                inplace_backward: bool):
        k = K(logits)
        x = logits.reshape(-1, logits.size(-1))
        t = targets.reshape(-1)
        stats = k.ce_fwd_stats(x, t, vocab_start, vocab_valid)  # (M, 3) fp32
        p = pm.pgm
        if p is not None and p.tp_size > 1:
            allst = stats.new_empty((p.tp_size * stats.size(0), 3))
            dist.all_gather_into_tensor(allst, stats.contiguous(), group=p.tp_group)
            allst = allst.view(p.tp_size, -1, 3)
        else:
            allst = stats.unsqueeze(0)
        mx = allst[..., 0].amax(0)
        se = (allst[..., 1] * torch.exp(allst[..., 0] - mx)).sum(0)
        lse = mx + torch.log(se)
        tl = allst[..., 2].sum(0)
        valid = t != ignore_index
        n_valid = valid.sum().clamp_min(1)
        losses = torch.where(valid, lse - tl, torch.zeros_like(lse))
        loss = losses.sum() / n_valid
        ctx.save_for_backward(x, t, lse, valid, n_valid)
        ctx.meta = (vocab_start, vocab_valid, inplace_backward, logits.shape)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, t, lse, valid, n_valid = ctx.saved_tensors
        vocab_start, vocab_valid, inplace, shp = ctx.meta
        gscale = valid.float() * (g.float() / n_valid.float())
        out = x if inplace else torch.empty_like(x)
        K(x).ce_bwd(x, t, lse, gscale, vocab_start, vocab_valid, out)
        return out.view(shp), None, None, None, None, None


def vocab_parallel_cross_entropy(logits_shard, targets, vocab_start: int, vocab_valid: int,
                                 ignore_index: int = IGNORE_INDEX, inplace_backward: bool = True):
    """Mean CE over non-ignored tokens from this rank's ``(..., V_local)`` logit shard.

    ``vocab_start`` is the global id of column 0 of the shard; ``vocab_valid`` is how many of
    the shard's columns are real vocabulary (``< V_local`` only on the rank owning padding).
    ``inplace_backward`` overwrites the saved logits with their gradient (only safe when
    nothing else reads the logits after the loss, as in training).
    """
    return VocabParallelCrossEntropyFn.apply(logits_shard, targets, vocab_start, vocab_valid,
                                             ignore_index, inplace_backward)
