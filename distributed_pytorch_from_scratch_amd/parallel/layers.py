"""Tensor-parallel layers.

Reference parity (``models/layers.py``):

* ``RowParallelLinear``            ``layers.py:14-55``   weight ``(odim, idim/n)``, bias replicated
* ``ColumnParallelLinear``         ``layers.py:58-100``  weight ``(odim/n, idim)``, bias sharded
* ``ParallelVocabularyEmbedding``  ``layers.py:103-141`` rows ``[vocab_st_idx, vocab_ed_idx)``
* ``RMSNorm``                      ``layers.py:145-155`` replicated, ``scale`` init to ones

Same constructor signatures, attribute names (``odim_partition``, ``idim_partition``,
``vocab_st_idx``, ``vocab_ed_idx``, ``add_bias``) and ``reset_parameters()`` semantics: every
sharded weight is initialised as the *full* matrix with the reference initialiser
(``kaiming_uniform_(a=sqrt(5))`` / ``normal_(0, 1)``), broadcast from rank 0 and sliced, so a
TP=k model is bit-identical at init to TP=1 under the same seed.

Fixed reference bugs (``SURVEY.md`` §2.7): the embedding does not mutate the caller's ids, and
non-divisible vocab sizes work (the init split uses the same ``[st, ed)`` ranges as the
forward).  Extensions: uneven shard sizes (``partition_sizes``) so e.g. 12 heads shard over 8
ranks, fused multi-output column layers (``FusedColumnParallelLinear``: QKV and gate|up in
one GEMM) that still save/load reference state-dict keys, ``LayerNorm``, sequence parallel.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import functional as Fn
from ..ops.dispatch import K
from . import comm_ops
from . import process_manager as pm
from .linear_fn import column_parallel_linear, row_parallel_linear


# ------------------------------------------------------------------------ helpers ----

def partition_sizes(total: int, n: int, granule: int = 1) -> List[int]:
    """Split ``total`` (a multiple of ``granule``) over ``n`` ranks as evenly as possible in
    units of ``granule``; the first ``units % n`` ranks get one extra unit."""
    assert total % granule == 0
    units = total // granule
    assert units >= n, f"cannot shard {units} units of {granule} over {n} ranks"
    base, extra = divmod(units, n)
    return [(base + (1 if r < extra else 0)) * granule for r in range(n)]


def _offsets(sizes: Sequence[int]) -> List[int]:
    out, acc = [], 0
    for s in sizes:
        out.append(acc)
        acc += s
    return out


@torch.no_grad()
def _full_init_then_shard(shape: Tuple[int, int], init: str, device, dtype, dim: int,
                          start: int, size: int) -> torch.Tensor:
    """Materialise the full matrix with the reference initialiser, make every rank agree
    (broadcast from global rank 0, as ``layers.py:38,83,116``), return rows/cols
    ``[start, start+size)`` along ``dim``."""
    full = torch.empty(shape, device=device, dtype=dtype)
    if init == "kaiming":
        nn.init.kaiming_uniform_(full, a=math.sqrt(5))
    elif init == "normal":
        nn.init.normal_(full, mean=0.0, std=1.0)
    else:
        raise ValueError(init)
    p = pm.pgm
    if p is not None and p.world_size > 1:
        dist.broadcast(full, src=0)
    return full.narrow(dim, start, size).contiguous()


def _tp_size_rank():
    p = pm.pgm
    if p is None:
        return 1, 0
    return p.tp_size, p.tp_rank


# --------------------------------------------------------------------------- linear ----

class ColumnParallelLinear(nn.Module):
    """``(..., idim) -> (..., odim/n)`` (or gathered ``(..., odim)``)."""

    def __init__(self, idim: int, odim: int, add_bias: bool = True, gather_output: bool = True,
                 sizes: Optional[Sequence[int]] = None, sequence_parallel: bool = False):
        super().__init__()
        n, r = _tp_size_rank()
        self.idim, self.odim = idim, odim
        self.gather_output = gather_output
        self.sequence_parallel = sequence_parallel
        if sizes is None:
            assert odim % n == 0, f"odim {odim} not divisible by tp_size {n}"
            sizes = [odim // n] * n
        assert sum(sizes) == odim and len(sizes) == n
        self.sizes = list(sizes)
        self.odim_partition = self.sizes[r]
        self.odim_start = sum(self.sizes[:r])
        self.weight = nn.Parameter(torch.empty(self.odim_partition, idim))
        self.add_bias = add_bias
        if add_bias:
            self.bias = nn.Parameter(torch.empty(self.odim_partition))
        else:
            self.register_parameter("bias", None)

    @torch.no_grad()
    def reset_parameters(self):
        w = _full_init_then_shard((self.odim, self.idim), "kaiming", self.weight.device,
                                  self.weight.dtype, 0, self.odim_start, self.odim_partition)
        self.weight.copy_(w)
        if self.add_bias:
            nn.init.zeros_(self.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = column_parallel_linear(x, self.weight, self.bias, self.sequence_parallel, True)
        if self.gather_output:
            y = comm_ops.Gather.apply(y, self.sizes)
        return y


class RowParallelLinear(nn.Module):
    """``(..., idim)`` (or pre-split ``(..., idim/n)``) -> ``(..., odim)`` summed over ranks."""

    def __init__(self, idim: int, odim: int, add_bias: bool = True, split_input: bool = True,
                 sizes: Optional[Sequence[int]] = None, sequence_parallel: bool = False):
        super().__init__()
        n, r = _tp_size_rank()
        self.idim, self.odim = idim, odim
        self.split_input = split_input
        self.sequence_parallel = sequence_parallel
        if sizes is None:
            assert idim % n == 0, f"idim {idim} not divisible by tp_size {n}"
            sizes = [idim // n] * n
        assert sum(sizes) == idim and len(sizes) == n
        self.sizes = list(sizes)
        self.idim_partition = self.sizes[r]
        self.idim_start = sum(self.sizes[:r])
        self.weight = nn.Parameter(torch.empty(odim, self.idim_partition))
        self.add_bias = add_bias
        if add_bias:
            self.bias = nn.Parameter(torch.empty(odim))
            # Replicated parameter whose grad is only rank-local under sequence parallelism.
            self.bias.sequence_parallel_grad = sequence_parallel
        else:
            self.register_parameter("bias", None)

    @torch.no_grad()
    def reset_parameters(self):
        w = _full_init_then_shard((self.odim, self.idim), "kaiming", self.weight.device,
                                  self.weight.dtype, 1, self.idim_start, self.idim_partition)
        self.weight.copy_(w)
        if self.add_bias:
            nn.init.zeros_(self.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.split_input:
            x = comm_ops.Split.apply(x, self.sizes)
        return row_parallel_linear(x, self.weight, self.bias, self.sequence_parallel, True)


class FusedColumnParallelLinear(nn.Module):
    """Several column-parallel projections of the same input in ONE GEMM.

    ``odims=[d, d, d]`` with ``names=['wq', 'wk', 'wv']`` stores this rank's shards
    ``[Wq_r; Wk_r; Wv_r]`` as one ``(sum_i odim_i/n, idim)`` weight.  ``state_dict`` /
    ``load_state_dict`` go through hooks that present the reference layout
    (``<parent>.wq.weight``, ``<parent>.wq.bias``, ...), so checkpoints interoperate with the
    reference's per-rank files (``train.py:121-126``, ``SURVEY.md`` §2.6).  One GEMM instead of
    three also means one dgrad all-reduce instead of three (``SURVEY.md`` §5.1 item 4).
    """

    def __init__(self, idim: int, odims: Sequence[int], names: Sequence[str], add_bias: bool = True,
                 sizes: Optional[Sequence[Sequence[int]]] = None, sequence_parallel: bool = False):
        super().__init__()
        n, r = _tp_size_rank()
        assert len(odims) == len(names)
        self.idim, self.odims, self.names = idim, list(odims), list(names)
        self.sequence_parallel = sequence_parallel
        if sizes is None:
            sizes = []
            for o in odims:
                assert o % n == 0, f"odim {o} not divisible by tp_size {n}"
                sizes.append([o // n] * n)
        self.sizes = [list(s) for s in sizes]
        self.local = [s[r] for s in self.sizes]
        self.starts = [sum(s[:r]) for s in self.sizes]
        self.local_offsets = _offsets(self.local)
        self.odim_partition = sum(self.local)
        self.weight = nn.Parameter(torch.empty(self.odim_partition, idim))
        self.add_bias = add_bias
        if add_bias:
            self.bias = nn.Parameter(torch.empty(self.odim_partition))
        else:
            self.register_parameter("bias", None)
        self._register_state_dict_hook(FusedColumnParallelLinear._sd_hook)

    @torch.no_grad()
    def reset_parameters(self):
        # Same RNG consumption order as the reference's separate modules (wq, wk, wv).
        for i, o in enumerate(self.odims):
            w = _full_init_then_shard((o, self.idim), "kaiming", self.weight.device,
                                      self.weight.dtype, 0, self.starts[i], self.local[i])
            self.weight[self.local_offsets[i]:self.local_offsets[i] + self.local[i]].copy_(w)
        if self.add_bias:
            nn.init.zeros_(self.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return column_parallel_linear(x, self.weight, self.bias, self.sequence_parallel, True)

    # --- reference state-dict layout ---------------------------------------------------
    @staticmethod
    def _parent_prefix(prefix: str) -> str:
        # "layers.0.attn.wqkv." -> "layers.0.attn."
        parts = prefix.rstrip(".").split(".")
        return ".".join(parts[:-1]) + ("." if len(parts) > 1 else "")

    @staticmethod
    def _sd_hook(module, state_dict, prefix, local_metadata):
        pp = FusedColumnParallelLinear._parent_prefix(prefix)
        w = state_dict.pop(prefix + "weight")
        b = state_dict.pop(prefix + "bias", None)
        for i, name in enumerate(module.names):
            o, s = module.local_offsets[i], module.local[i]
            state_dict[f"{pp}{name}.weight"] = w[o:o + s]
            if b is not None:
                state_dict[f"{pp}{name}.bias"] = b[o:o + s]
        return state_dict

    def parent_load_hook(self, attr: str):
        """Load pre-hook to register on the PARENT module (``torch`` hands a child only the keys
        under its own prefix, so the merge of ``wq/wk/wv`` keys must happen one level up)."""
        def hook(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys, error_msgs):
            keys = [f"{prefix}{n}.weight" for n in self.names]
            if all(k in state_dict for k in keys):
                state_dict[f"{prefix}{attr}.weight"] = torch.cat([state_dict.pop(k) for k in keys], 0)
                bkeys = [f"{prefix}{n}.bias" for n in self.names]
                if all(k in state_dict for k in bkeys):
                    state_dict[f"{prefix}{attr}.bias"] = torch.cat([state_dict.pop(k) for k in bkeys], 0)
        return hook


def attach_fused(parent: nn.Module, attr: str, fused: "FusedColumnParallelLinear") -> None:
    """``parent.<attr> = fused`` plus the reference-layout load hook on ``parent``."""
    setattr(parent, attr, fused)
    parent._register_load_state_dict_pre_hook(fused.parent_load_hook(attr))


# ------------------------------------------------------------------------ embedding ----

class _VocabEmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, vocab_start: int, out_dtype):
        k = K(weight, out_dtype)
        out = k.embedding_fwd(ids, weight, vocab_start, out_dtype)
        ctx.save_for_backward(ids)
        ctx.meta = (weight.size(0), vocab_start, weight.dtype)
        return out

    @staticmethod
    def backward(ctx, dout):
        (flat,) = ctx.saved_tensors
        vl, st, wdt = ctx.meta
        d2 = dout.reshape(-1, dout.size(-1)).contiguous()
        dw = K(d2).embedding_bwd_sorted(d2, flat.contiguous(), vl, st)   # deterministic (no atomics)
        return None, dw.to(wdt), None, None


class ParallelVocabularyEmbedding(nn.Module):
    """Vocab-sharded embedding: masked local lookup + all-reduce(SUM) over the TP group."""

    def __init__(self, vocab_size: int, hdim: int, out_dtype: Optional[torch.dtype] = None,
                 sequence_parallel: bool = False, sizes: Optional[Sequence[int]] = None):
        super().__init__()
        self.vocab_size = vocab_size
        self.hdim = hdim
        self.out_dtype = out_dtype
        self.sequence_parallel = sequence_parallel
        if sizes is None:
            self.vocab_st_idx, self.vocab_ed_idx = self._get_vocab_range(vocab_size)
        else:   # explicit per-rank shard sizes (e.g. models.config.vocab_partition)
            n, r = _tp_size_rank()
            assert len(sizes) == n and sum(sizes) == vocab_size
            self.vocab_st_idx = sum(sizes[:r])
            self.vocab_ed_idx = self.vocab_st_idx + sizes[r]
        self.weight = nn.Parameter(torch.empty(self.vocab_ed_idx - self.vocab_st_idx, hdim))

    def _get_vocab_range(self, vocab_size: int) -> Tuple[int, int]:
        n, r = _tp_size_rank()
        assert n < vocab_size
        per = vocab_size // n
        st = per * r
        ed = vocab_size if r == n - 1 else st + per   # last rank takes the remainder
        return st, ed

    @torch.no_grad()
    def reset_parameters(self):
        w = _full_init_then_shard((self.vocab_size, self.hdim), "normal", self.weight.device,
                                  self.weight.dtype, 0, self.vocab_st_idx,
                                  self.vocab_ed_idx - self.vocab_st_idx)
        self.weight.copy_(w)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        assert x.ndim == 2, f"Input should be 2D tensor (B, L), but got {x.ndim}D tensor."
        dt = self.out_dtype or self.weight.dtype
        out = _VocabEmbeddingFn.apply(x.reshape(-1), self.weight, self.vocab_st_idx, dt)
        if self.sequence_parallel:
            return comm_ops.ScatterSeq.apply(out)
        return comm_ops.Reduce.apply(out).view(*x.shape, self.hdim)


# ---------------------------------------------------------------------------- norms ----

class RMSNorm(nn.Module):
    """Replicated RMSNorm (``layers.py:145-155``); output dtype = input dtype."""

    def __init__(self, hdim: int, eps: float = 1e-5, sequence_parallel: bool = False):
        super().__init__()
        self.eps = eps
        self.scale = nn.Parameter(torch.ones(hdim))
        self.scale.sequence_parallel_grad = sequence_parallel

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return Fn.rms_norm(x, self.scale, self.eps)


class LayerNorm(nn.Module):
    """Replicated LayerNorm (extension; the north star asks for it, GPT-2-style blocks)."""

    def __init__(self, hdim: int, eps: float = 1e-5, sequence_parallel: bool = False):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hdim))
        self.bias = nn.Parameter(torch.zeros(hdim))
        self.weight.sequence_parallel_grad = sequence_parallel
        self.bias.sequence_parallel_grad = sequence_parallel

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return Fn.layer_norm(x, self.weight, self.bias, self.eps)
